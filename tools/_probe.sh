set -e
mkdir -p gpurun_out
for M in 16 32; do
for L in prod dbg1 dbg2 dbg5 dbg6; do
  timeout -k 10 120 python tools/gemm_probe.py --lib $L --shape 14336,4096 --m $M --cfg 2,4,2,4,4 --cfg 2,8,2,2,4 --cfg 2,8,2,4,4 | sed "s/^/{\"lib\":\"$L\",\"M\":$M,\"r\":/; s/$/}/"
done
done > gpurun_out/probe.jsonl 2>&1
