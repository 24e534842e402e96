set -e
mkdir -p gpurun_out
C="--cfg 2,8,2,1,4 --cfg 2,8,2,1,1"
for L in prod dbg1 dbg5 dbg7; do
  timeout -k 10 120 python tools/gemm_probe.py --lib $L --shape 14336,4096 --shape 4096,4096 --m 1 $C
done > gpurun_out/probe.jsonl 2>&1
