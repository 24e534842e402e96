set -e
mkdir -p gpurun_out
for M in 16 32; do
  timeout -k 10 120 python tools/gemm_probe.py --lib prod --shape 14336,4096 --shape 4096,14336 --shape 4096,4096 --m $M \
    --cfg 1,8,2,1,1 --cfg 1,8,2,1,2 --cfg 1,8,2,1,4 --cfg 1,8,1,1,4 --cfg 1,4,2,1,4 --cfg 1,8,2,2,4 --cfg 1,8,2,2,2 --cfg 1,8,1,4,4
done > gpurun_out/probe.jsonl 2>&1
