set -e
mkdir -p gpurun_out
for M in 1 4 8 16; do
  timeout -k 10 120 python tools/gemm_probe.py --lib prod --shape 4096,14336 --m $M \
    --cfg 3,8,2,7,2 --cfg 3,8,2,7,4 --cfg 3,4,2,7,2 --cfg 3,8,2,14,4 --cfg 3,4,2,4,4 --cfg 3,8,2,2,4 --cfg 3,8,4,7,4 --cfg 3,4,2,14,2 \
    --cfg 2,8,2,1,1 --cfg 2,8,2,2,2 --cfg 2,8,2,4,4 --cfg 1,8,1,2,2
done > gpurun_out/probe.jsonl 2>&1
for M in 1 8; do
  timeout -k 10 120 python tools/gemm_probe.py --lib prod --shape 4096,4096 --shape 28672,4096 --shape 1024,4096 --m $M \
    --cfg 3,8,2,1,1 --cfg 3,8,2,2,2 --cfg 3,8,2,2,4 --cfg 3,4,2,2,2
done >> gpurun_out/probe.jsonl 2>&1
