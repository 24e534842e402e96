set -e
mkdir -p gpurun_out
for L in head prod; do
  timeout -k 10 120 python tools/gemm_probe.py --lib $L --shape 14336,4096 --shape 4096,14336 --shape 4096,4096 --shape 28672,4096 --shape 6144,4096 --shape 1024,4096 --m 32 \
    --cfg 1,8,1,1,4 --cfg 1,4,1,1,4 --cfg 1,8,2,1,4 --cfg 1,8,1,2,4 --cfg 1,8,1,4,4 --cfg 1,4,1,4,2 --cfg 1,8,1,2,2 --cfg 1,4,2,4,1 --cfg 1,8,1,1,2 --cfg 1,8,1,2,1
  timeout -k 10 120 python tools/gemm_probe.py --lib $L --shape 4096,14336 --shape 1024,4096 --shape 4096,4096 --m 16 \
    --cfg 1,8,2,1,1 --cfg 1,8,1,2,2 --cfg 1,4,2,4,1 --cfg 1,8,1,1,4
done > gpurun_out/probe.jsonl 2>&1
