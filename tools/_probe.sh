# Scratch A/B probe (tools only): the last decode-GEMM comparison run on the GPU box,
# head library (tools/_build/libnf4dq_head.so, built from HEAD) vs the working tree
# (tools/_build/libnf4dq_prod.so).  Edit and run as: gpurun -- 'bash tools/_probe.sh'
set -e
mkdir -p gpurun_out
for L in head prod; do
  timeout -k 10 120 python tools/gemm_probe.py --lib $L --shape 14336,4096 --shape 4096,14336 --shape 4096,4096 \
    --shape 28672,4096 --shape 6144,4096 --shape 1024,4096 --m 32 \
    --cfg 1,8,1,1,4 --cfg 1,4,1,1,4 --cfg 1,8,1,4,4 --cfg 1,4,1,4,2 --cfg 1,8,1,2,2
done > gpurun_out/probe.jsonl 2>&1
