# Scratch A/B probe (tools only): the last decode-GEMM comparison run on the GPU box,
# head library (tools/_build/libnf4dq_head.so, built from HEAD) vs the working tree
# (tools/_build/libnf4dq_prod.so).  Edit and run as: gpurun -- 'bash tools/_probe.sh'
set -e
mkdir -p gpurun_out
for L in head prod; do
  timeout -k 10 200 python tools/bench_gemm.py --ms 16,24,32 --no-bf16 --no-composite --lib $L
done > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
