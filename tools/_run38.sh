# MALL residency / next-weight prefetch probe for the decode GEMM
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r38 && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/mall_prefetch_probe.py --ms 1,32 --shape 14336,4096 > gpurun_out/r38/probe.jsonl 2> gpurun_out/r38/probe.err &&
timeout -k 10 300 python -u tools/mall_prefetch_probe.py --ms 1,32 --shape 4096,4096 --copies 48 >> gpurun_out/r38/probe.jsonl 2>> gpurun_out/r38/probe.err; rc=$?; cat gpurun_out/r38/probe.jsonl; tail -3 gpurun_out/r38/probe.err; exit $rc
