# bitsandbytes-semantics flat kernel with the code staged in LDS: full GPU suite, then the configs bench (bnb row)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r31 && export TMPDIR=/tmp
O=gpurun_out/r31
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit 1
grep bnb $O/configs.jsonl
