# full GEMM parity suite with the register-resident default for the widest M > 16 launches, then the Llama-3-8B decode pass
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r19 && export TMPDIR=/tmp
O=gpurun_out/r19
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_strided.py -q -x --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1; rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_gemm.py --ms 1,8,16,24,32 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err || exit 1
echo ALLDONE
