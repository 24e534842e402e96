# register-resident GEMM with two 256-deep chunks per wave (KPW 4): parity, correctness probe, M = 24/32 sweep, decode pass
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r32 && export TMPDIR=/tmp
O=gpurun_out/r32
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 120 --timeout-method thread -k "register_resident" > $O/pytest_xr.log 2>&1; rc=$?; tail -3 $O/pytest_xr.log; [ $rc -eq 0 ] || { grep -E "^E  .*cfg|FAILED" $O/pytest_xr.log | head -40; exit $rc; }
timeout -k 10 240 python -u tools/xr_probe.py > $O/xr_probe.jsonl 2> $O/xr_probe.err || exit 1
timeout -k 10 600 python -u tools/sweep_gemm.py --ms 24,32 --kernels 5 --shapes "14336,4096;4096,4096;4096,14336;6144,4096;28672,4096" > $O/sweep.jsonl 2> $O/sweep.err || exit 1
timeout -k 10 400 python -u tools/bench_gemm.py --ms 1,16,24,32 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err || exit 1
echo ALLDONE
