# register-resident GEMM with grouped reductions (one barrier pair per RG strips): parity, probe, sweep
# (the grouped-reduction variant it measured was an uncommitted build, not kept -- see DESIGN §4b and commit 96ff5c7; re-running this measures the product kernel)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r36 && export TMPDIR=/tmp
O=gpurun_out/r36
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1; rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/xr_probe.py > $O/xr_probe.jsonl 2> $O/xr_probe.err || exit 1
timeout -k 10 600 python -u tools/sweep_gemm.py --ms 1,16,24,32 --kernels 5 --shapes "14336,4096;4096,4096;4096,14336;6144,4096;28672,4096" > $O/sweep.jsonl 2> $O/sweep.err || exit 1
echo ALLDONE
