# concurrent-stream determinism and hipGraph capture of the product API
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r40 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrency.py -v --timeout 300 --timeout-method thread > gpurun_out/r40/pytest.log 2>&1; rc=$?; tail -30 gpurun_out/r40/pytest.log; exit $rc
