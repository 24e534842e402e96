# guard-band (red-zone) checks of every C-ABI entry point
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r39 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_redzones.py -v --timeout 300 --timeout-method thread > gpurun_out/r39/pytest.log 2>&1; rc=$?; tail -25 gpurun_out/r39/pytest.log; exit $rc
