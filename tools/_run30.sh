# GEMM parity suite incl. the register-resident library choice at single-weight shapes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r30 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 120 --timeout-method thread > gpurun_out/r30/pytest_gemm.log 2>&1; rc=$?; tail -3 gpurun_out/r30/pytest_gemm.log; exit $rc
