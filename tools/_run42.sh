# GEMM property tests (single weight and grouped) with hypothesis statistics
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r42 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 300 --timeout-method thread -k "property" --hypothesis-show-statistics > gpurun_out/r42/pytest.log 2>&1; rc=$?; tail -25 gpurun_out/r42/pytest.log; exit $rc
