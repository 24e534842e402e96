# GEMM property test over the library's decomposition choices (hypothesis draws)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r34 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 300 --timeout-method thread -k "property" --hypothesis-show-statistics > gpurun_out/r34/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r34/pytest.log; exit $rc
