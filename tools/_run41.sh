# dequantize_nf4_many into caller-owned outputs + the API tests around it
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r41 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_concurrency.py -q --timeout 300 --timeout-method thread > gpurun_out/r41/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r41/pytest.log; exit $rc
