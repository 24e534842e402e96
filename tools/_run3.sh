cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 900 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu3.log; exit 1; }
tail -25 gpurun_out/pytest_gpu3.log
timeout -k 10 300 python -u tools/harness_reference_style.py --iterations 300 > gpurun_out/harness3.log 2>&1 ; tail -5 gpurun_out/harness3.log
