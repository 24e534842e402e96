# bitsandbytes-semantics path under the weight's device guard; checkpoint loader; GEMM property test with statistics
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r37 && export TMPDIR=/tmp
O=gpurun_out/r37
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -k "bnb or checkpoint or property" --hypothesis-show-statistics > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
