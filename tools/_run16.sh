cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r16 && export TMPDIR=/tmp
O=gpurun_out/r16
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/harness_reference_style.py > $O/harness.jsonl 2> $O/harness.err || exit 1
cat $O/harness.jsonl
echo ALLDONE
