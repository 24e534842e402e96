#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Each GPU step has its own
# time limit; a crash/abort/timeout (rc not in {0,1}) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name: $*" >&2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -n 25 "gpurun_out/$name.log" >&2
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
    return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python __graft_entry__.py smoke
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
exit 0
