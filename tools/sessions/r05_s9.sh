# round 5 session 9: rocprofv3 kernel trace of the bench (K = 200), PMC traffic in bf16 and
# fp16, the driver's bench command
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/session.sh r05_s9 rocprof pmc bench20
