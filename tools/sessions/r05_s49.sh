# round 5 session 49: the final tree's rocprof kernel trace of the bench command (K = 200) and
# the PMC traffic passes (bf16 + fp16), then the driver's command three times on this box
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/session.sh r05_s49 rocprof pmc
bash tools/sessions/r05_box.sh 6
