# round 5 session 29: the Llama-3-8B decode pass through the fused GEMM on the final tree
# (its split-K reducers now read the workspace error word): no regression vs round 4
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/session.sh r05_s29 gemmpass
