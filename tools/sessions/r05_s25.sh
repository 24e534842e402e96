# round 5 session 25: split-K hand-off soak on the final tree (the reducers now read the
# workspace error word: no false poisoning, bitwise-reproducible outputs, clean workspaces)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s25
mkdir -p $O
timeout -k 10 600 python -u tools/soak_gemm.py --iters 5000 --seconds 420 > $O/soak_gemm.jsonl 2> $O/soak.err
tail -2 $O/soak_gemm.jsonl
