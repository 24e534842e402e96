# round 5 session 50: 10-minute soak of every dequant kernel form on the final tree, outputs
# checked bit for bit against the C oracle throughout
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s50
mkdir -p $O
timeout -k 10 720 python -u tools/soak_dequant.py --seconds 600 --check-every 64 > $O/soak_dequant.jsonl 2> $O/err.txt
tail -1 $O/soak_dequant.jsonl
