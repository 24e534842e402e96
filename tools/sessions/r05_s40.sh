# round 5 session 40: parity sweep over the chunk kernels -- drop-in calls and C-ABI calls
# with the packed weight / output off their alignment (sentinels both sides)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s40
mkdir -p $O
timeout -k 10 560 python -u tools/fuzz_dequant.py --cases 60000 --seed 53 --seconds 480 --abi-rate 0.4 > $O/fuzz_chunks.jsonl 2> $O/err.txt
tail -1 $O/fuzz_chunks.jsonl
