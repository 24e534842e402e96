# round 5 session 34: the chunk kernel vs the flat kernel on the same stream (A/B), and
# the rocprof kernel durations of the same cases
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s34
mkdir -p $O
timeout -k 10 300 python -u tools/chunk_ab.py --rounds 7 > $O/chunk_ab.jsonl 2> $O/err.txt
cat $O/chunk_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/chunk_ab.py --rounds 2 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-8 $O/kernel_stats.csv
