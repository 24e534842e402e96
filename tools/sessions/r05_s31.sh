# round 5 session 31: capped (looping) grids vs the default one-tile grid on the final
# kernel, at the headline and the large shapes (bf16, weights streamed from HBM)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s31
mkdir -p $O
timeout -k 10 600 python -u tools/dq_ab.py --shapes 4096x4096,8192x8192,14336x4096,16384x8192 --bpcu 0,1,2,4,8 --flags 0 --rounds 7 --steps 64 > $O/capped_grid.jsonl 2> $O/err.txt
cat $O/capped_grid.jsonl | python -c "import sys,json;[print(d['m'],d['n'],d['blocks_per_cu'],d['us_median'],d['frac']) for d in map(json.loads,sys.stdin)]"
