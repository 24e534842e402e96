# round 5 session 32: the general (rows) kernel's speed at a BASELINE-sized matrix with
# n % 64 != 0, beside the flat kernel's c4 lines on the same box
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s32
mkdir -p $O
timeout -k 10 400 python -u tools/bench_configs.py --configs rows,c4 --reps 5 > $O/configs_rows.jsonl 2> $O/err.txt
python -c "import sys,json;[print(d['config'],d.get('out_dtype'),round(d['us_per_launch'],2),round(d['frac'],4)) for d in map(json.loads,open('$O/configs_rows.jsonl'))]"
