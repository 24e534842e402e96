# round 5 session 44: bitsandbytes mode with the early code-book load -- parity (every bnb
# test of the GPU suite) and its config line
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s44
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "bnb or bitsandbytes or large" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_bnb.txt 2>&1
tail -2 $O/pytest_bnb.txt
timeout -k 10 300 python -u tools/bench_configs.py --configs bnb,c4 > $O/configs_bnb.jsonl 2> $O/err.txt
python -c "import json;[print(d['config'],d.get('out_dtype',''),round(d['us_per_launch'],3),round(d['frac'],4),d['verified']) for d in map(json.loads,open('$O/configs_bnb.jsonl'))]"
