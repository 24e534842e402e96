# round 5 session 33: the chunk kernel (shapes the flat kernel does not take) --
# parity through every load / store form, then its speed at 4096x4080
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s33
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_parity.py tests/test_gpu_strided.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -3 $O/pytest.txt
timeout -k 10 400 python -u tools/bench_configs.py --configs rows,c4 --reps 5 > $O/configs_rows.jsonl 2> $O/err.txt
python -c "import sys,json;[print(d['config'],d.get('out_dtype'),round(d['us_per_launch'],2),round(d['frac'],4)) for d in map(json.loads,open('$O/configs_rows.jsonl'))]"
