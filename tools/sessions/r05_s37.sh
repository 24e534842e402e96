# round 5 session 37: the chunk kernel's dense form (n % 8 == 0, dense rows: the flat stream
# with row-following scale blocks) -- parity, then A/B against the flat kernel
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s37
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
timeout -k 10 400 python -u tools/chunk_ab.py --rounds 9 > $O/chunk_ab.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_ab.jsonl'))]"
