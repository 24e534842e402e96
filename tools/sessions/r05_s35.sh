# round 5 session 35: the chunk kernel (table decode) vs the flat kernel, with and without a
# workgroup barrier after the block tables (tools/_build/libnf4dq_dqv_csync.so); narrow-piece
# stores now default-policy
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s35
mkdir -p $O
timeout -k 10 400 python -u tools/chunk_ab.py --rounds 7 --libs tools/_build/libnf4dq_dqv_csync.so > $O/chunk_ab.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_ab.jsonl'))]"
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
