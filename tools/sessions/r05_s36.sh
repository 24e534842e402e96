# round 5 session 36: the chunk kernel's scale-gather placement (after the packed loads /
# before them / after the first load is back), A/B against the flat kernel
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s36
mkdir -p $O
timeout -k 10 400 python -u tools/chunk_ab.py --rounds 9 --cases flat_4096,chunk_4096,chunk_4080 --libs tools/_build/libnf4dq_dqv_cg1.so,tools/_build/libnf4dq_dqv_cg2.so > $O/chunk_gather.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_gather.jsonl'))]"
