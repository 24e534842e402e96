# round 5 session 45: the general chunk kernel's dword loads under the default cache policy
# (tools/_build/libnf4dq_dqv_cld0.so) vs nt (product), padded rows and n = 4095
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s45
mkdir -p $O
timeout -k 10 400 python -u tools/chunk_ab.py --rounds 9 --cases chunk_4080,pad_4096,chunk_4095 --libs tools/_build/libnf4dq_dqv_cld0.so > $O/chunk_cld.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_cld.jsonl'))]"
