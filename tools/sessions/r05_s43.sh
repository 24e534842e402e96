# round 5 session 43: bitsandbytes mode with each thread's code-book word loaded ahead of
# the tile's loads (tools/_build/libnf4dq_dqv_bnbe.so) against the product's bnb and ref modes
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s43
mkdir -p $O
timeout -k 10 400 python -u tools/stream_probe.py --kernels prod,bnb,dqv_bnbe@bnb --libs tools/_build/libnf4dq_dqv_bnbe.so --steps 20,128 --rounds 11 --tag bnbe > $O/probe_bnbe.jsonl 2> $O/err.txt
python -c "
import json
for l in open('$O/probe_bnbe.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
