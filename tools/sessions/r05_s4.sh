# round 5 session 4: ablation -- the flat kernel without its scale gathers
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s4
mkdir -p $O
D=tools/_build
timeout -k 10 400 python -u tools/stream_probe.py --tag abl --steps 128 --rounds 7 --libs $D/libnf4dq_dqv_tbl.so,$D/libnf4dq_dqv_tbl_noscale.so,$D/libnf4dq_dqv_noscale.so --kernels prod,dqv_noscale,dqv_tbl,dqv_tbl_noscale,mix:2:18:1 > $O/probe_abl.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_abl.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
