# round 5 session 5: table decode with a sleep between a tile's loads and its stores
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s5
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in tbl tbl_d2 tbl_d4 tbl_d8 tbl_d16 tbl_d32 tbl_st2_d8 tbl_st2_d16; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag delay --steps 20,128 --rounds 7 --libs ${L#,} --kernels $K,mix:2:18:1 > $O/probe_delay.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_delay.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
