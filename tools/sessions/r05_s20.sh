# round 5 session 20: a sleep between a tile's packed loads and its scale gathers
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s20
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in gd1 gd2 gd4 gd8 gd16; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag gdelay --steps 20,128 --rounds 11 --libs ${L#,} --kernels $K,mix:2:18:1 > $O/probe_gdelay.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_gdelay.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
