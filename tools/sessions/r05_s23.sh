# round 5 session 23: launch shape on top of the final kernel (one-tile waves outside the
# loop): 2 / 8 dwords per lane, 2 / 8 / 16 waves per workgroup
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s23
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in u2 u8 wg2 wg8 wg16; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag shape --steps 20,128 --rounds 11 --libs ${L#,} --kernels $K > $O/probe_shape.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_shape.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
