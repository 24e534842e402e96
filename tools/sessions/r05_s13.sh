# round 5 session 13: does synchronising a workgroup's waves help? (the table decode without
# its start barrier measured 8 % slower): a barrier before each tile's stores, 2-16 waves
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s13
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in sync sync_wg8 sync_wg16 wg2 sync_u2 nolut; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag sync --steps 20,128 --rounds 9 --libs ${L#,} --kernels $K,mix:2:18:1 > $O/probe_sync.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_sync.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
