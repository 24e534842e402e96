# round 5 session 26: bitsandbytes-semantics mode (6 % behind the reference mode in
# bench_configs): its nested-code table load, an early one-instruction load, and an
# ablation without the table, next to the reference-mode product
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s26
mkdir -p $O
D=tools/_build
timeout -k 10 400 python -u tools/stream_probe.py --tag bnb --steps 20,128 --rounds 11 --libs $D/libnf4dq_dqv_bnbc1.so,$D/libnf4dq_dqv_bnbc2.so --kernels prod,bnb,dqv_bnbc1@bnb,dqv_bnbc2@bnb > $O/probe_bnb.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_bnb.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
