# round 5 session 27: bitsandbytes mode with a sleep between the packed loads and the
# absmax gathers (the reference mode's index arithmetic sits there)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s27
mkdir -p $O
D=tools/_build
timeout -k 10 400 python -u tools/stream_probe.py --tag bnbgd --steps 20,128 --rounds 11 --libs $D/libnf4dq_dqv_bgd1.so,$D/libnf4dq_dqv_bgd2.so,$D/libnf4dq_dqv_bgd4.so --kernels prod,bnb,dqv_bgd1@bnb,dqv_bgd2@bnb,dqv_bgd4@bnb > $O/probe_bnbgd.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_bnbgd.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
