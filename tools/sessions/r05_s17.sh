# round 5 session 17: one-tile waves without the pipelined loop (next-tile loads + dropped
# store burst), at 4096^2 (one tile per wave) and 8192^2 (several)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s17
mkdir -p $O
D=tools/_build
L="$D/libnf4dq_dqv_single.so,$D/libnf4dq_dqv_single_st2.so"
timeout -k 10 400 python -u tools/stream_probe.py --tag single --steps 20,128 --rounds 11 --libs $L --kernels prod,dqv_single,dqv_single_st2,prod16,dqv_single@16,mix:2:18:1 > $O/probe_single.jsonl 2> $O/probe.err
timeout -k 10 400 python -u tools/stream_probe.py --tag single8k --shape 8192x8192 --steps 32 --rounds 5 --libs $L --kernels prod,dqv_single >> $O/probe_single.jsonl 2>> $O/probe.err
python -c "
import json
for l in open('$O/probe_single.jsonl'):
    d=json.loads(l); print(d['m'], d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
