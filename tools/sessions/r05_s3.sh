# round 5 session 3: what makes nt-only stores lose in the product -- twins with the scale
# gathers and a decode-latency stand-in, under both store policies
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s3
mkdir -p $O
D=tools/_build
timeout -k 10 400 python -u tools/stream_probe.py --tag ms --steps 128 --rounds 7 --libs $D/libnf4dq_dqv_tbl.so,$D/libnf4dq_dqv_tbl_st2.so --kernels prod,dqv_tbl,dqv_tbl_st2,mix:2:18:1,mix:2:2:1,mixs:18:0,mixs:2:0,mixs:18:8,mixs:2:8,mixs:18:24,mixs:2:24 > $O/probe_ms.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_ms.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
