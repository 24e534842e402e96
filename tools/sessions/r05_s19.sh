# round 5 session 19: host-proven scale-index shortcuts (one shift instead of three
# magic-number divisions) vs the product; parity of the variant on the GPU suite's dequant
# tests and a 20,000-case fuzz through it
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s19
mkdir -p $O
D=tools/_build
timeout -k 10 400 python -u tools/stream_probe.py --tag fastidx --steps 20,128 --rounds 15 --libs $D/libnf4dq_dqv_fastidx.so --kernels prod,dqv_fastidx,prod16,dqv_fastidx@16,mix:2:18:1 > $O/probe_fastidx.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_fastidx.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
NF4DQ_LIB_PATH=$D/libnf4dq_dqv_fastidx.so timeout -k 10 300 python -u tools/fuzz_dequant.py --cases 20000 --seed 29 --seconds 200 > $O/fuzz_fastidx.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_fastidx.jsonl
