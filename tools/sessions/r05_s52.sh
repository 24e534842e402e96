# round 5 session 52: the product against its memory-system twin at 8192^2 and 16384x8192
# (HBM-streamed, bench.py's method): is there decode cost left at the large sizes?
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s52
mkdir -p $O
timeout -k 10 400 python -u tools/stream_probe.py --shape 8192x8192 --tag big --steps 32 --rounds 7 --kernels prod,prod16,mix:2:18:1,rd:2:1,wr:18:1 > $O/probe_8192.jsonl 2> $O/err.txt
python -c "
import json
for l in open('$O/probe_8192.jsonl'):
    d=json.loads(l); print(d['kernel'], d['m'], d['n'], d['steps'], d['us_median'], d['dequant_frac_at_this_time'])
"
