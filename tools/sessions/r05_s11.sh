# round 5 session 11: table decode without LDS code table / barrier, scale loads first,
# nt-only stores on top of them; the driver's bench command on this box
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s11
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in nolut nolut_st2 sf sf_st2; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag nolut --steps 20,128 --rounds 11 --libs ${L#,} --kernels $K,mix:2:18:1 > $O/probe_nolut.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_nolut.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print('bench',r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured']['launch_us'])"
