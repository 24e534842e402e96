# round 5 session 18: the one-tile fast path as the product -- GPU suite, smoke, driver's
# bench command, A/B against the loop form (K = 20 and 128, 15 rounds), 20,000-case fuzz
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s18
mkdir -p $O
D=tools/_build
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1; cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print('bench',r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured']['launch_us'])"
timeout -k 10 400 python -u tools/stream_probe.py --tag fast --steps 20,128 --rounds 15 --libs $D/libnf4dq_dqv_loop1.so --kernels prod,dqv_loop1,prod16,dqv_loop1@16,mix:2:18:1 > $O/probe_fast.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_fast.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
timeout -k 10 300 python -u tools/fuzz_dequant.py --cases 20000 --seed 23 --seconds 200 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
