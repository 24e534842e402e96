# round 5 session 14: the pruned final tree -- GPU suite, smoke, the driver's bench command,
# a longer dequant parity sweep
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s14
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1; cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print('bench',r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured']['launch_us'])"
timeout -k 10 300 python -u tools/fuzz_dequant.py --cases 60000 --seed 17 --seconds 240 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
