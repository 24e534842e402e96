# round 5 session 21: the final kernel -- GPU suite, smoke, the driver's bench command,
# rocprofv3 kernel trace and PMC traffic (bf16, fp16), BASELINE configs
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s21
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1; cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print('bench',r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured']['launch_us'])"
bash tools/session.sh r05_s21 rocprof pmc configs > $O/session.log 2>&1 || { tail -20 $O/session.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/rocprof_bench_summary.json'));print(d['timed_region'])"
grep -h traffic_over $O/pmc_traffic.json $O/pmc_traffic_f16.json
