# round 5 session 28: the final tree once more -- GPU suite, smoke, the driver's bench
# command, API and GEMM parity sweeps
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s28
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1; cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print('bench',r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured']['launch_us'])"
timeout -k 10 300 python -u tools/fuzz_api.py --rounds 800 --seed 31 --seconds 200 > $O/fuzz_api.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 400 python -u tools/fuzz_gemm.py --cases 6000 --seed 37 --seconds 300 --boundary-rate 0.2 > $O/fuzz_gemm.jsonl 2>> $O/fuzz.err
tail -1 $O/fuzz_gemm.jsonl
