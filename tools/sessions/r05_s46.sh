# round 5 session 46: final tree -- GPU suite, smoke, parity sweeps (drop-in + misaligned
# C-ABI calls, API entries), the driver's bench command
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s46
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gputest.log.txt 2>&1
tail -2 $O/gputest.log.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 400 python -u tools/fuzz_dequant.py --cases 40000 --seed 59 --seconds 300 --abi-rate 0.4 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
timeout -k 10 300 python -u tools/fuzz_api.py --rounds 800 --seed 61 --seconds 200 > $O/fuzz_api.jsonl 2>> $O/fuzz.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));print(round(d['ms_per_step']*1e3,3),round(d['roofline']['frac'],4))"
