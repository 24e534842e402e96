cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_k20a.json 2> $O/bench_k20a.err &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_k20b.json 2> $O/bench_k20b.err &&
for f in bench bench_k20a bench_k20b; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['config']['buffer_sets'], d['steps'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; done &&
timeout -k 10 120 python -u tools/flat_stamps.py > $O/stamps.json 2> $O/stamps.err && cat $O/stamps.json &&
timeout -k 10 120 python -u tools/flat_stamps.py --shape 8192,8192 > $O/stamps8k.json 2> $O/stamps8k.err && cat $O/stamps8k.json &&
timeout -k 10 300 python -u tools/harness_reference_style.py --iterations 300 > $O/harness.jsonl 2> $O/harness.err && tail -1 $O/harness.jsonl &&
timeout -k 10 300 python -u tools/bench_prefill.py > $O/prefill.jsonl 2> $O/prefill.err && cat $O/prefill.jsonl &&
echo ALLDONE
