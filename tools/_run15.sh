# headline refresh: default bench, driver-shaped K=20 runs, rocprof kernel-trace --stats of the K=20 command
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r15 && export TMPDIR=/tmp
O=gpurun_out/r15
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
for rep in 1 2 3; do
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20_$rep.json 2> $O/bench_k20_$rep.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o bench -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_rocprof.log 2>&1 || exit 1
python tools/rocprof_summary.py $O/rocprof nf4_flat_kernel $O/rocprof_summary.json $O/rocprof_kernel_stats.csv > /dev/null
python tools/trace_gaps.py $O/rocprof nf4_flat_kernel 20 > $O/rocprof_timed20.txt
for f in $O/bench.json $O/bench_k20_*.json; do python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['steps'], round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4))" $f; done
cat $O/rocprof_timed20.txt; python -c "import json;d=json.load(open('$O/rocprof_summary.json'));print({k:d[k] for k in list(d)[:12]})"
echo ALLDONE
