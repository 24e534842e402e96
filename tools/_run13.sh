cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r13 && export TMPDIR=/tmp
O=gpurun_out/r13
run() { local name=$1; shift; timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; };
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['steps'], d['config']['launch'], d['config']['lead'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; }
for rep in 1 2; do
run k20_graph_$rep --steps 20 --warmup 5
run k20_eager_$rep --steps 20 --warmup 5 --no-graph
run k20_eager_spin_$rep --steps 20 --warmup 5 --no-graph --lead spin
run k200_graph_$rep --steps 200
run k200_eager_$rep --steps 200 --no-graph
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp20 -o k20 -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/rp20.log 2>&1 || exit 1
python tools/trace_gaps.py $O/rp20 nf4_flat_kernel 20
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp20e -o k20e -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph > $O/rp20e.log 2>&1 || exit 1
python tools/trace_gaps.py $O/rp20e nf4_flat_kernel 20
tail -1 $O/rp20.log; tail -1 $O/rp20e.log
echo ALLDONE
