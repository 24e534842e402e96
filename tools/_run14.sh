cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r14 && export TMPDIR=/tmp
O=gpurun_out/r14
run() { local name=$1; shift; timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; };
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['steps'], d['config']['launch'], d['config']['lead'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; }
for rep in 1 2 3; do
run k20_graph_$rep --steps 20 --warmup 5
run k20_eager_$rep --steps 20 --warmup 5 --no-graph
run k20_eager_steps_$rep --steps 20 --warmup 5 --no-graph --lead steps
run k200_graph_$rep --steps 200
run k200_eager_steps_$rep --steps 200 --no-graph --lead steps
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp20s -o k20s -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph --lead steps > $O/rp20s.log 2>&1 || exit 1
python tools/trace_gaps.py $O/rp20s nf4_flat_kernel 28
tail -1 $O/rp20s.log
echo ALLDONE
