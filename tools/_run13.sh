cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r13 && export TMPDIR=/tmp
O=gpurun_out/r13
run() { local name=$1; shift; timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; };
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['steps'], d['config']['events'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; }
for rep in 1 2 3; do
run k20_stream_$rep --steps 20 --warmup 5
run k20_graph_$rep --steps 20 --warmup 5 --events graph
run k200_stream_$rep --steps 200
run k200_graph_$rep --steps 200 --events graph
done
echo ALLDONE
