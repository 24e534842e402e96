cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r7 && export TMPDIR=/tmp
O=gpurun_out/r7
run() { local name=$1; shift; timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || exit 1;
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['config']['buffer_sets'], d['steps'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; }
for rep in 1 2; do
run k20_replay_$rep --steps 20 --warmup 5 --lead replay
run k20_spin_$rep --steps 20 --warmup 5 --lead spin
run k20_none_$rep --steps 20 --warmup 5 --lead none
run k200_replay_$rep --steps 200 --lead replay
run k200_none_$rep --steps 200 --lead none
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp20 -o k20 -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --lead none > $O/rp20.log 2>&1
echo ALLDONE
