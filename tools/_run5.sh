# A/B of bench.py buffer-set / flush settings on one box + flat-kernel stamps
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5 && export TMPDIR=/tmp
O=gpurun_out/r5
run() { local name=$1; shift; timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || exit 1;
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', d['config']['buffer_sets'], d['steps'], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))"; }
for rep in 1 2; do
run s16_k20_noflush_$rep --sets 16 --steps 20 --warmup 5 --no-flush
run s16_k20_flush_$rep --sets 16 --steps 20 --warmup 5
run s26_k20_noflush_$rep --steps 20 --warmup 5 --no-flush
run s26_k200_noflush_$rep --steps 200 --no-flush
run s26_k200_flush_$rep --steps 200
run s16_k200_noflush_$rep --sets 16 --steps 200 --no-flush
run s200_k200_noflush_$rep --sets 200 --steps 200 --no-flush
run s8_k200_noflush_$rep --sets 8 --steps 200 --no-flush
done
timeout -k 10 120 python -u tools/flat_stamps.py > $O/stamps.json 2> $O/stamps.err && cat $O/stamps.json
echo ALLDONE
