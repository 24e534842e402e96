# bench A/B on one box: untimed lead launches ahead of the start event (8 / 16 / 24) at the driver's K = 20, 3 reps each
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r21 && export TMPDIR=/tmp
O=gpurun_out/r21
for rep in 1 2 3; do
  for ln in 8 16 24; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --lead-n $ln > $O/k20_lead${ln}_$rep.json 2>> $O/err.log || exit 1
  done
done
for f in $O/k20_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['ms_per_step']*1e3, round(d['roofline']['frac'],4))"; done
