# headline variance on one box: the driver's command shape (K = 20, W = 5) five times, then the default K = 200 once
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r29 && export TMPDIR=/tmp
O=gpurun_out/r29/$(date +%s)
mkdir -p $O
for rep in 1 2 3 4 5; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/k20_$rep.json 2>> $O/err.log || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/k200.json 2>> $O/err.log || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4))"; done
