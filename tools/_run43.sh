# Full GPU suite + smoke on the final tree, then A/B of the 16 B/lane direct-store tile
# shape (NF4DQ_CFG_X4_DIRECT, bench --flags 4) against the default, and the twins
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r43 && export TMPDIR=/tmp
O=gpurun_out/r43
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
for r in 1 2 3; do
  for f in 0 4 2; do
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --flags $f > $O/bench_f${f}_$r.json 2>> $O/bench.err || exit 1
    echo "flags=$f round=$r $(python -c "import json,sys; d=json.load(open('$O/bench_f${f}_$r.json')); print(d['ms_per_step']*1e3, d['roofline']['frac'])")"
  done
done
timeout -k 10 300 python -u tools/hbm_ceiling.py > $O/hbm_ceiling.jsonl 2> $O/hbm_ceiling.err || exit 1
cat $O/hbm_ceiling.jsonl
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json
