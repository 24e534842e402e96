# Absmax bytes a tile ahead (NF4DQ_CFG_A1_AHEAD, bench --flags 8): parity, then A/B
# against the default at 4096^2 and 8192^2 (per-set absmax, bench.py's sets), then the GPU suite
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r45 && export TMPDIR=/tmp
O=gpurun_out/r45
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ahead or launch_configs" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for r in 1 2 3; do
  for sz in 4096 8192; do
    for f in 0 8; do
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --m $sz --n $sz --flags $f > $O/bench_${sz}_f${f}_$r.json 2>> $O/bench.err || exit 1
      echo "size=$sz flags=$f round=$r $(python -c "import json; d=json.load(open('$O/bench_${sz}_f${f}_$r.json')); print(round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4))")"
    done
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
