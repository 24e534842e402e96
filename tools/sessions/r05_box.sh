# round 5, per-box headline sample: the driver's exact command three times (three fresh
# processes) on whatever box this call landed on, plus the twin and K = 128 for the box
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_box_$1
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20_$r.json 2>> $O/bench.err
  python -c "import json;d=json.load(open('$O/bench_k20_$r.json'));r=d['roofline'];print(json.dumps({'run':$r,'us':r['launch_us'],'frac':r['frac'],'min':r['launch_us_min'],'max':r['launch_us_max'],'twin':r['ceiling_measured']['launch_us'],'c5':d['c5']['frac_of_peak'],'cpu':d['cpu_baseline']['value']}))" | tee -a $O/summary.jsonl
done
timeout -k 10 300 python -u tools/stream_probe.py --tag box --steps 20,128 --rounds 7 --kernels prod,prod16,mix:2:18:1,empty > $O/probe.jsonl 2> $O/probe.err
cat $O/probe.jsonl
