# round 5 session 16: does the lead ahead of the timed regions matter? bench.py at the driver's
# K = 20 with 16 / 48 lead launches and a 30 / 10 us-per-launch spin, interleaved x3
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s16
mkdir -p $O
for rep in 1 2 3; do
  for cfg in "16 30" "48 30" "16 10" "48 10"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c5 --lead-n $1 --spin-us-per-launch $2 > $O/b.json 2>> $O/bench.err
    python -c "import json,sys;d=json.load(open('$O/b.json'));r=d['roofline'];print(json.dumps({'lead':$1,'spin':$2,'rep':$rep,'us':r['launch_us'],'frac':r['frac'],'min':r['launch_us_min'],'max':r['launch_us_max'],'twin':r['ceiling_measured']['launch_us']}))" >> $O/lead_ab.jsonl
  done
done
cat $O/lead_ab.jsonl
