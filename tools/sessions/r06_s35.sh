# round 6 session 35: the rebuilt final library (comment-only source changes since s32) --
# the whole GPU suite, smoke and the driver's bench command once more.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s35
mkdir -p $O
bash tools/session.sh r06_s35 gputest smoke
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print('driver cmd', round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4), d['roofline'].get('frac_of_measured_copy'))"
