# round 6 session 32: the final tree, with the decode GEMV as the M = 1 choice --
# whole GPU suite, smoke, the driver's bench command.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s32
mkdir -p $O
bash tools/session.sh r06_s32 gputest smoke
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print('driver cmd', round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4), d['roofline'].get('frac_of_measured_copy'))"
