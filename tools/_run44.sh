# C5 single-launch anomaly: 8192^2 through bench.py (eager, >= 1 GiB sets), bench_configs c5
# (graph replay over 8 sets with per-set absmax), and the absmax-placement probe
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r44 && export TMPDIR=/tmp
O=gpurun_out/r44
timeout -k 10 180 python -u bench.py --no-cpu-baseline --m 8192 --n 8192 > $O/bench_8192.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench_8192.json')); print('bench 8192^2', d['ms_per_step']*1e3, d['roofline']['frac'], d['config']['buffer_sets'])"
timeout -k 10 300 python -u tools/bench_configs.py --configs c5 > $O/configs_c5.jsonl 2> $O/configs.err || exit 1
cat $O/configs_c5.jsonl
timeout -k 10 300 python -u tools/value_sensitivity.py > $O/value_sensitivity.jsonl 2> $O/vs.err || exit 1
cat $O/value_sensitivity.jsonl
