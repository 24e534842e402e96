# round 6 session 8: (1) the headline through bench.py's own timing on the current library
# and the previous one (tools/_build/libnf4dq_prev.so; identical flat-kernel ISA), interleaved --
# chunk_ab.py read the current library's flat kernel 3-5 % slow; (2) the final tree: GPU suite,
# smoke, the driver's bench command, rocprofv3 kernel trace of the bench command, PMC traffic.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s8
mkdir -p $O
for i in 1 2; do
    for lib in prod prev; do
        if [ $lib = prev ]; then export NF4DQ_LIB_PATH=tools/_build/libnf4dq_prev.so; else unset NF4DQ_LIB_PATH; fi
        timeout -k 10 200 python3 -u bench.py --steps 128 --warmup 5 --no-cpu-baseline --no-c5 --no-ceiling > $O/bench_ab_${lib}_$i.json 2>> $O/bench_ab.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4))" $O/bench_ab_${lib}_$i.json $lib
    done
done
unset NF4DQ_LIB_PATH
bash tools/session.sh r06_s8 gputest smoke bench20 rocprof pmc
# the driver's exact command (CPU baseline included)
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print('driver cmd', round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4), d['roofline'].get('frac_of_measured_copy'))"
