# round 6 session 19: (1) the chunk kernel's fp32 half-chunk stores (padded rows, 57 us at
# 4096^2 in s18) with the default / sc1 policy instead of sc1 + nt; (2) the current tree: the
# whole GPU suite, smoke, the driver's bench command.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s19
mkdir -p $O
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 32 --dtype f32 --cases pad_4096,chunk_4090 \
    --libs tools/_build/libnf4dq_dqv_f32st0.so,tools/_build/libnf4dq_dqv_f32st16.so > $O/chunk_ab_f32st.jsonl 2> $O/chunk_ab_f32st.err
cat $O/chunk_ab_f32st.jsonl
bash tools/session.sh r06_s19 gputest smoke
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print('driver cmd', round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4), d['roofline'].get('frac_of_measured_copy'))"
