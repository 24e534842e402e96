# round 5 session 24: bench.py over a one-rank RCCL group (--dist-backend nccl at --gpus 1):
# the quant statistics go through sharding.scatter_quant_stats on RCCL, timed
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s24
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 1 --dist-backend nccl --steps 20 --warmup 5 > $O/bench_nccl_g1.json 2> $O/bench_nccl.err
python -c "import json;d=json.load(open('$O/bench_nccl_g1.json'));print('c2', d['config']['dist_backend'], d['config']['quant_state_scatter_ms'], d['roofline']['frac'], 'c5', d['c5']['quant_state_scatter_ms'], d['c5']['frac_of_peak'])"
timeout -k 10 300 python -u bench.py --gpus 1 --dist-backend nccl --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nccl_g1_c5.json 2>> $O/bench_nccl.err
python -c "import json;d=json.load(open('$O/bench_nccl_g1_c5.json'));print('c5 workload', d['config']['dist_backend'], d['config']['quant_state_scatter_ms'], d['roofline']['frac'], d['value'])"
