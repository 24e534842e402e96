#!/bin/bash
# One GPU-box session that refreshes every measurement committed under profiles/<round>/.
#   bash tools/measure_round.sh [round]      (default r01; outputs in gpurun_out/meas/)
# Each GPU step has its own time limit and the chain stops at the first failure.
set -e
ROUND=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
M=gpurun_out/meas
mkdir -p $M
# tool libraries are built here, not on the box (make -C tools)
test -f tools/_build/libpmccalib.so || { echo 'tools/_build/libpmccalib.so missing: run make -C tools first' >&2; exit 2; }
timeout -k 10 300 python -u bench.py > $M/bench.log 2> $M/bench.err && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $M/bench_k20.log 2>> $M/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof -o bench -- \
    python -u bench.py --steps 200 --no-cpu-baseline > $M/bench_rocprof.log 2>&1
python tools/rocprof_summary.py $M/rocprof nf4_flat_kernel $M/rocprof_bench_summary.json \
    $M/rocprof_bench_kernel_stats.csv --last 200 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $M/pmc -o fetch -- \
    python -u tools/pmc_probe.py > $M/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $M/pmc -o write -- \
    python -u tools/pmc_probe.py > $M/pmc_write.log 2>&1
python tools/pmc_traffic.py $M/pmc $M/pmc_traffic.json > $M/pmc_traffic.log 2>&1
timeout -k 10 600 python -u tools/bench_configs.py > $M/configs.jsonl 2> $M/configs.err
timeout -k 10 300 python -u tools/hbm_ceiling.py > $M/hbm_ceiling.jsonl 2> $M/hbm_ceiling.err
timeout -k 10 300 python -u tools/harness_reference_style.py > $M/harness_reference_style.jsonl 2> $M/harness.err
timeout -k 10 400 python -u tools/bench_gemm.py --ms 1,4,8,12,16,24,32 > $M/bench_gemm.jsonl 2> $M/bench_gemm.err
echo "measure_round $ROUND done" >&2
