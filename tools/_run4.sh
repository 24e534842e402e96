# round-2 bench checks: default bench, C5 at N=1, 2-rank gloo rehearsal on one GPU, rocprof of the default bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=gpurun_out/r4
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err && tail -c 1500 $O/bench.json &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driverlike.json 2> $O/bench_driverlike.err &&
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err &&
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --workload c5 --no-cpu-baseline > $O/bench_g2_c5.json 2> $O/bench_g2_c5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o bench -- python -u bench.py --steps 200 --no-cpu-baseline > $O/bench_rocprof.log 2>&1 &&
python tools/rocprof_summary.py $O/rocprof nf4_flat_kernel $O/rocprof_bench_summary.json $O/rocprof_bench_kernel_stats.csv &&
echo ALLDONE
