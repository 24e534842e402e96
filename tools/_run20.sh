# multi-rank launch paths on the 1-GPU box (both ranks on device 0, gloo): spawned ranks and torch.distributed.run
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r20 && export TMPDIR=/tmp
O=gpurun_out/r20
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_g2_c5.json 2> $O/bench_g2_c5.err || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_torchrun_g2.json 2> $O/bench_torchrun_g2.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_g1.json 2> $O/bench_g1.err || exit 1
echo ALLDONE
