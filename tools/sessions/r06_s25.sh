# round 6 session 25: the final tree -- whole GPU suite, smoke, the driver's bench command,
# rocprofv3 kernel trace of the bench command, calibrated PMC traffic (bf16 / fp16) and the
# GEMM SQ counters, a dequant soak over every form, the API and GEMM fuzzers, and the
# distributed path on one GPU (RCCL one-rank group; two gloo ranks sharing the GPU).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s25
mkdir -p $O
bash tools/session.sh r06_s25 gputest smoke
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print('driver cmd', round(d['ms_per_step']*1e3,3), round(d['roofline']['frac'],4), d['roofline'].get('frac_of_measured_copy'))"
bash tools/session.sh r06_s25 rocprof pmc
timeout -k 10 300 python3 -u tools/soak_dequant.py --seconds 180 > $O/soak_dequant_180s.jsonl 2> $O/soak.err
tail -1 $O/soak_dequant_180s.jsonl
timeout -k 10 300 python3 -u tools/fuzz_api.py --rounds 1000 --seed 80 --seconds 200 > $O/fuzz_api.jsonl 2> $O/fuzz_api.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 300 python3 -u tools/fuzz_gemm.py --cases 2000 --seed 81 --seconds 200 > $O/fuzz_gemm.jsonl 2> $O/fuzz_gemm.err
tail -1 $O/fuzz_gemm.jsonl
timeout -k 10 300 python3 -u bench.py --gpus 1 --dist-backend nccl --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nccl_g1.json 2> $O/bench_nccl.err
python3 -c "import json; d=json.load(open('$O/bench_nccl_g1.json')); print('nccl g1', round(d['ms_per_step']*1e3,3), d['config']['dist_backend'])"
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_g2_gloo.json 2> $O/bench_g2.err
python3 -c "import json; d=json.load(open('$O/bench_g2_gloo.json')); print('gloo g2 on one GPU', d['n_gpus'], round(d['ms_per_step']*1e3,3))"
