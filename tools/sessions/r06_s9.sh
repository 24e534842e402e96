# round 6 session 9: the final tree under long randomized and repeated checks -- the dequant
# soak (every kernel form, the staged n % 8 != 0 form included), API and GEMM fuzzers, and the
# distributed path on one GPU (RCCL one-rank group; 2 gloo ranks sharing the GPU).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s9
mkdir -p $O
timeout -k 10 420 python3 -u tools/soak_dequant.py --seconds 300 > $O/soak_dequant_300s.jsonl 2> $O/soak.err
tail -1 $O/soak_dequant_300s.jsonl
timeout -k 10 400 python3 -u tools/fuzz_api.py --rounds 1500 --seed 68 --seconds 300 > $O/fuzz_api.jsonl 2> $O/fuzz_api.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 400 python3 -u tools/fuzz_gemm.py --cases 3000 --seed 69 --seconds 300 > $O/fuzz_gemm.jsonl 2> $O/fuzz_gemm.err
tail -1 $O/fuzz_gemm.jsonl
timeout -k 10 300 python3 -u bench.py --gpus 1 --dist-backend nccl --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nccl_g1.json 2> $O/bench_nccl.err
python3 -c "import json; d=json.load(open('$O/bench_nccl_g1.json')); print('nccl g1', round(d['ms_per_step']*1e3,3), d['config']['dist_backend'], d['config']['quant_state_scatter_ms'])"
timeout -k 10 400 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_g2_gloo.json 2> $O/bench_g2.err
python3 -c "import json; d=json.load(open('$O/bench_g2_gloo.json')); print('gloo g2 on one GPU', d['n_gpus'], round(d['ms_per_step']*1e3,3), [round(r['ms_per_step']*1e3,3) for r in d['per_rank']])"
