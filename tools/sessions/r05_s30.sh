# round 5 session 30: long parity sweeps on the final tree (drop-in dequant, multi-weight /
# single-quant / grouped entries, fused GEMM with boundary shapes)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s30
mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_dequant.py --cases 150000 --seed 41 --seconds 420 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
timeout -k 10 500 python -u tools/fuzz_api.py --rounds 3000 --seed 43 --seconds 300 > $O/fuzz_api.jsonl 2>> $O/fuzz.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 700 python -u tools/fuzz_gemm.py --cases 20000 --seed 47 --seconds 540 --boundary-rate 0.15 > $O/fuzz_gemm.jsonl 2>> $O/fuzz.err
tail -1 $O/fuzz_gemm.jsonl
