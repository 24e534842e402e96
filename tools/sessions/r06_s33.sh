# round 6 session 33: the GEMM fuzzer with a third of its cases in the decode GEMV's domain
# (M = 1, K % 2048 == 0, N <= 4096: the library's choice; a fifth with wrapping absmax, which
# falls back to the persistent kernel) and drawn GEMV configurations among the explicit ones.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s33
mkdir -p $O
timeout -k 10 400 python3 -u tools/fuzz_gemm.py --cases 3000 --seed 91 --seconds 300 --gemv-rate 0.33 --cfg-rate 0.4 \
    > $O/fuzz_gemm_gemv.jsonl 2> $O/fuzz_gemm_gemv.err
tail -1 $O/fuzz_gemm_gemv.jsonl
