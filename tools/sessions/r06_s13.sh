# round 6 session 13: the piece kernel without per-step branches or multiplies (row bases by
# additions, ib by min3, byte masks by per-byte subtraction) -- correctness, then A/B against
# its first version (piece1) and the staged library.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s13
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 6000 --seed 73 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 \
    --cases chunk_4090,chunk_4095,oal_4096 \
    --libs tools/_build/libnf4dq_piece1.so,tools/_build/libnf4dq_staged.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
