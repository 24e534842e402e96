# round 6 session 23: padded 16-bit rows stored whole stay on the chunk kernel; the padded
# forms that were staged (n % 8 != 0) through the piece kernel -- correctness and A/B.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s23
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 6000 --seed 79 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 64 --cases padodd_4090,pad_4096 \
    --libs tools/_build/libnf4dq_staged.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 32 --dtype f32 --cases padodd_4090 \
    --libs tools/_build/libnf4dq_staged.so > $O/chunk_ab_f32.jsonl 2> $O/chunk_ab_f32.err
cat $O/chunk_ab_f32.jsonl
