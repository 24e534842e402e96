# round 6 session 22: padded packed rows through the piece kernels (a piece crossing its row's
# end loads the next row's first bytes apart) -- correctness, soak, and padded 4096^2 bf16 /
# fp32 against the staged library.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s22
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 8000 --seed 78 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 200 python3 -u tools/soak_dequant.py --seconds 90 > $O/soak_dequant_90s.jsonl 2> $O/soak.err
tail -1 $O/soak_dequant_90s.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 64 --cases pad_4096,chunk_4090,chunk_4095 \
    --libs tools/_build/libnf4dq_staged.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 32 --dtype f32 --cases pad_4096,chunk_4090 \
    --libs tools/_build/libnf4dq_staged.so > $O/chunk_ab_f32.jsonl 2> $O/chunk_ab_f32.err
cat $O/chunk_ab_f32.jsonl
