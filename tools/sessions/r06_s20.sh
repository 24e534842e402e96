# round 6 session 20: the piece kernels after factoring their shared parts (piece_wave,
# piece_scale, piece_codes) -- correctness and a timing check against the staged library.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s20
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 8000 --seed 76 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 64 --cases chunk_4090,chunk_4095,oal_4096,unal_4096,pad_4096 \
    --libs tools/_build/libnf4dq_staged.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 32 --dtype f32 --cases chunk_4090,chunk_4095,pad_4096,flat_4096 \
    > $O/chunk_ab_f32.jsonl 2> $O/chunk_ab_f32.err
cat $O/chunk_ab_f32.jsonl
