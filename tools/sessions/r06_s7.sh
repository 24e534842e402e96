# round 6 session 7: the chunk kernel's staged forms store each step's finished pieces while
# the next steps decode (instead of all after the last step) -- correctness (chunk + past-the-
# end suites, fuzz with odd pointer offsets) and A/B against the previous library (prev: edge
# lines default policy + one end-piece pass) and the s3 variant fe1.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s7
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 8000 --seed 67 --seconds 240 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 \
    --cases chunk_4090,chunk_4095,pad_4096,unal_4096,chunk_4080,flat_4096 \
    --libs tools/_build/libnf4dq_prev.so,tools/_build/libnf4dq_dqv_fe1.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
