# round 6 session 4: (1) chunk kernel staged forms: the product now writes the span's edge
# lines with the default policy and both end pieces in one pass -- tests, fuzz, A/B against
# the s3 variant with the edge-line policy only (dqv_fe1) and the round-start library (prev);
# (2) decode GEMM: the persistent kernel's x staging now runs only the iterations that hold
# pieces -- A/B against the previous library, 8 vs 16 waves per workgroup at M = 1 / 8 on the
# Llama-3-8B launch shapes (eager, streamed weights); the persistent GEMM tests.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py -k "persistent or retired" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 6000 --seed 63 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 \
    --cases flat_4096,chunk_4080,chunk_4090,chunk_4095,pad_4096,unal_4096 \
    --libs tools/_build/libnf4dq_dqv_fe1.so,tools/_build/libnf4dq_prev.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
S="14336,4096;4096,4096;6144,4096;28672,4096"
C="default;3,16,2,1,4;3,16,2,1,2;3,16,2,1,1;3,16,4,1,4;3,8,2,1,4;3,8,2,1,2"
for lib in prod prev; do
    if [ $lib = prev ]; then export NF4DQ_LIB_PATH=tools/_build/libnf4dq_prev.so; fi
    timeout -k 10 400 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "$S" --cfgs "$C" --label $lib >> $O/gemm_waves_ab.jsonl 2>> $O/gemm_ab.err
done
unset NF4DQ_LIB_PATH
cat $O/gemm_waves_ab.jsonl
