# round 6 session 2: the chunk kernel's staged-store change (one address per chunk, range-
# checked end pieces) -- correctness (chunk + past-the-end suites, fuzz), A/B against the
# previous library on every chunk form; decode-GEMM phase stamps in the back-to-back regime
# (chain 8) for the product, the skeleton and the no-memory build; the reference harness.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/fuzz_dequant.py --cases 4000 --seed 62 --seconds 200 --abi-rate 0.5 > $O/fuzz.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 \
    --cases flat_4096,chunk_4080,chunk_4090,chunk_4095,pad_4096,unal_4096 --libs tools/_build/libnf4dq_prev.so \
    > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
for V in "" skeleton noring; do
    timeout -k 10 300 python3 -u tools/gemm_stamps.py ${V:+--variant $V} --chain 8 --shape 14336,4096 --m 1 --launches 6 \
        >> $O/stamps_chain8.jsonl 2>> $O/stamps.err
done
cat $O/stamps_chain8.jsonl
timeout -k 10 300 python3 -u tools/harness_reference_style.py --iterations 1000 > $O/harness_reference_style.jsonl 2> $O/harness.err
cat $O/harness_reference_style.jsonl
