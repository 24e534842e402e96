# round 6 session 14: piece kernel -- output halves joined by one v_perm (product) and the
# 8-byte packed-load variant (dqv_ld64): correctness of both, then A/B with the first version.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s14
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_edges.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks.log 2>&1
tail -2 $O/tests_chunks.log
NF4DQ_LIB_PATH=tools/_build/libnf4dq_dqv_ld64.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py \
    tests/test_gpu_edges.py -x -q -k "not drop_in" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_chunks_ld64.log 2>&1
tail -2 $O/tests_chunks_ld64.log
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 \
    --cases chunk_4090,chunk_4095,oal_4096 \
    --libs tools/_build/libnf4dq_dqv_ld64.so,tools/_build/libnf4dq_piece1.so > $O/chunk_ab.jsonl 2> $O/chunk_ab.err
cat $O/chunk_ab.jsonl
