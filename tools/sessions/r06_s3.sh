# round 6 session 3: what makes the chunk kernel's LDS-staged forms (n % 8 != 0) slow --
# the span-edge lines shared by two waves?  A/B of the product against three flush variants
# (tools/dq_variants.hip DQV_FE: edge lines default policy / no end-piece element stores
# (timing only) / every flush store default policy), interleaved, HBM-streamed.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s3
mkdir -p $O
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 7 --steps 64 --cases chunk_4090,chunk_4095,pad_4096 \
    --libs tools/_build/libnf4dq_dqv_fe1.so,tools/_build/libnf4dq_dqv_fe2.so,tools/_build/libnf4dq_dqv_fe3.so \
    > $O/chunk_flush_variants.jsonl 2> $O/chunk_ab.err
cat $O/chunk_flush_variants.jsonl
