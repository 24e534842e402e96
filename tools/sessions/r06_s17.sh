# round 6 session 17: the fp32-output forms of the chunk kernels (and fp16 of the piece
# kernel), HBM-streamed, one library -- where fp32 output of odd shapes stands.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s17
mkdir -p $O
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 32 --dtype f32 \
    --cases flat_4096,chunk_4080,chunk_4090,chunk_4095,oal_4096,pad_4096,unal_4096 > $O/chunk_ab_f32.jsonl 2> $O/chunk_ab_f32.err
cat $O/chunk_ab_f32.jsonl
timeout -k 10 300 python3 -u tools/chunk_ab.py --rounds 5 --steps 64 --dtype f16 \
    --cases flat_4096,chunk_4090,chunk_4095,oal_4096 > $O/chunk_ab_f16.jsonl 2> $O/chunk_ab_f16.err
cat $O/chunk_ab_f16.jsonl
