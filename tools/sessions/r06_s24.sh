# round 6 session 24: the x-fragment ablation redone cleanly (one constant fragment in
# registers, no VALU per step; s16's build rebuilt each fragment with 4 VALU per step).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s24
mkdir -p $O
timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "14336,4096;4096,4096" > $O/gemm_prod.jsonl 2> $O/gemm_prod.err
cat $O/gemm_prod.jsonl
NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_noxr.so timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "14336,4096;4096,4096" --label noxr > $O/gemm_noxr.jsonl 2> $O/gemm_noxr.err
cat $O/gemm_noxr.jsonl
