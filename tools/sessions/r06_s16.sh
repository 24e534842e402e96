# round 6 session 16: what the persistent decode GEMM's per-step x-fragment LDS reads cost
# (ablation noxr: x from registers, wrong results) at M = 1, 14336x4096 and 4096^2, and the
# library default against strips = 1 (the decomposition a register-resident x would need).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s16
mkdir -p $O
timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1 --shapes "14336,4096;4096,4096" --cfgs "default;3,8,2,1,1;3,8,2,1,2" > $O/gemm_prod.jsonl 2> $O/gemm_prod.err
cat $O/gemm_prod.jsonl
NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_noxr.so timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1 --shapes "14336,4096;4096,4096" --cfgs "default;3,8,2,1,1" --label noxr > $O/gemm_noxr.jsonl 2> $O/gemm_noxr.err
cat $O/gemm_noxr.jsonl
