# round 6 session 6: the persistent decode-GEMM kernel with ONE lookup pipeline across
# chunks (NF4_PERSIST_CONT, tools/_build/libnf4dq_abl_cont.so) -- correctness (fuzz against the
# float64 oracle) and A/B against the product, eager, streamed weights.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s6
mkdir -p $O
NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_cont.so timeout -k 10 300 python3 -u tools/fuzz_gemm.py --cases 600 --seed 66 \
    > $O/fuzz_gemm_cont.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_gemm_cont.jsonl
S="14336,4096;4096,4096;6144,4096;28672,4096;4096,14336"
C="default;3,8,4,1,4;3,8,2,1,4;3,8,4,1,2;3,8,2,1,2"
for round in 1 2; do
    timeout -k 10 400 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "$S" --cfgs "$C" --label prod >> $O/gemm_cont_ab.jsonl 2>> $O/ab.err
    NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_cont.so timeout -k 10 400 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "$S" \
        --cfgs "$C" --label cont >> $O/gemm_cont_ab.jsonl 2>> $O/ab.err
done
grep -c . $O/gemm_cont_ab.jsonl
