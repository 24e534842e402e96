# round 6 session 5: the decode GEMM's floor on the current tree -- ablation builds of the
# persistent kernel (tools/gemm_ablate.hip) at 14336x4096 and 4096^2, M = 1, eager, streamed;
# SQ counters of the product and the no-memory build; the Llama-3-8B decode pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s5
mkdir -p $O
S="14336,4096;4096,4096"
timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1 --shapes "$S" --label prod >> $O/ablation.jsonl 2>> $O/ab.err
for v in empty noloop noring skeleton nomma nolut; do
    NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_$v.so timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1 --shapes "$S" \
        --label $v >> $O/ablation.jsonl 2>> $O/ab.err
done
timeout -k 10 300 python3 -u tools/gemm_ab.py --ms 1 --shapes "$S" --label prod_again >> $O/ablation.jsonl 2>> $O/ab.err
cat $O/ablation.jsonl
GA="tools/gemm_ab.py --ms 1 --shapes 14336,4096 --budget-mb 512"
for lib in prod noring; do
    if [ $lib = noring ]; then export NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_noring.so; fi
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmca_$lib" -o a -- \
        python3 -u $GA > "$O/pmca_$lib.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL --output-format csv -d "$O/pmcb_$lib" -o b -- \
        python3 -u $GA > "$O/pmcb_$lib.log" 2>&1
done
unset NF4DQ_LIB_PATH
python3 tools/pmc_sq_summary.py nf4_gemm_persist $O/pmca_prod $O/pmcb_prod $O/pmca_noring $O/pmcb_noring > $O/pmc_sq.jsonl
cat $O/pmc_sq.jsonl
timeout -k 10 600 python3 -u tools/bench_gemm.py --ms 1,8,32 --no-composite > $O/bench_gemm.jsonl 2> $O/bench_gemm.err
cat $O/bench_gemm.jsonl
