# round 5 session 10: parity sweeps of the table-decode kernel (drop-in, multi-weight,
# single-quant), every BASELINE config re-timed and re-verified, and the decode-GEMM
# occupancy close-out (persistent kernel, 8 vs 16 waves per workgroup, SQ counters)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s10
mkdir -p $O
timeout -k 10 200 python -u tools/fuzz_dequant.py --cases 20000 --seed 5 --seconds 150 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
timeout -k 10 200 python -u tools/fuzz_api.py --rounds 400 --seed 5 --seconds 150 > $O/fuzz_api.jsonl 2>> $O/fuzz.err
tail -1 $O/fuzz_api.jsonl
timeout -k 10 900 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err
python -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print({k: d[k] for k in list(d)[:8]})
"
for cfg in default "3,8,2,1,4" "3,16,2,1,4" "3,16,4,1,4"; do
  for M in 1 8; do
    GA="tools/gemm_ab.py --ms $M --shapes 14336,4096 --budget-mb 512 --cfgs $cfg"
    timeout -k 10 200 python -u $GA >> $O/gemm_occ.jsonl 2>> $O/gemm_occ.err
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmcg_a" -o a -- \
        python3 -u $GA > "$O/pmcg_a.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM \
        SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL \
        --output-format csv -d "$O/pmcg_b" -o b -- python3 -u $GA > "$O/pmcg_b.log" 2>&1
    python3 tools/pmc_gemm.py "$O" nf4_gemm_persist_kernel | sed "s/^{/{\"cfg\": \"$cfg\", \"M\": $M, /" >> $O/pmc_gemm_occ.jsonl
    rm -rf "$O/pmcg_a" "$O/pmcg_b"
  done
done
cat $O/gemm_occ.jsonl
cat $O/pmc_gemm_occ.jsonl
