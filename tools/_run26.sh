# PMC counters of the M = 32 decode GEMM on 14336x4096: register-resident (library default) vs shared-activation kernel
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r26 && export TMPDIR=/tmp
O=gpurun_out/r26
P="python -u tools/gemm_probe.py --shape 14336,4096 --m 32 --cfg 5,8,2,2,2 --cfg 4,8,8,4,1 --budget-mb 256"
timeout -k 10 200 $P > $O/probe_times.jsonl 2> $O/probe.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL --output-format csv -d $O/pmc -o passA -- $P > $O/passA.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --output-format csv -d $O/pmc -o passB -- $P > $O/passB.log 2>&1 || exit 1
python tools/pmc_gemm.py $O/pmc nf4_gemm_xr_kernel nf4_gemm_xs_kernel > $O/pmc_summary.jsonl
cat $O/probe_times.jsonl $O/pmc_summary.jsonl
echo ALLDONE
