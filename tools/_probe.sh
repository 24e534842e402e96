set -e
cd /tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_gemm
P="python $R/tools/gemm_probe.py --shape 14336,4096 --m 32 --cfg 1,8,1,1,4 --budget-mb 256"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA --output-format csv -d $R/gpurun_out/pmc_gemm -o p1 -- $P > $R/gpurun_out/pmc_gemm/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_gemm -o p2 -- $P > $R/gpurun_out/pmc_gemm/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_gemm -o kt -- $P > $R/gpurun_out/pmc_gemm/kt.log 2>&1
