# round 6 session 1: measurements the round-5 verdict asks for, on the current tree
#  (a) decode-GEMM phase stamps, product (M = 1, 8) and the no-memory/no-lookup/no-MFMA
#      skeleton (M = 1), 14336x4096
#  (b) PMC traffic of the chunk kernel's forms (item 3) + SQ instruction counters
#  (c) the reference harness's timing loop, split into its parts (item 6)
#  (d) the GEMM tests touched by the SK removal
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py -k "retired or persistent" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_redzones.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_rz.log 2>&1
tail -2 $O/tests_rz.log
for M in 1 8; do
    timeout -k 10 300 python3 -u tools/gemm_stamps.py --shape 14336,4096 --m $M --launches 8 >> $O/stamps.jsonl 2> $O/stamps.err
done
timeout -k 10 300 python3 -u tools/gemm_stamps.py --variant skeleton --shape 14336,4096 --m 1 --launches 8 >> $O/stamps.jsonl 2>> $O/stamps.err
cat $O/stamps.jsonl
for C in chunk_4080 chunk_4090 chunk_4095 pad_4096 unal_4096; do
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_$C" -o fetch -- \
        python3 -u tools/pmc_chunk.py > "$O/pmc_fetch_$C.log" 2>&1
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_$C" -o write -- \
        python3 -u tools/pmc_chunk.py > "$O/pmc_write_$C.log" 2>&1
    PMC_KERNEL=nf4_chunk PMC_CASE=$C python3 tools/pmc_traffic.py "$O/pmc_$C" "$O/pmc_chunk_$C.json" >> $O/pmc_chunk.jsonl 2>&1
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
        SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$O/pmcsq_$C" -o sq -- \
        python3 -u tools/pmc_chunk.py > "$O/pmcsq_$C.log" 2>&1 || echo "sq pass failed: $C"
    rm -rf "$O/pmc_$C"
done
cat $O/pmc_chunk.jsonl
timeout -k 10 300 python3 -u tools/harness_reference_style.py --iterations 1000 > $O/harness_reference_style.jsonl 2> $O/harness.err
cat $O/harness_reference_style.jsonl
