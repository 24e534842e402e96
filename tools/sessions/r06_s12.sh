# round 6 session 12: the piece kernel's counters (HBM traffic from calibrated FETCH_SIZE /
# WRITE_SIZE passes, SQ instruction counts per wave) on its three 4096-row forms; then the
# whole GPU suite, a dequant soak with the piece and LDS-staged forms, and the API fuzzer.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s12
mkdir -p $O
for C in chunk_4090 chunk_4095 oal_4096; do
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_$C" -o fetch -- \
        python3 -u tools/pmc_chunk.py > "$O/pmc_fetch_$C.log" 2>&1
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_$C" -o write -- \
        python3 -u tools/pmc_chunk.py > "$O/pmc_write_$C.log" 2>&1
    PMC_KERNEL=nf4_piece PMC_CASE=$C python3 tools/pmc_traffic.py "$O/pmc_$C" "$O/pmc_piece_$C.json" >> $O/pmc_piece.jsonl 2>&1
    PMC_CASE=$C timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
        SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$O/pmcsq_$C" -o sq -- \
        python3 -u tools/pmc_chunk.py > "$O/pmcsq_$C.log" 2>&1
    rm -rf "$O/pmc_$C"
done
cat $O/pmc_piece.jsonl
python3 tools/pmc_sq_summary.py nf4_piece $O/pmcsq_chunk_4090 $O/pmcsq_chunk_4095 $O/pmcsq_oal_4096 > $O/pmc_sq_piece.jsonl
cat $O/pmc_sq_piece.jsonl
rm -rf $O/pmcsq_*
bash tools/session.sh r06_s12 gputest smoke
timeout -k 10 240 python3 -u tools/soak_dequant.py --seconds 150 > $O/soak_dequant_150s.jsonl 2> $O/soak.err
tail -1 $O/soak_dequant_150s.jsonl
timeout -k 10 300 python3 -u tools/fuzz_api.py --rounds 1000 --seed 72 --seconds 200 > $O/fuzz_api.jsonl 2> $O/fuzz_api.err
tail -1 $O/fuzz_api.jsonl
