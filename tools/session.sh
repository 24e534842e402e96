#!/bin/bash
# One parametrised GPU-box session (replaces the per-call tools/_run*.sh scripts of
# rounds 1-2, which are in git history).  Usage, on the box:
#   bash tools/session.sh <out-subdir> <stage> [<stage> ...]
# Every stage writes under gpurun_out/<out-subdir>/; every GPU step runs under its
# own time limit and the session stops at the first failing step.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
PY="python -u"

trace() {  # trace <name> <kernel-substring> <last-K> <timeout> -- <python args...>
    local name=$1 kern=$2 k=$3 to=$4
    shift 5
    timeout -k 10 "$to" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o "$name" -- \
        python3 -u "$@" > "$O/$name.out" 2> "$O/$name.err"
    python3 tools/trace_gaps.py "$O/prof_$name" "$kern" "$k" > "$O/${name}_gaps.txt"
    tail -1 "$O/${name}_gaps.txt"
}

for stage in "$@"; do
    echo "== stage $stage" >&2
    case $stage in
    gputest)
        timeout -k 10 900 $PY -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > "$O/gputest.log" 2>&1 || { tail -30 "$O/gputest.log"; exit 1; }
        tail -3 "$O/gputest.log" ;;
    smoke)
        timeout -k 10 300 $PY __graft_entry__.py smoke > "$O/smoke.log" 2>&1; cat "$O/smoke.log" ;;
    bench)
        timeout -k 10 300 $PY bench.py > "$O/bench.json" 2> "$O/bench.err"; cat "$O/bench.json" ;;
    bench20)
        timeout -k 10 200 $PY bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_k20.json" 2>> "$O/bench.err"
        cat "$O/bench_k20.json" ;;
    multirank)  # N ranks on the one GPU of a lease (gloo; the driver's 8-GPU node runs RCCL)
        timeout -k 10 400 $PY bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 > "$O/bench_g2_gloo.json" 2> "$O/bench_g2.err"
        cat "$O/bench_g2_gloo.json" ;;
    c5probe)
        timeout -k 10 400 $PY tools/c5_probe.py > "$O/c5_probe.jsonl" 2> "$O/c5_probe.err"; cat "$O/c5_probe.jsonl" ;;
    valsens)
        timeout -k 10 300 $PY tools/value_sensitivity.py > "$O/value_sensitivity.jsonl" 2> "$O/vs.err"
        cat "$O/value_sensitivity.jsonl" ;;
    c5bench)
        timeout -k 10 200 $PY bench.py --m 8192 --n 8192 --steps 64 --no-cpu-baseline > "$O/bench_8192.json" 2> "$O/bench_8192.err"
        timeout -k 10 200 $PY bench.py --workload c5 --steps 20 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err"
        timeout -k 10 600 $PY tools/bench_configs.py --configs c5 > "$O/configs_c5.jsonl" 2> "$O/configs_c5.err"
        cat "$O/bench_8192.json" "$O/bench_c5.json" "$O/configs_c5.jsonl" ;;
    c5knobs)  # launch-shape variants at 8192^2 (eager, per-set absmax): KNOBS="label:args;label:args"
        IFS=';' read -ra KS <<< "${KNOBS:-default:;bpc8:--blocks-per-cu 8;bpc8_a1ahead:--blocks-per-cu 8 --flags 8;bpc4_a1ahead:--blocks-per-cu 4 --flags 8;bpc16_a1ahead:--blocks-per-cu 16 --flags 8;u8:--tile-dwords 8}"
        for kv in "${KS[@]}"; do
            lab=${kv%%:*}; a=${kv#*:}
            timeout -k 10 200 $PY bench.py --m 8192 --n 8192 --steps 64 --no-cpu-baseline $a > "$O/knob_$lab.json" 2>> "$O/knobs.err"
            python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['roofline']['launch_us_mean'],3), round(d['roofline']['frac'],4))" "$O/knob_$lab.json" "$lab"
        done ;;
    gstamps)  # fused-GEMM phase stamps (tools/_build/libnf4dq_gstamps.so, built here)
        for spec in ${GSTAMPS:-"14336,4096:32" "14336,4096:16" "14336,4096:1" "4096,4096:32" "4096,14336:32"}; do
            timeout -k 10 200 $PY tools/gemm_stamps.py --shape ${spec%%:*} --m ${spec##*:} ${GSTAMP_CFGS:-} >> "$O/gemm_stamps.jsonl" 2>> "$O/gemm_stamps.err"
        done
        cat "$O/gemm_stamps.jsonl" ;;
    dqab)  # interleaved dequant launch-config A/B: DQAB_ARGS passed to tools/dq_ab.py
        timeout -k 10 400 $PY tools/dq_ab.py ${DQAB_ARGS:-} > "$O/dq_ab.jsonl" 2> "$O/dq_ab.err"; cat "$O/dq_ab.jsonl" ;;
    cacheab)  # independent input / output rotation (tools/cache_ab.py): CACHEAB_RUNS="tag|args;tag|args"
        IFS=';' read -ra RS <<< "${CACHEAB_RUNS:-bf16|}"
        for kv in "${RS[@]}"; do
            timeout -k 10 300 $PY tools/cache_ab.py --tag "${kv%%|*}" ${kv#*|} >> "$O/cache_ab.jsonl" 2>> "$O/cache_ab.err"
        done
        cat "$O/cache_ab.jsonl" ;;
    tprobe)  # split-K timeout is reported (tools/_build/libnf4dq_abl_dropslice.so, built here): ONE run
        test -f tools/_build/libnf4dq_abl_dropslice.so
        NF4DQ_LIB_PATH=tools/_build/libnf4dq_abl_dropslice.so timeout -k 10 120 $PY tools/splitk_timeout_probe.py \
            > "$O/splitk_timeout_probe.jsonl" 2> "$O/tprobe.err"
        timeout -k 10 120 $PY tools/splitk_timeout_probe.py >> "$O/splitk_timeout_probe.jsonl" 2>> "$O/tprobe.err"
        cat "$O/splitk_timeout_probe.jsonl" ;;
    gemmab)  # decode GEMM per launch, product vs the A/B libraries named in ABLIBS (tools/_build/libnf4dq_<x>.so)
        timeout -k 10 300 $PY tools/gemm_ab.py ${GEMMAB_ARGS:-} >> "$O/gemm_ab.jsonl" 2>> "$O/gemm_ab.err"
        for x in ${ABLIBS:-}; do
            NF4DQ_LIB_PATH=tools/_build/libnf4dq_$x.so timeout -k 10 300 $PY tools/gemm_ab.py ${GEMMAB_ARGS:-} >> "$O/gemm_ab.jsonl" 2>> "$O/gemm_ab.err"
        done
        cat "$O/gemm_ab.jsonl" ;;
    gemmab2)  # a second decode-GEMM A/B with its own arguments (GEMMAB2_ARGS)
        timeout -k 10 300 $PY tools/gemm_ab.py ${GEMMAB2_ARGS:-} >> "$O/gemm_ab2.jsonl" 2>> "$O/gemm_ab2.err"
        cat "$O/gemm_ab2.jsonl" ;;
    ceiling)  # memory-system twin of the dequant access mix vs the kernel (tools/hbm_ceiling.py)
        timeout -k 10 300 $PY tools/hbm_ceiling.py > "$O/hbm_ceiling.jsonl" 2> "$O/hbm_ceiling.err"
        cat "$O/hbm_ceiling.jsonl" ;;
    gemmtest)
        timeout -k 10 600 $PY -m pytest tests/test_gpu_gemm.py tests/test_gpu_redzones.py tests/test_gpu_concurrency.py -x -q \
            --timeout 300 --timeout-method thread > "$O/gemmtest.log" 2>&1 || { tail -30 "$O/gemmtest.log"; exit 1; }
        tail -2 "$O/gemmtest.log" ;;
    dqtest)
        timeout -k 10 600 $PY -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_configs.py -x -q \
            --timeout 300 --timeout-method thread > "$O/dqtest.log" 2>&1 || { tail -30 "$O/dqtest.log"; exit 1; }
        tail -2 "$O/dqtest.log" ;;
    c5trace)
        trace configs_c5 nf4_flat_kernel 32 600 -- tools/bench_configs.py --configs c5
        trace bench_8192 nf4_flat_kernel 64 300 -- bench.py --m 8192 --n 8192 --steps 64 --no-cpu-baseline ;;
    rocprof)
        trace bench nf4_flat_kernel 200 300 -- bench.py --steps 200 --repeats 1 --no-cpu-baseline --no-c5 \
            --no-ceiling --spin-us-per-launch 500
        python3 tools/rocprof_summary.py "$O/prof_bench" nf4_flat_kernel "$O/rocprof_bench_summary.json" \
            "$O/rocprof_bench_kernel_stats.csv" --last 200 > /dev/null ;;
    pmc)  # headline HBM traffic (FETCH_SIZE / WRITE_SIZE passes, calibrated) + decode-GEMM SQ counters
        test -f tools/_build/libpmccalib.so
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc" -o fetch -- \
            python3 -u tools/pmc_probe.py > "$O/pmc_fetch.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc" -o write -- \
            python3 -u tools/pmc_probe.py > "$O/pmc_write.log" 2>&1
        python3 tools/pmc_traffic.py "$O/pmc" "$O/pmc_traffic.json" > "$O/pmc_traffic.log" 2>&1
        cat "$O/pmc_traffic.json"
        rm -rf "$O/pmc"
        # the fp16 leg of BASELINE configs[3] (C4), same passes
        PMC_DTYPE=f16 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc" -o fetch -- \
            python3 -u tools/pmc_probe.py > "$O/pmc_fetch_f16.log" 2>&1
        PMC_DTYPE=f16 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc" -o write -- \
            python3 -u tools/pmc_probe.py > "$O/pmc_write_f16.log" 2>&1
        PMC_DTYPE=f16 python3 tools/pmc_traffic.py "$O/pmc" "$O/pmc_traffic_f16.json" > "$O/pmc_traffic_f16.log" 2>&1
        cat "$O/pmc_traffic_f16.json"
        GA="tools/gemm_ab.py --ms ${PMC_M:-32} --shapes ${PMC_SHAPE:-14336,4096} --budget-mb 512"
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmcg_a" -o a -- \
            python3 -u $GA > "$O/pmcg_a.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM \
            SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL \
            --output-format csv -d "$O/pmcg_b" -o b -- python3 -u $GA > "$O/pmcg_b.log" 2>&1
        python3 tools/pmc_gemm.py "$O" nf4_gemm_xrg_kernel nf4_gemm_xr_kernel nf4_gemm_persist_kernel nf4_gemm_stream_kernel > "$O/pmc_gemm.jsonl"
        cat "$O/pmc_gemm.jsonl" ;;
    pmcg)  # decode-GEMM SQ counters only (PMC_M, PMC_SHAPE; NF4DQ_LIB_PATH selects a build)
        GA="tools/gemm_ab.py --ms ${PMC_M:-1} --shapes ${PMC_SHAPE:-14336,4096} --budget-mb 512"
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d "$O/pmcg_a" -o a -- \
            python3 -u $GA > "$O/pmcg_a.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM \
            SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL \
            --output-format csv -d "$O/pmcg_b" -o b -- python3 -u $GA > "$O/pmcg_b.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA \
            SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY \
            --output-format csv -d "$O/pmcg_c" -o c -- python3 -u $GA > "$O/pmcg_c.log" 2>&1
        python3 tools/pmc_gemm.py "$O" nf4_gemm_persist_kernel nf4_gemm_xrg_kernel nf4_gemm_xr_kernel > "$O/pmcg${PMC_TAG:-}.jsonl"
        rm -rf "$O/pmcg_a" "$O/pmcg_b" "$O/pmcg_c"
        cat "$O/pmcg${PMC_TAG:-}.jsonl" ;;
    sweep)  # fused-GEMM decomposition sweep: SWEEP_ARGS passed to tools/sweep_gemm.py
        timeout -k 10 600 $PY tools/sweep_gemm.py ${SWEEP_ARGS:-} > "$O/sweep_gemm.jsonl" 2> "$O/sweep_gemm.err"
        python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(d['N'], d['K'], d['M'], 'default', d['default_us'], 'best', d['best'][:3])" "$O/sweep_gemm.jsonl" ;;
    gemmpass)  # the Llama-3-8B decode pass, fused GEMM (tools/bench_gemm.py)
        timeout -k 10 500 $PY tools/bench_gemm.py --ms ${GEMM_MS:-1,4,8,12,16,24,32} > "$O/bench_gemm.jsonl" 2> "$O/bench_gemm.err"
        cat "$O/bench_gemm.jsonl" ;;
    gemmtrace)  # kernel trace + stats of the fused decode pass (grouped form only), GEMM_MS (default 1,32)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_gemm" -o gemm -- \
            python3 -u tools/bench_gemm.py --ms ${GEMM_MS:-1,32} --no-bf16 --no-composite > "$O/gemmtrace.out" 2> "$O/gemmtrace.err"
        find "$O/prof_gemm" -name "*kernel_stats.csv" -exec cp {} "$O/gemm_kernel_stats.csv" \;
        rm -rf "$O/prof_gemm"
        cat "$O/gemm_kernel_stats.csv" ;;
    configs)
        timeout -k 10 900 $PY tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err"; cat "$O/configs.jsonl" ;;
    *)
        echo "unknown stage $stage" >&2; exit 2 ;;
    esac
done
echo "session done" >&2
