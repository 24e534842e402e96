cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r12 && export TMPDIR=/tmp
O=gpurun_out/r12
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_strided.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1; rc=$?; tail -5 $O/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_gemm.py --ms 1,8,16,24,32 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err || exit 1
python -c "
import json
for l in open('$O/bench_gemm.jsonl'):
    d=json.loads(l); print(d['M'], 'grouped_ms', round(d['grouped_ms'],3), 'fused_ms', round(d['fused_ms'],3), 'composite', round(d['composite_ms'],3), 'bf16', d.get('bf16_ms'))
"
echo ALLDONE
