cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r10 && export TMPDIR=/tmp
O=gpurun_out/r10
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "shared_activation or slices_starting" > $O/xs_tests.log 2>&1; rc=$?; tail -15 $O/xs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/sweep_gemm.py --ms 16,24,32 --kernels 1,4 --shapes "14336,4096;4096,4096;4096,14336;1024,4096;6144,4096;28672,4096" > $O/sweep.jsonl 2> $O/sweep.err
python - <<'PY'
import json
for l in open('gpurun_out/r10/sweep.jsonl'):
    d=json.loads(l); b=d['best'][:4]
    xs=[r for r in d['all'] if r['cfg'][0]==4][:2]
    print(d['N'],d['K'],d['M'],'default',d['default_us'],'best',[(r['cfg'],r['us']) for r in b],'best_xs',[(r['cfg'],r['us']) for r in xs])
PY
echo ALLDONE
