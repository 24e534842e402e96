cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r11 && export TMPDIR=/tmp
O=gpurun_out/r11
for v in prod xs1 xs2; do
  if [ $v = prod ]; then unset NF4DQ_LIB_PATH; else export NF4DQ_LIB_PATH=$PWD/tools/_build/libnf4dq_$v.so; fi
  timeout -k 10 300 python -u tools/sweep_gemm.py --ms 32 --kernels 4 --shapes "14336,4096;28672,4096" > $O/sweep_$v.jsonl 2> $O/sweep_$v.err || exit 1
  python - $v <<'PY'
import json,sys
for l in open(f'gpurun_out/r11/sweep_{sys.argv[1]}.jsonl'):
    d=json.loads(l); print(sys.argv[1], d['N'], d['K'], d['M'], [(r['cfg'][1:3], r['us']) for r in d['all']])
PY
done
echo ALLDONE
