# register-resident decode GEMM: parity tests, product vs diagnostic builds (tools/Makefile xrdbg), sweep vs the other kernels
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r18 && export TMPDIR=/tmp
O=gpurun_out/r18
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread -k "register_resident" > $O/pytest_xr.log 2>&1; rc=$?; tail -3 $O/pytest_xr.log; [ $rc -eq 0 ] || exit $rc
for v in prod 1 2 3; do
  if [ $v = prod ]; then unset NF4DQ_LIB_PATH; else export NF4DQ_LIB_PATH=$PWD/tools/_build/libnf4dq_xr$v.so; fi
  timeout -k 10 300 python -u tools/sweep_gemm.py --ms 1,32 --kernels 5 --shapes "14336,4096" > $O/sweep_$v.jsonl 2> $O/sweep_$v.err || exit 1
done
unset NF4DQ_LIB_PATH
timeout -k 10 600 python -u tools/sweep_gemm.py --ms 1,8,16,32 --kernels 1,4,5 --shapes "14336,4096;4096,4096;4096,14336;1024,4096;6144,4096;28672,4096" > $O/sweep.jsonl 2> $O/sweep.err || exit 1
echo ALLDONE
