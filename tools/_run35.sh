# register-resident GEMM today: product vs no-LDS-reduction (xr1) vs no dequant/MFMA (xr3) at M = 1, 32 on 14336x4096
# needs the diagnostic builds staged where the GPU box receives them: make -C tools xrdbg; mkdir -p tools/_diag; cp tools/_build/libnf4dq_xr1.so tools/_diag/diag_xr1.so; cp tools/_build/libnf4dq_xr3.so tools/_diag/diag_xr3.so
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r35 && export TMPDIR=/tmp
O=gpurun_out/r35
for v in prod 1 3; do
  if [ $v = prod ]; then unset NF4DQ_LIB_PATH; else export NF4DQ_LIB_PATH=$PWD/tools/_diag/diag_xr$v.so; fi
  timeout -k 10 300 python -u tools/sweep_gemm.py --ms 1,32 --kernels 5 --shapes "14336,4096;4096,14336" > $O/sweep_$v.jsonl 2> $O/sweep_$v.err || exit 1
done
echo ALLDONE
