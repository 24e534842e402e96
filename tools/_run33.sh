# persistent (3) vs register-resident (5) decode GEMM at 8 < M <= 16 on the Llama shapes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r33 && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/sweep_gemm.py --ms 12,16 --kernels 3,5 --shapes "14336,4096;4096,4096;4096,14336;1024,4096;6144,4096;28672,4096" > gpurun_out/r33/sweep.jsonl 2> gpurun_out/r33/sweep.err || exit 1
echo ALLDONE
