set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q > gpurun_out/gemm_tests.log 2>&1
timeout -k 10 200 python tools/gemm_stamps.py --shape 14336,4096 --cfg 2,8,8,1,4 --cfg 2,4,8,1,2 > gpurun_out/stamps.jsonl 2>&1
timeout -k 10 200 python tools/gemm_stamps.py --shape 4096,14336 --cfg 2,8,8,1,1 >> gpurun_out/stamps.jsonl 2>&1
C="--cfg 2,8,8,1,4 --cfg 2,4,8,1,2 --cfg 2,8,8,1,1 --cfg 2,4,8,1,1 --cfg 2,8,4,1,4 --cfg 2,8,2,1,4 --cfg 2,8,2,1,1"
timeout -k 10 120 python tools/gemm_probe.py --lib prod --shape 14336,4096 --shape 4096,4096 --shape 4096,14336 --shape 1024,4096 --m 1 $C > gpurun_out/probe.jsonl 2>&1
