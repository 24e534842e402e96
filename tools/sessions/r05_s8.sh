# round 5 session 8: scale gathers as buffer loads (default / sc0 policy) vs the product, 15
# interleaved rounds; the split-K error-path tests
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s8
mkdir -p $O
D=tools/_build
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "error_word or check_gemm" > $O/gemm_err_tests.log 2>&1 || { tail -30 $O/gemm_err_tests.log; exit 1; }
tail -2 $O/gemm_err_tests.log
timeout -k 10 500 python -u tools/stream_probe.py --tag a1buf --steps 20,128 --rounds 15 --libs $D/libnf4dq_dqv_a1p0.so,$D/libnf4dq_dqv_a1sc0.so --kernels prod,dqv_a1p0,dqv_a1sc0,mix:2:18:1 > $O/probe_a1buf.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_a1buf.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
