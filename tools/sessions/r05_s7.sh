# round 5 session 7: cache policy of the scale gathers (absmax byte / nested absmax) x store policy
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s7
mkdir -p $O
D=tools/_build
L=""; K="prod"
for v in a1nt a1sc1 a1sc0 a1p0 a1nt_st2 a1sc1_st2 a2nt; do L="$L,$D/libnf4dq_dqv_$v.so"; K="$K,dqv_$v"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag scalepol --steps 20,128 --rounds 7 --libs ${L#,} --kernels $K,mix:2:18:1,mix:2:2:1 > $O/probe_scalepol.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_scalepol.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "error_word or check_gemm or round4" > $O/gemm_err_tests.log 2>&1 || { tail -30 $O/gemm_err_tests.log; exit 1; }
tail -2 $O/gemm_err_tests.log
