# round 5 session 15: store policy at large launches (8192^2, 16384x8192): the product's
# sc1+nt vs nt-only / sc0+nt stores, and the twins
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s15
mkdir -p $O
D=tools/_build
L="$D/libnf4dq_dqv_tbl_st2.so,$D/libnf4dq_dqv_tbl_st3.so"
for sh in 8192x8192 16384x8192; do
  timeout -k 10 400 python -u tools/stream_probe.py --tag big --shape $sh --steps 32 --rounds 7 --libs $L --kernels prod,dqv_tbl_st2,dqv_tbl_st3,mix:2:18:1,mix:2:2:1,mix:2:3:1 >> $O/probe_big.jsonl 2>> $O/probe.err
done
python -c "
import json
for l in open('$O/probe_big.jsonl'):
    d=json.loads(l); print(d['m'], d['n'], d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['dequant_frac_at_this_time'], d['checked'])
"
