# round 5 session 2: table decode x store policy variants of the flat kernel, nt-only-store
# twins, the empty launch by grid size
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s2
mkdir -p $O
D=tools/_build
L=""
for v in st2 st3 tbl tbl_st2 tbl_st3 tbl_st2_wg8 tbl_st2_u8 tbl_st2_u2; do L="$L,$D/libnf4dq_dqv_$v.so"; done
timeout -k 10 400 python -u tools/stream_probe.py --tag dec --libs ${L#,} --kernels prod,dqv_st2,dqv_st3,dqv_tbl,dqv_tbl_st2,dqv_tbl_st3,dqv_tbl_st2_wg8,dqv_tbl_st2_u8,dqv_tbl_st2_u2,prod16,dqv_tbl_st2@16,mix:2:18:1,mix:2:2:1,mix:2:3:1,mix:2:2:2,mix:2:2:4,mix:2:3:2,mix:0:2:1,wr:2:2,wr:2:4 > $O/probe_dec.jsonl 2> $O/probe.err
python -c "
import json
for l in open('$O/probe_dec.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'], d['checked'])
"
timeout -k 10 300 python -u tools/stream_probe.py --tag grid --steps 20,128 --rounds 5 --kernels empty,emptydiv:2,emptydiv:4,emptydiv:8,emptydiv:16,empty1 > $O/probe_grid.jsonl 2>> $O/probe.err
python -c "
import json
for l in open('$O/probe_grid.jsonl'):
    d=json.loads(l); print(d['kernel'], d['steps'], d['us_median'], d['us_min'], d['us_max'])
"
