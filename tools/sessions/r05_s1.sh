# round 5 session 1: memory-system twins at 4096^2 (streamed), store/load policy sweep,
# table-decode variant A/B, the driver's bench command
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s1
mkdir -p $O
D=tools/_build
timeout -k 10 300 python -u tools/stream_probe.py --tag base --libs $D/libnf4dq_dqv_tbl.so,$D/libnf4dq_dqv_tbl_wg8.so,$D/libnf4dq_dqv_wg8.so --kernels prod,dqv_tbl,dqv_tbl_wg8,dqv_wg8,prod16,mix:2:18:1,rd:2:1,wr:18:1,empty > $O/probe_base.jsonl 2> $O/probe.err
cat $O/probe_base.jsonl
timeout -k 10 300 python -u tools/stream_probe.py --tag wpol --steps 128 --rounds 5 --kernels prod,wr:18:1,wr:2:1,wr:0:1,wr:16:1,wr:19:1,wr:3:1,wr:17:1,wr:1:1,wr:18:2,wr:18:4,rd:2:1,rd:0:1,rd:2:2,rd:2:4,mix:2:18:1,mix:0:18:1,mix:2:2:1,mix:2:0:1,mix:2:16:1,mix:2:19:1,mix:2:3:1,mix:2:17:1,mix:2:18:2,mix:2:18:4 > $O/probe_wpol.jsonl 2>> $O/probe.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench_k20.json'));r=d['roofline'];print(r['launch_us'],r['frac'],r['launch_us_min'],r['launch_us_max'],r['ceiling_measured'])"
