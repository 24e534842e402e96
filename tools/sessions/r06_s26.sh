# round 6 session 26: BASELINE configs on the final tree (c3, c3b, c4, c5, big, odd, the piece
# kernel's forms, bitsandbytes mode; every output verified against the C oracle) and the
# Llama-3-8B decode pass of the fused GEMM at M = 1 / 8 / 32.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s26
mkdir -p $O
timeout -k 10 900 python3 -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); print(d['config'], d.get('out_dtype'), round(d.get('us_per_launch', d.get('us_per_pass', 0)), 2), round(d.get('frac', 0), 4), d.get('verified'))"
timeout -k 10 600 python3 -u tools/bench_gemm.py --ms 1,8,32 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err
cat $O/bench_gemm.jsonl
