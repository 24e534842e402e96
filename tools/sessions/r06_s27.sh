# round 6 session 27: persistent-kernel decompositions for the down projection (4096 x 14336,
# K = 14336: 56 chunks) at M = 1 and 8 against the library's default (the 128-deep kernel).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s27
mkdir -p $O
C="default;3,4,2,1,1;3,4,2,1,2;3,4,2,1,4;3,4,2,2,2;3,4,2,2,4;3,4,2,4,4;3,4,2,7,1;3,4,2,7,2;3,4,2,7,4;3,4,2,14,2;3,4,2,14,4;3,4,4,1,2;3,4,4,1,4;3,4,4,2,4;3,4,4,7,2;3,4,4,7,4;3,4,4,14,4;3,8,2,1,2;3,8,2,1,4;3,8,2,2,4;3,8,2,7,2;3,8,2,7,4;3,8,2,14,4;3,8,4,1,4;3,8,4,7,4;3,16,2,1,4;3,16,2,7,4"
timeout -k 10 900 python3 -u tools/gemm_ab.py --ms 1,8 --shapes "4096,14336" --cfgs "$C" > $O/gemm_down_cfgs.jsonl 2> $O/gemm_down_cfgs.err
python3 - "$O/gemm_down_cfgs.jsonl" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
for M in (1, 8):
    rs = sorted([r for r in rows if r.get("M") == M and "eager_us" in r], key=lambda r: r["eager_us"])
    print(M, [(r["cfg"], round(r["eager_us"], 2)) for r in rs[:8]])
PY
