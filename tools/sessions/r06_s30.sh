# round 6 session 30: the decode GEMV (NF4DQ_GEMM_GEMV, M = 1) -- its parity test against
# the float64 oracle (x held in registers at K = 4096; rings of 2 and 4 units), then per-launch time against the library's default on the Llama-3-8B
# shapes (single weights and the grouped q/k/v and gate/up column totals).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s30
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py -k "gemv or invalid" -x -q --timeout 120 \
    --timeout-method thread > $O/gemv_test.log 2>&1 || { tail -30 $O/gemv_test.log; exit 1; }
tail -2 $O/gemv_test.log
C="default;7,16,1,1,0;7,16,1,1,4;7,16,2,1,0;7,16,2,1,4;7,16,4,1,0;7,8,1,1,2;7,8,1,1,6;7,8,2,1,2;7,8,2,1,6;7,8,2,1,4;7,8,4,1,2;7,8,4,1,6"
timeout -k 10 600 python3 -u tools/gemm_ab.py --ms 1 --shapes "14336,4096;4096,4096;4096,14336;6144,4096;28672,4096" \
    --cfgs "$C" > $O/gemv_ab.jsonl 2> $O/gemv_ab.err
python3 - "$O/gemv_ab.jsonl" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
for sh in sorted({(r["N"], r["K"]) for r in rows}):
    rs = [r for r in rows if (r["N"], r["K"]) == sh]
    print(sh, [(r["cfg"], r.get("eager_us", r.get("skipped"))) for r in rs])
PY
