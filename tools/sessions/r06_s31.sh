# round 6 session 31: the decode GEMV as the library's choice at M = 1 (launches of up to
# 4096 columns) -- the GEMM test files (parity vs the float64 oracle, red zones, concurrent
# streams), per-launch time of the library's choice against the persistent kernel named
# explicitly, and the Llama-3-8B decode pass at M = 1 / 8 / 32.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s31
mkdir -p $O
bash tools/session.sh r06_s31 gemmtest
C="default;3,8,2,1,1;7,16,1,1,0"
timeout -k 10 600 python3 -u tools/gemm_ab.py --ms 1 --shapes "4096,4096;4096,14336;1024,4096;2048,4096" \
    --cfgs "$C" > $O/gemv_default_ab.jsonl 2> $O/gemv_default_ab.err
python3 - "$O/gemv_default_ab.jsonl" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
for sh in sorted({(r["N"], r["K"]) for r in rows}):
    print(sh, [(r["cfg"], r.get("eager_us", r.get("skipped"))) for r in rows if (r["N"], r["K"]) == sh])
PY
timeout -k 10 600 python3 -u tools/bench_gemm.py --ms 1,8,32 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err
cat $O/bench_gemm.jsonl
