# round 5 session 55: narrow 16-bit outputs staged as 4-byte pairs when n and the shift are even --
# chunk tests, a misaligned C-ABI sweep, the timing
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s55
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_parity.py tests/test_gpu_strided.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
timeout -k 10 400 python -u tools/fuzz_dequant.py --cases 30000 --seed 97 --seconds 240 --abi-rate 0.7 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
timeout -k 10 300 python -u tools/chunk_ab.py --rounds 7 --cases flat_4096,chunk_4080,pad_4096,unal_4096,chunk_4090,chunk_4095 > $O/chunk_forms.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_forms.jsonl'))]"
