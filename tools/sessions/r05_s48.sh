# round 5 session 48: parity sweeps after the past-end-wave fix -- drop-in + misaligned C-ABI
# dequant calls (wide sentinels), the API entries on three seeds
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s48
mkdir -p $O
timeout -k 10 560 python -u tools/fuzz_dequant.py --cases 80000 --seed 67 --seconds 420 --abi-rate 0.5 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
for sd in 71 73 79; do
  timeout -k 10 300 python -u tools/fuzz_api.py --rounds 1500 --seed $sd --seconds 150 > $O/fuzz_api_$sd.jsonl 2>> $O/fuzz.err
  tail -1 $O/fuzz_api_$sd.jsonl
done
