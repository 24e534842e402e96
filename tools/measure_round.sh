set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/meas
timeout -k 10 300 python -u bench.py > gpurun_out/meas/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/meas/rocprof -o bench -- python -u bench.py --steps 200 > gpurun_out/meas/bench_rocprof.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/meas/pmc -o fetch -- python -u tools/pmc_probe.py > gpurun_out/meas/pmc_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/meas/pmc -o write -- python -u tools/pmc_probe.py > gpurun_out/meas/pmc_write.log 2>&1
python tools/pmc_traffic.py gpurun_out/meas/pmc gpurun_out/meas/pmc_traffic.json > gpurun_out/meas/pmc_traffic.log 2>&1
timeout -k 10 300 python -u tools/bench_configs.py > gpurun_out/meas/configs.jsonl 2>&1
timeout -k 10 300 python -u tools/hbm_ceiling.py > gpurun_out/meas/hbm_ceiling.jsonl 2>&1
