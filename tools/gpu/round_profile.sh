# headline bench + rocprofv3 kernel-trace stats of the same command + PMC traffic passes
# (separate runs, per MI355X_MICROARCH.md); outputs under gpurun_out/, copied to profiles/ by hand
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_write.log 2>&1
