# round 3: kernel timeline of the headline bench (idle-gap analysis)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r03n
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03n/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03n/bench_rocprof.json 2> gpurun_out/r03n/bench_rocprof.err
echo done
