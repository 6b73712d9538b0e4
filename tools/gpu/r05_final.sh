# round 5, final build (1/2): the full GPU suite (one process), then the headline bench with the
# CPU baseline, rocprofv3 kernel stats of the same bench command, and the driver-form headline
# (20 steps after 5 warmups).  Stops at the first failing step.
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 200 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
echo done
