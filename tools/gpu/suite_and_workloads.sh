# full GPU suite, then the secondary workloads' bench lines
export PYTHONUNBUFFERED=1
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload two_set_50k_exact --no-cpu-baseline > gpurun_out/bench_c2x.json 2> gpurun_out/bench_c2x.err
timeout -k 10 300 python -u bench.py --workload two_set_50k --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 300 python -u bench.py --workload atlas_c4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
