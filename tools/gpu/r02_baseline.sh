# round-2 baseline on a fresh box: GPU test suite, then a short headline bench
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
