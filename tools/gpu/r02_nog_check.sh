set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nog_tests.log 2>&1 || { tail -30 gpurun_out/nog_tests.log; exit 1; }
tail -1 gpurun_out/nog_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nog.json 2> gpurun_out/bench_nog.err
python -c "import json; d=json.load(open('gpurun_out/bench_nog.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernels'])"
