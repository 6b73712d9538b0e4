set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/zs0_tests.log 2>&1 || { tail -40 gpurun_out/zs0_tests.log; exit 1; }
tail -1 gpurun_out/zs0_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zs0.json 2> gpurun_out/bench_zs0.err
python -c "
import json
d=json.load(open('gpurun_out/bench_zs0.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], {k:round(v['ms']/v['launches'],3) for k,v in d['kernels'].items()})"
