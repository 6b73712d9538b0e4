set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out


timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/eta_tests.log 2>&1 || { tail -40 gpurun_out/eta_tests.log; exit 1; }
tail -1 gpurun_out/eta_tests.log
timeout -k 10 400 python -u bench.py --workload two_set_50k_exact --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2x.json 2> gpurun_out/bench_c2x.err
python -c "import json; d=json.load(open('gpurun_out/bench_c2x.json')); print(d['value'], d['ms_per_step'], d['kernels'])"
