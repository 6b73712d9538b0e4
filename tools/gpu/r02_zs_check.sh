# divergence-row reuse: full GPU suite (incl. tests/test_gpu_zs.py), kernel A/B, bench with / without
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/zs_tests.log 2>&1 || { tail -40 gpurun_out/zs_tests.log; exit 1; }
tail -1 gpurun_out/zs_tests.log
timeout -k 10 300 python -u tools/zs_ab.py > gpurun_out/zs_ab.json 2> gpurun_out/zs_ab.err
cat gpurun_out/zs_ab.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zs.json 2> gpurun_out/bench_zs.err
DICP_ZS=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nozs.json 2> gpurun_out/bench_nozs.err
python -c "
import json
for f in ('bench_zs','bench_nozs'):
    d=json.load(open('gpurun_out/%s.json'%f)); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
