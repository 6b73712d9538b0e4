# round 6: validate HEAD after the eta != 0 forward rework: full GPU suite (no -x), smoke,
# the headline bench and the exact two-set line
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || true
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
timeout -k 10 300 python -u bench.py --workload two_set_50k_exact --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_exact.json 2> $O/bench_exact.err
tail -c 200 $O/bench_exact.json
