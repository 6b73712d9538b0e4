# round 6, final build (1/2): the full GPU suite (one process), smoke(), the headline bench with
# the CPU baseline, rocprofv3 kernel stats of the same bench command
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06zz
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { rc=$?; echo "suite rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
echo done
