# round 4, call D: full GPU suite, headline bench + rocprofv3 stats, 2D line, rehearsals
# through bench.py's own launcher, and the atlas with lockstep batches (geometry as alone /
# sized for the group) against per-frame streams
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --lib-opt fwd_alg=6 > $O/bench_fwd6.json 2> $O/bench_fwd6.err
tail -c 300 $O/bench_fwd6.json
echo done
