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
tail -c 400 $O/bench.json
for cfg in "off 4 1" "on 4 1" "on 4 0" "on 2 0" "on 1 0"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --batch-frames $1 --concurrent-frames $2 --batch-share $3 > $O/c4fixed_$1_$2_$3.json 2> $O/c4fixed_$1_$2_$3.err
  tail -c 200 $O/c4fixed_$1_$2_$3.json
done
timeout -k 10 300 python -u bench.py --workload two_set_100k_2d --steps 3 --warmup 1 > $O/bench_2d.json 2> $O/bench_2d.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_two_set_w2.json 2> $O/rehearse_two_set_w2.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --workload atlas_c4_fixed --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_c4fixed_w2.json 2> $O/rehearse_c4fixed_w2.err
echo done
