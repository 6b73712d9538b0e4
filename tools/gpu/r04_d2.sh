# round 4, call D2: the atlas under per-frame streams with the kernel-geometry hint (as alone /
# sized for the concurrent frames) and in lockstep batches, the 2D line, and the 2-rank
# rehearsals through bench.py's own launcher (gloo, both ranks on cuda:0)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
for cfg in "off 4 1" "off 4 0" "off 4 2" "on 4 1" "on 1 1" "on 1 0" "on 4 0"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --batch-frames $1 --concurrent-frames $2 --batch-share $3 > $O/c4fixed_$1_$2_$3.json 2> $O/c4fixed_$1_$2_$3.err
  tail -c 200 $O/c4fixed_$1_$2_$3.json
done
timeout -k 10 300 python -u bench.py --workload two_set_100k_2d --steps 3 --warmup 1 > $O/bench_2d.json 2> $O/bench_2d.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_two_set_w2.json 2> $O/rehearse_two_set_w2.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --workload atlas_c4_fixed --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_c4fixed_w2.json 2> $O/rehearse_c4fixed_w2.err
echo done
