# round 4, call B: full GPU suite at the 4-row VJP build, headline bench + rocprofv3 stats,
# 2-rank rehearsals through bench.py's own launcher (--gpus 2, no torchrun on the command
# line), the 2D workload, and atlas_c4_fixed under kernel-geometry options
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_two_set_w2.json 2> $O/rehearse_two_set_w2.err
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --workload atlas_c4_fixed --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_c4fixed_w2.json 2> $O/rehearse_c4fixed_w2.err
timeout -k 10 300 python -u bench.py --workload two_set_100k_2d --steps 3 --warmup 1 > $O/bench_2d.json 2> $O/bench_2d.err
for opt in none sym_L=4 pk_rp=2 sym_rp=2; do
  a=""; [ "$opt" != none ] && a="--lib-opt $opt"
  timeout -k 10 200 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --no-profile $a > $O/c4fixed_$opt.json 2> $O/c4fixed_$opt.err
done
echo done
