# round 4, final build (2/2): the secondary workload lines
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_default_agg.json 2> $O/bench_default_agg.err
tail -c 150 $O/bench_default_agg.json
for w in two_set_50k two_set_200k two_set_50k_exact two_set_100k_2d atlas_c4 atlas_c4_fixed c5; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err
  tail -c 150 $O/bench_$w.json
done
echo done
