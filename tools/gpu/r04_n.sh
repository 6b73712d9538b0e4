# round 4, call N: the symmetric 4-row forward from 20k (tail-aware column groups) -- full GPU
# suite, the forward against the ordered pass under the automatic rule, the default / 50k lines
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
tail -2 $O/gpu_suite.log
SIZES=20000,30000,40000,50000,60000,80000,100000 timeout -k 10 300 python -u tools/probes/fwd_sym4_ab.py > $O/fwd_sym4_ab.jsonl 2> $O/fwd_sym4_ab.err
cut -c1-300 $O/fwd_sym4_ab.jsonl
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
tail -c 150 $O/bench.json
timeout -k 10 300 python -u bench.py --workload two_set_50k --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_50k.json 2> $O/bench_50k.err
tail -c 150 $O/bench_50k.json
echo done
