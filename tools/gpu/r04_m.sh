# round 4, call M: 4 rows per lane for whole VJP passes from 40k with the tail-aware L --
# parity, the automatic rule against forced 2 rows, the C2 (50k) line
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pk_rows.py tests/test_gpu_e2e_fullsize.py > $O/tests.log 2>&1
tail -2 $O/tests.log
SIZES=36000,40000,46000,50000,52000,60000,70000,100000 timeout -k 10 300 python -u tools/probes/sym_rp_ab.py > $O/sym_rp_ab.jsonl 2> $O/sym_rp_ab.err
cut -c1-260 $O/sym_rp_ab.jsonl
timeout -k 10 300 python -u bench.py --workload two_set_50k --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_50k.json 2> $O/bench_50k.err
tail -c 200 $O/bench_50k.json
FWD_ALG=5 KIND=fwd SIZES=20000,40000,50000,60000,80000 REPS=10 ROUNDS=4 LS=1,2,4 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/fwd4_L.jsonl 2> $O/fwd4_L.err
cat $O/fwd4_L.jsonl
FWD_ALG=6 KIND=fwd SIZES=20000,40000,50000,60000,80000 REPS=10 ROUNDS=4 LS=0 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/fwd_ordered.jsonl 2> $O/fwd_ordered.err
cat $O/fwd_ordered.jsonl
echo done
