# round 4, call J: the symmetric 4-row forward's column groups (L auto / 2 / 4 / 8), and the
# driver-form headline (20 steps after 5 warmups)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
KIND=fwd SIZES=80000,100000,140000,200000 REPS=8 ROUNDS=5 LS=0,2,4,8 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/sym_L_fwd.jsonl 2> $O/sym_L_fwd.err
cat $O/sym_L_fwd.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_form.json 2> $O/bench_driver_form.err
tail -c 200 $O/bench_driver_form.json
echo done
