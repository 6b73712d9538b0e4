# round 4, call H: column groups per workgroup of the 4-row VJP (more repetitions), and a
# rocprofv3 stats pass of the default bench on this box
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
SIZES=70000,100000,140000,200000 REPS=8 ROUNDS=5 LS=0,2,4 timeout -k 10 400 python -u tools/probes/sym_L_rows4.py > $O/sym_L_rows4.jsonl 2> $O/sym_L_rows4.err
cat $O/sym_L_rows4.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
tail -c 200 $O/bench_rocprof.json
echo done
