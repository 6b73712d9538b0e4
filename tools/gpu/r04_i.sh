# round 4, call I: the 4-row VJP with L = 2 -- parity (forced 4-row forms, full-size end to
# end), the L probe (auto should now equal L = 2 at 70k-100k), the default bench
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pk_rows.py tests/test_gpu_e2e_fullsize.py tests/test_gpu_rowsplit.py > $O/tests.log 2>&1
tail -2 $O/tests.log
SIZES=70000,100000 REPS=8 ROUNDS=5 LS=0,2,4 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/sym_L_rows4.jsonl 2> $O/sym_L_rows4.err
cat $O/sym_L_rows4.jsonl
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
tail -c 200 $O/bench.json
echo done
