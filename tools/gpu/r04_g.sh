# round 4, call G: row-split tests (2 ranks with the column phases forced on, async RCCL
# gather), and the 100k two-rank rehearsal with the phases on / default (gloo, one GPU)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rowsplit.py > $O/rowsplit_tests.log 2>&1
tail -3 $O/rowsplit_tests.log
DICP_ROWSPLIT_OVERLAP=1 DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_two_set_w2_overlap.json 2> $O/rehearse_two_set_w2_overlap.err
tail -c 200 $O/rehearse_two_set_w2_overlap.json
DICP_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/rehearse_two_set_w2.json 2> $O/rehearse_two_set_w2.err
tail -c 200 $O/rehearse_two_set_w2.json
echo done
