# round 4, call E: the row split's forward steps in column phases (overlap of the all-gather):
# parity tests, per-rank cost of the phases on one GPU, and the atlas at more concurrent frames
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rowsplit.py > $O/rowsplit_tests.log 2>&1
tail -3 $O/rowsplit_tests.log
timeout -k 10 200 python -u tools/probes/rowsplit_phases.py > $O/rowsplit_phases.jsonl 2> $O/rowsplit_phases.err
cat $O/rowsplit_phases.jsonl
for cfg in "off 8 0" "off 6 0" "off 8 1"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --batch-frames $1 --concurrent-frames $2 --batch-share $3 > $O/c4fixed_$1_$2_$3.json 2> $O/c4fixed_$1_$2_$3.err
  tail -c 300 $O/c4fixed_$1_$2_$3.json | head -c 120; echo
done
echo done
