# round 4, call C: launch batching (dicp_batch_*) parity tests and the atlas with the frames in
# lockstep batches (groups = --concurrent-frames), against the per-frame concurrent streams
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_pk_rows.py -k "batch or sym4" -x -v --timeout 300 --timeout-method thread > $O/batch_tests.log 2>&1
tail -2 $O/batch_tests.log
SIZES=20000,50000,100000,200000 timeout -k 10 300 python -u tools/probes/fwd_sym4_ab.py > $O/fwd_sym4_ab.jsonl 2> $O/fwd_sym4_ab.err
SIZES=100000,200000 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/sym_L_rows4.jsonl 2> $O/sym_L_rows4.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_atlas_shapes.py -x -q --timeout 300 --timeout-method thread > $O/atlas_tests.log 2>&1
tail -2 $O/atlas_tests.log
for cfg in "off 4" "on 1" "on 2" "on 4" "on 8"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --batch-frames $1 --concurrent-frames $2 > $O/c4fixed_$1_$2.json 2> $O/c4fixed_$1_$2.err
  tail -c 300 $O/c4fixed_$1_$2.json
done
timeout -k 10 240 python -u bench.py --workload atlas_c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
echo done
