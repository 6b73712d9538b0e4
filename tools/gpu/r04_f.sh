# round 4, call F: the two-phase row-split step (parity, per-rank cost), then the GPU suite
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rowsplit.py > $O/rowsplit_tests.log 2>&1
tail -3 $O/rowsplit_tests.log
timeout -k 10 200 python -u tools/probes/rowsplit_phases.py > $O/rowsplit_phases.jsonl 2> $O/rowsplit_phases.err
cat $O/rowsplit_phases.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
tail -3 $O/gpu_suite.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/frame20k -o frame --output-format csv -- python3 -u tools/probes/small_frame_kernels.py > $O/frame20k.log 2>&1
# the concurrent atlas with the 4-row kernels forced (a frame's launch shares the chip with
# the other streams' launches, so the 4-row forms' quarter-size grids leave no tail of their own)
i=0
for opts in "--lib-opt sym_rp=2" "--lib-opt sym_rp=2 --lib-opt fwd_alg=5" "--lib-opt fwd_alg=5"; do
  i=$((i+1))
  timeout -k 10 240 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline --concurrent-frames 4 --batch-share 0 $opts > $O/c4fixed_r4_$i.json 2> $O/c4fixed_r4_$i.err
  tail -c 300 $O/c4fixed_r4_$i.json | head -c 100; echo
done
echo done
