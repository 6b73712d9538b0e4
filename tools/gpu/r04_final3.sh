# round 4, final build (later)
# (the GPU suite ran in call N on this build): the headline bench with the CPU baseline, rocprofv3
# kernel stats of the same command, PMC FETCH/WRITE/issue passes, the driver-form headline
# (20 steps after 5 warmups), and the secondary workload lines
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04z2
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 200 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o fetch --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/pmc_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_issue.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_form.json 2> $O/bench_driver_form.err
tail -c 200 $O/bench_driver_form.json

for w in two_set_50k two_set_50k_exact two_set_100k_2d atlas_c4 atlas_c4_fixed c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err
  tail -c 120 $O/bench_$w.json; echo
done
echo done2
