# round 6, final build (2/2): the driver-form headline (20 steps after 5 warmups), the PMC
# traffic / issue passes, the secondary workload lines and the host floor
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06zz
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/batch_tests.log 2>&1 || { rc=$?; echo "batch rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -2 $O/batch_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_form.json 2> $O/bench_driver_form.err
tail -c 200 $O/bench_driver_form.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o fetch --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/pmc_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_issue.log 2>&1
python3 tools/pmc_traffic.py $O/pmc > $O/pmc_traffic.json
python3 tools/pmc_issue.py $O/pmc_issue > $O/pmc_issue.json
for w in two_set_50k two_set_50k_exact two_set_100k_2d two_set_200k atlas_c4 atlas_c4_fixed c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err
  tail -c 120 $O/bench_$w.json; echo
done
timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > $O/host_floor.txt 2>&1
echo done2
