# round 6: the 1024-thread bound pass; EM tests, the headline bench under rocprofv3, and the
# E-step's PMC traffic (unhinted + hinted, as the EM loop runs it)
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py tests/test_gpu_golden.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/em.log 2>&1 || { rc=$?; echo "em rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -2 $O/em.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err
tail -c 150 $O/bench_rocprof.json; echo
PMC_OPS=estep timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o fetch --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_fetch.log 2>&1
PMC_OPS=estep timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- python3 tools/pmc_probe.py > $O/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc > $O/pmc_traffic_estep.json
cat $O/pmc_traffic_estep.json
