# round 6: the bound shift on hinted E-steps only: EM tests, the sigma sweep, the hinted
# E-step against the sampled shift on the exact workload's points, the exact two-set line
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py tests/test_gpu_golden.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/em.log 2>&1 || { rc=$?; echo "em rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -2 $O/em.log
timeout -k 10 200 python -u tools/probes/estep_bound.py > $O/estep_bound.jsonl 2> $O/estep_bound.err
cat $O/estep_bound.jsonl
timeout -k 10 300 python -u tools/probes/estep_workload_diff.py > $O/estep_diff.jsonl 2> $O/estep_diff.err
cat $O/estep_diff.jsonl
timeout -k 10 300 python -u bench.py --workload two_set_50k_exact --steps 3 --warmup 1 --no-cpu-baseline > $O/exact.json 2> $O/exact.err
grep "FE=\|NaN" $O/exact.err || true
tail -c 200 $O/exact.json; echo
