# round 6: the exact two-set line (eta != 0) with the E-step's bound shift off / on: FE trace,
# closure counts (a NaN line-search loss appeared with the bound shift on)
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
for b in 0 1; do
  DICP_LSE_BOUND=$b timeout -k 10 300 python -u bench.py --workload two_set_50k_exact --steps 3 --warmup 1 --no-cpu-baseline > $O/exact_b$b.json 2> $O/exact_b$b.err
  grep "FE=\|NaN" $O/exact_b$b.err || true
  tail -c 200 $O/exact_b$b.json; echo
done
DICP_LSE_BOUND=1 timeout -k 10 300 python -u tools/probes/estep_workload_diff.py > $O/estep_diff.jsonl 2> $O/estep_diff.err
cat $O/estep_diff.jsonl
