# round 6: the hinted E-step's stats against float64 rows, sampled vs bound shift
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python -u tools/probes/estep_workload_diff.py > $O/estep_diff.jsonl 2> $O/estep_diff.err
cat $O/estep_diff.jsonl
