# round 4, call K: 2 vs 4 rows per lane for the symmetric VJP around the size threshold, now
# that the 4-row form takes L = 2 (the rule picks 4 rows from 64k)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
SIZES=40000,50000,56000,64000,80000 timeout -k 10 300 python -u tools/probes/sym_rp_ab.py > $O/sym_rp_ab.jsonl 2> $O/sym_rp_ab.err
cat $O/sym_rp_ab.jsonl | cut -c1-400
echo done
