# round 4, call L: the symmetric VJP at 45k-60k with 4 rows per lane and L = 1 / 2 / 4
# against 2 rows (auto), to see whether the 4-row form's loss at 50k is its grid's tail
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
SYM_RP=2 SIZES=46000,50000,52000 REPS=10 ROUNDS=4 LS=1,2,4 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/rows4_L.jsonl 2> $O/rows4_L.err
cat $O/rows4_L.jsonl
SYM_RP=1 SIZES=46000,50000,52000 REPS=10 ROUNDS=4 LS=0 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/rows2.jsonl 2> $O/rows2.err
cat $O/rows2.jsonl
echo done
