# round 4, call O: L = 1 for the 4-row VJP at 90k-120k (the tail model's favourite there)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
SIZES=90000,100000,120000 REPS=8 ROUNDS=5 LS=1,2 timeout -k 10 300 python -u tools/probes/sym_L_rows4.py > $O/vjp_L12.jsonl 2> $O/vjp_L12.err
cat $O/vjp_L12.jsonl
echo done
