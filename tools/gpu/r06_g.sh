# round 6: eta != 0 forward cost of the double sub-tile totals (32 / 64 / 128 columns against
# the round-5 library "pre"), and the symmetric forward's 4 vs 8 rows at 100k / 120k
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
DICP_AB_ONLY=fwd_eta,step_eta,fwd,step_zs timeout -k 10 300 python -u tools/ab_libs.py --M 50000 --passes 3 base pre f64s64 f64s128 > $O/ab_eta.json 2> $O/ab_eta.err
cat $O/ab_eta.json
timeout -k 10 300 python -u tools/probes/fwd8_ab.py 100000 120000 > $O/fwd8.jsonl 2> $O/fwd8.err
cat $O/fwd8.jsonl
timeout -k 10 300 python -u tools/probes/symfwd_L.py 100000 > $O/symfwd_L.jsonl 2> $O/symfwd_L.err
cat $O/symfwd_L.jsonl
