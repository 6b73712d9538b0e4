# round 6: symmetric forward rows per lane 4 / 6 / 8 (automatic L) against M, and at 100k with
# the 6-row form's L = 2 rule; the E-step tests with the float32-derived tolerance
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
SYMFWD_CFGS="4:0,6:0,6:1,6:2,8:0" timeout -k 10 400 python -u tools/probes/symfwd_L.py 40000 60000 80000 100000 120000 150000 200000 > $O/symfwd_rows.jsonl 2> $O/symfwd_rows.err
cat $O/symfwd_rows.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_em.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/em.log 2>&1 || { rc=$?; echo "em rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -3 $O/em.log
