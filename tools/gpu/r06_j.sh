# round 6 (1/2): eta != 0 forward with exact-alpha coordinates (A/B against the round-5
# library), the 6-row symmetric forward (tests + sym_L sweep at 100k), the E-step's bound shift
# (EM tests + sigma sweep)
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
run_tests() {  # name, timeout, pytest args...: assertion failures (rc 1) are reported, anything else stops
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/$n.log 2>&1 || { rc=$?; echo "$n rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
  tail -2 $O/$n.log
}
run_tests em 400 tests/test_gpu_em.py
timeout -k 10 200 python -u tools/probes/estep_bound.py > $O/estep_bound.jsonl 2> $O/estep_bound.err
cat $O/estep_bound.jsonl
DICP_AB_ONLY=fwd_eta,step_eta timeout -k 10 300 python -u tools/ab_libs.py --M 50000 --passes 3 base pre > $O/ab_eta.json 2> $O/ab_eta.err
cat $O/ab_eta.json
run_tests fwd_rows 400 tests/test_gpu_fwd8.py tests/test_gpu_pk_rows.py
timeout -k 10 300 python -u tools/probes/symfwd_L.py 100000 > $O/symfwd_L.jsonl 2> $O/symfwd_L.err
cat $O/symfwd_L.jsonl
