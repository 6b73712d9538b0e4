# round 6: the logdet end-to-end cases on this build (exact-alpha coordinates, every channel's
# sub-tile partials) and on the f74c1be library (exponent correction), and the eta forward A/B
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
run_tests() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/$n.log 2>&1 || { rc=$?; echo "$n rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
  tail -2 $O/$n.log
}
run_tests e2e_logdet 500 tests/test_gpu_e2e_fullsize.py -k logdet
grep "^e2e" $O/e2e_logdet.log || true
export DICP_LIB_PATH=$PWD/diff-icp_amd/variants/libdifficp_hip_fix.so
run_tests e2e_logdet_fix 500 tests/test_gpu_e2e_fullsize.py -k logdet
grep "^e2e" $O/e2e_logdet_fix.log || true
unset DICP_LIB_PATH
DICP_AB_ONLY=fwd_eta,step_eta timeout -k 10 300 python -u tools/ab_libs.py --M 50000 --passes 3 base fix pre > $O/ab_eta.json 2> $O/ab_eta.err
cat $O/ab_eta.json
