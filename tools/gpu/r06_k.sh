# round 6 (2/2): the logdet end-to-end and eta parity tests (exact-alpha forward), the EM
# goldens, then the L-BFGS trace parity tests against the float32 envelopes and the HIP path's
# own ensemble over the same 7 float32 realisations
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
run_tests() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/$n.log 2>&1 || { rc=$?; echo "$n rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
  tail -2 $O/$n.log
}
DICP_AB_ONLY=fwd_eta,step_eta timeout -k 10 300 python -u tools/ab_libs.py --M 50000 --passes 3 base pre f64a64 > $O/ab_eta.json 2> $O/ab_eta.err
cat $O/ab_eta.json
run_tests fwd_rows 400 tests/test_gpu_fwd8.py
run_tests e2e_logdet 700 tests/test_gpu_e2e_fullsize.py -k logdet
grep "^e2e" $O/e2e_logdet.log || true
run_tests eta 400 tests/test_gpu_fullsize_eta.py tests/test_gpu_golden.py tests/test_gpu_api.py
run_tests traces 400 tests/test_gpu_support.py tests/test_gpu_multi.py -k "psr_std or multi_structure"
grep -E "^psr_std|^m2d|^m3d" $O/traces.log || true
timeout -k 10 400 python -u tools/probes/fp32_ensemble.py gpu 6 > $O/ensemble_gpu.jsonl 2> $O/ensemble_gpu.err
grep -c '^{' $O/ensemble_gpu.jsonl
