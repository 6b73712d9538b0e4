# round 6: eta != 0 forward with exact-alpha coordinates (no exponent correction in the pair
# loop): A/B against the round-5 library, the logdet end-to-end and eta parity tests; then the
# L-BFGS trace parity tests against the float32 envelopes and the HIP path's own ensemble
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
DICP_AB_ONLY=fwd_eta,step_eta timeout -k 10 300 python -u tools/ab_libs.py --M 50000 --passes 3 base pre f64s64 > $O/ab_eta.json 2> $O/ab_eta.err
cat $O/ab_eta.json
run_tests() {  # name, timeout, pytest args...: assertion failures (rc 1) are reported, anything else stops
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/$n.log 2>&1 || { rc=$?; echo "$n rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
  tail -2 $O/$n.log
}
run_tests fwd_rows 600 tests/test_gpu_fwd8.py tests/test_gpu_pk_rows.py
timeout -k 10 300 python -u tools/probes/symfwd_L.py 100000 > $O/symfwd_L.jsonl 2> $O/symfwd_L.err
cat $O/symfwd_L.jsonl
run_tests e2e_logdet 900 tests/test_gpu_e2e_fullsize.py -k logdet
grep "^e2e" $O/e2e_logdet.log || true
run_tests eta 600 tests/test_gpu_fullsize_eta.py tests/test_gpu_golden.py tests/test_gpu_api.py
run_tests traces 600 tests/test_gpu_support.py tests/test_gpu_multi.py -k "psr_std or multi_structure"
grep -E "^psr_std|^m2d|^m3d" $O/traces.log || true
timeout -k 10 600 python -u tools/probes/fp32_ensemble.py gpu 6 > $O/ensemble_gpu.jsonl 2> $O/ensemble_gpu.err
grep -c '^{' $O/ensemble_gpu.jsonl
