# round 6: the L-BFGS trace parity tests against the float32 drift envelopes (PSR_std support
# schemes, multi-structure) and the HIP path's own spread over the same 7 float32 realisations
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_support.py tests/test_gpu_multi.py -k "psr_std or multi_structure" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
tail -5 $O/tests.log
timeout -k 10 600 python -u tools/probes/fp32_ensemble.py gpu 6 > $O/ensemble_gpu.jsonl 2> $O/ensemble_gpu.err
grep -c '^{' $O/ensemble_gpu.jsonl
