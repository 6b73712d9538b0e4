# MFMA forward: kernel parity tests, then a per-kernel timing A/B (fwd_alg 2 vs 3)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "fwd or mfma or euler or shoot or empty" > gpurun_out/mfma_tests.log 2>&1 || { tail -40 gpurun_out/mfma_tests.log; exit 1; }
tail -3 gpurun_out/mfma_tests.log
timeout -k 10 300 python -u tools/fwd_ab.py > gpurun_out/fwd_ab.log 2>&1
cat gpurun_out/fwd_ab.log
