set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fwd or mfma or euler" > gpurun_out/fwd4_tests.log 2>&1 || { tail -40 gpurun_out/fwd4_tests.log; exit 1; }
tail -2 gpurun_out/fwd4_tests.log
timeout -k 10 300 python -u tools/fwd_ab.py > gpurun_out/fwd_ab.log 2>&1
cat gpurun_out/fwd_ab.log
