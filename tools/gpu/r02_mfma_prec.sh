set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mfma_precision.py > gpurun_out/mfma_prec.log 2>&1
cat gpurun_out/mfma_prec.log
timeout -k 10 300 python -u tools/fwd_ab.py > gpurun_out/fwd_ab.log 2>&1
cat gpurun_out/fwd_ab.log
