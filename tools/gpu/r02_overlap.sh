set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/mfma_overlap_probe.py > gpurun_out/overlap.log 2>&1
cat gpurun_out/overlap.log
