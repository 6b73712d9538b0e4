set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/part_timing.py > gpurun_out/part_timing.log 2>&1 || { tail -30 gpurun_out/part_timing.log; exit 1; }
cat gpurun_out/part_timing.log
