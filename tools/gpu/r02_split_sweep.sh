set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/split_sweep.py > gpurun_out/split_sweep.log 2>&1 || { tail -30 gpurun_out/split_sweep.log; exit 1; }
cat gpurun_out/split_sweep.log
