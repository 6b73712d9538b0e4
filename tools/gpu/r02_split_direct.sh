# row split with direct all-gathers: GPU suite, multi-rank rehearsal of the bench (gloo, 1 GPU)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sd_tests.log 2>&1 || { tail -40 gpurun_out/sd_tests.log; exit 1; }
tail -1 gpurun_out/sd_tests.log
bash tools/gpu/rehearse_n.sh
tail -n 2 gpurun_out/rehearse2.err gpurun_out/rehearse4.err
cat gpurun_out/rehearse2.json gpurun_out/rehearse4.json | python -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'): d=json.loads(l); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('parallelism'))"
