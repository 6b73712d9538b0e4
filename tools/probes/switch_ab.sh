# A/B of the interpreter's GIL switch interval on the concurrent-frame atlas (C4): default
# 5 ms against 0.5 ms and 0.1 ms, alternating, one GPU
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03sw
mkdir -p $O
for rep in 1 2; do
  for si in 0.005 0.0005 0.0001; do
    timeout -k 10 200 python -u -c "import sys; sys.setswitchinterval($si); import runpy; sys.argv=['bench.py','--workload','atlas_c4','--steps','3','--warmup','1','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > $O/c4_${si}_$rep.json 2> $O/c4_${si}_$rep.err
    python -c "import json; d=json.load(open('$O/c4_${si}_$rep.json')); print('$si', $rep, d['value'], d['ms_per_step'])"
  done
done
