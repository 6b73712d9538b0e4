# round-2 bench lines of the other workloads at the final build (one GPU)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --workload two_set_50k --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c2.json 2> gpurun_out/c2.err
timeout -k 10 300 python -u bench.py --workload two_set_200k --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c3.json 2> gpurun_out/c3.err
timeout -k 10 240 python -u bench.py --workload two_set_50k_exact --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c2x.json 2> gpurun_out/c2x.err
timeout -k 10 240 python -u bench.py --workload atlas_c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err
echo done
