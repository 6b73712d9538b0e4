# round-3 final build: bench lines of the other workloads (one GPU) and the driver-form
# headline (20 steps after 5 warmups)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03fw
mkdir -p $O
timeout -k 10 240 python -u bench.py --workload two_set_50k --steps 5 --warmup 1 --no-cpu-baseline > $O/c2.json 2> $O/c2.err
timeout -k 10 300 python -u bench.py --workload two_set_200k --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --workload two_set_50k_exact --steps 3 --warmup 1 --no-cpu-baseline > $O/c2x.json 2> $O/c2x.err
timeout -k 10 240 python -u bench.py --workload atlas_c4 --steps 5 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
timeout -k 10 300 python -u bench.py --workload atlas_c4_fixed --steps 2 --warmup 1 --no-cpu-baseline > $O/c4f.json 2> $O/c4f.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_form.json 2> $O/driver_form.err
echo done
