# round 6: where the 2k host floor goes (cProfile of one PSR iteration)
set -eo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 200 python -u tools/host_profile.py --N 2000 --top 60 > $O/host_profile_2k.txt 2>&1
timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > $O/host_floor.txt 2>&1
tail -1 $O/host_floor.txt
