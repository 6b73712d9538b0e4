# round 4: the driver's smoke entry on the final build
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r04s
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04s/smoke.log 2>&1
tail -3 gpurun_out/r04s/smoke.log
