# round 5, last build: the full GPU suite (one process), smoke(), the headline bench line
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05zc
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 200 $O/bench.json
echo done
