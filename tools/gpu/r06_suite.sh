# full GPU test suite (one process, no -x: every failure listed), log under gpurun_out/
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_suite.log 2>&1
