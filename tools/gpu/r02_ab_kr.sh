set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 3 base kr1 kr4 > gpurun_out/ab_kr100k.json 2> gpurun_out/ab_kr.err
cat gpurun_out/ab_kr100k.json
