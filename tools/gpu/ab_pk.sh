export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 2 base pkw4 pku1 pku4 > gpurun_out/ab_pk100k.json 2> gpurun_out/ab_pk.err
