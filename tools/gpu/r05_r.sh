# round 5: E-step time against sigma (re-reference events); the in-bench kernel-sum probe
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_sigma.py > gpurun_out/r05r_estep_sigma.jsonl 2> gpurun_out/r05r.err
step timeout -k 10 200 python -u tools/probes/sym_red_ab.py 4:0 > gpurun_out/r05r_sym_ab.jsonl 2>> gpurun_out/r05r.err
echo done
