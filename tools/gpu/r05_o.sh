# round 5: what moves the PSR_std grid trace (host mechanisms switched off one at a time)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
O=gpurun_out/r05o_psr_std.jsonl
: > $O
step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
DICP_WS_NOCACHE=1 step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
DICP_WS_POISON=1 step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
DICP_SHOOT_GRAPH=0 step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
DICP_DIRECT_LOSSGRAD=0 step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
DICP_LSE_PK=0 step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 1 >> $O 2>> gpurun_out/r05o.err
step timeout -k 10 120 python -u tools/probes/psr_std_trace.py grid 0 >> $O 2>> gpurun_out/r05o.err
echo done
