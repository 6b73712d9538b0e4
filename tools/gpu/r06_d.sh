set -eo pipefail
mkdir -p gpurun_out
O=gpurun_out/r06_rowsplit_fe.jsonl
timeout -k 10 120 python -u tools/probes/rowsplit_fe.py > $O 2> gpurun_out/r06_d.err
DICP_DIRECT_LOSSGRAD=0 timeout -k 10 120 python -u tools/probes/rowsplit_fe.py >> $O 2>> gpurun_out/r06_d.err
DICP_LIB_PATH=$PWD/diff-icp_amd/variants/r05.so timeout -k 10 120 python -u tools/probes/rowsplit_fe.py >> $O 2>> gpurun_out/r06_d.err
DICP_ESTEP_HINT_ANY=1 timeout -k 10 120 python -u tools/probes/rowsplit_fe.py >> $O 2>> gpurun_out/r06_d.err
