# round 4, call A: the new parity tests (4-row VJP, far-extent completion), the VJP regression
# bisect (libraries of earlier commits vs HEAD, one box), the 4-row VJP size sweep incl.
# row-split parts, and 4-row variant builds (scalar column sums, unroll 1, >= 3 waves)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pk_rows.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1
tail -2 $O/new_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_fullsize.py tests/test_gpu_fullsize.py -k "e2e or estep" -x -v -s --timeout 900 --timeout-method thread > $O/e2e_tests.log 2>&1
tail -2 $O/e2e_tests.log
timeout -k 10 500 python -u tools/bisect_vjp.py time --M 100000 --passes 3 c092ecc 73d3f8c~1 73d3f8c cca942e~1 cca942e d93a18f 41216bc HEAD > $O/bisect.jsonl 2> $O/bisect.err
tail -1 $O/bisect.jsonl
SIZES=50000,70000,90000,100000,150000,200000 PARTS=2,4,8 timeout -k 10 400 python -u tools/probes/sym_rp_ab.py > $O/sym_rp_ab.jsonl 2> $O/sym_rp_ab.err
DICP_AB_OPTS=sym_rp=2 timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 3 base rows4sct rows4u1 rows4w3 > $O/ab_rows4_variants.json 2> $O/ab_rows4_variants.err
echo done
