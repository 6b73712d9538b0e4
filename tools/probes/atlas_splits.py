"""Atlas workload with a forced column-split count for the row passes (dicp_set_option
"force_splits"; 0 = automatic): do concurrent frames (4 HIP streams, each kernel a quarter of
the chip) prefer fewer, longer workgroups than the single-kernel split heuristic picks?

    python tools/probes/atlas_splits.py S [bench.py args...]
"""
import os
import sys

sys.path.insert(0, os.getcwd())
S = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
from difficp_amd import _lib  # noqa: E402

_lib.set_option("force_splits", S)
import bench  # noqa: E402

bench.main()
