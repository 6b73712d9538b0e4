"""Per-stage float32 drift of the PSR_std support-scheme traces (tests/std_support_case.py)
from the reference's float64 energies (tests/golden/psr_std_support.npz), for the oracle-backed
host logic in float32 with the oracle's kernels in float64 (FAKE_HIP_DTYPE unset) or in float32
(FAKE_HIP_DTYPE=float32: the reference's torch path in float32, SURVEY 8(c)'s oracle32).
CPU only:  FAKE_HIP_DTYPE=float32 python tools/probes/psr_std_fp32_dev.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


class _MP:
    """monkeypatch stand-in for fake_hip.install outside pytest"""
    def setattr(self, obj, name, value, raising=True):
        setattr(obj, name, value)


def main():
    import fake_hip
    import std_support_case as C
    fake_hip.install(_MP())
    for scheme in ("grid", "decim"):
        for weights in (False, True):
            warned = []
            _, Es = C.run({"device": "cpu", "dtype": torch.float32}, scheme, weights, warned)
            ref = C.reference(scheme, weights)
            print(json.dumps({"scheme": scheme, "weights": weights,
                              "kernels": os.environ.get("FAKE_HIP_DTYPE", "float64"),
                              "rel_dev": [abs(a - b) / abs(b) for a, b in zip(Es, ref)],
                              "E": Es, "ref": ref, "warnings": len(warned),
                              "ref_warnings": C.reference_warnings(scheme, weights)}), flush=True)


if __name__ == "__main__":
    main()
