"""Float32 drift envelopes of the L-BFGS-driven traces (VERDICT r05 "What's weak" 1): the
PSR_std support-scheme traces (tests/std_support_case.py) and the multi-structure traces
(tests/multi_case.py) run on float32 realisations of their inputs -- every coordinate moved by
-1 / 0 / +1 float32 ulp (std_support_case.ulp_perturb, seeds 1..R; seed 0 = the inputs as
drawn) -- and compared stage by stage with the reference's float64 goldens.

    FAKE_HIP_DTYPE=float32 python tools/probes/fp32_ensemble.py oracle [R]   # CPU: the float32 oracle
    python tools/probes/fp32_ensemble.py gpu [R]                            # the HIP path

One JSON line per (case, seed): the per-stage relative energy deviations (psr_std) or the
per-(stage, iteration) worst deviation per quantity group (multi), plus the energy-increase
warnings.  The oracle's envelope (max over seeds) is what tests/test_gpu_support.py and
tests/test_gpu_multi.py take 2 x of.
"""
import json
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


class _MP:
    """monkeypatch stand-in for fake_hip.install outside pytest"""
    def setattr(self, obj, name, value, raising=True):
        setattr(obj, name, value)


def main():
    mode = sys.argv[1]
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else None
    if mode == "oracle":
        import fake_hip
        fake_hip.install(_MP())
        dev = "cpu"
    else:
        dev = torch.device("cuda:0")
    spec = {"device": dev, "dtype": torch.float32}
    import multi_case
    import std_support_case as C
    for seed in range(R + 1):
        pert = None if seed == 0 else seed
        for scheme in ("grid", "decim"):
            for weights in (False, True):
                name = f"{scheme}_w{int(weights)}"
                if only and name not in only:
                    continue
                warned = []
                _, Es = C.run(spec, scheme, weights, warned, perturb=pert)
                ref = C.reference(scheme, weights)
                print(json.dumps({"mode": mode, "case": name, "seed": seed,
                                  "rel_dev": [abs(a - b) / abs(b) for a, b in zip(Es, ref)],
                                  "E": Es, "warnings": len(warned),
                                  "ref_warnings": C.reference_warnings(scheme, weights)}), flush=True)
        for case in multi_case.CASES:
            if only and case not in only:
                continue
            rows = {}

            def check(stage, it, PS, z):
                if stage == "init":
                    return
                d = multi_case.deviations(PS, z, case, stage, it)
                g = {}
                for k, v in d.items():
                    gk = multi_case.group(k)
                    g[gk] = max(g.get(gk, 0.0), v)
                rows[f"{stage}{it}"] = g
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                multi_case.run_multi(spec, case, iters=2, check=check, perturb=pert)
            print(json.dumps({"mode": mode, "case": case, "seed": seed, "dev": rows}), flush=True)


if __name__ == "__main__":
    main()
