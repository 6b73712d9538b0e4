"""FE of the two-set iteration of tests/test_gpu_rowsplit.py::test_rowsplit_two_set_on_gpu on one
device, under environment switches (DICP_DIRECT_LOSSGRAD, ...): which host path moves it.

    python tools/probes/rowsplit_fe.py   (GPU box; prints one JSON line)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from difficp_amd import workloads
    dev = torch.device("cuda:0")
    psr = workloads.build_two_set(3000, dev, seed=4, nt=5)
    fes = [float(psr.FE)]
    psr.GMM_opt(max_iterations=3, tol=1e-6)
    fes.append(float(psr.FE))
    psr.Reg_opt(nmax=1, tol=1e-6) if hasattr(psr, "Reg_opt") else None
    fes.append(float(psr.FE))
    env = {k: v for k, v in os.environ.items() if k.startswith("DICP_")}
    print(json.dumps({"env": env, "FE": fes}), flush=True)


if __name__ == "__main__":
    main()
