"""dtype/device "spec" dictionaries (mirror of diffICP/tools/spec.py:24-43).

The hot path runs on a HIP device only; `defspec` is the GPU spec when one is visible.
"""
import torch

cpuspec = {"device": "cpu", "dtype": torch.float32}          # spec.py:24
gpuspec = {"device": "cuda", "dtype": torch.float32}         # spec.py:27 ("cuda" = HIP on ROCm)
use_cuda = torch.cuda.is_available()
defspec = gpuspec if use_cuda else cpuspec                   # spec.py:30-32


def getspec(*T):
    """Common (device, dtype) of the given tensors; ValueError if they differ (spec.py:39-43).
    None entries are ignored."""
    L = [(t.device, t.dtype) for t in T if t is not None]
    if len(set(L)) != 1:
        raise ValueError("the different input tensors to this function should be on the same "
                         "device and use the same dtype !")
    return dict(zip(("device", "dtype"), L[0]))
