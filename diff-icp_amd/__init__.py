"""difficp_amd -- MI355X (gfx950) native hot path of diff-ICP.

Drop-in counterparts of the reference package's hot-path API (diffICP, AdrienWohrer/diff-icp):
    tools.kernel.GaussKernel        (diffICP/tools/kernel.py)
    core.LDDMM.LDDMMModel           (diffICP/core/LDDMM.py)
    core.GMM.GaussianMixtureUnif    (diffICP/core/GMM.py)
    core.PSR.MultiPSR / DiffPSR     (diffICP/core/PSR.py)
    core.registrations.LDDMMRegistration (diffICP/core/registrations.py)
backed by hand-written HIP kernels in libdifficp_hip.so (C-ABI: include/difficp_hip.h).
The package directory is `diff-icp_amd/`; it is importable as `difficp_amd` (repo-root
symlink) or through `difficp_amd.load()` semantics in bench/tests.
"""
__version__ = "0.1.0"
