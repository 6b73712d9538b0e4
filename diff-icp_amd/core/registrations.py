"""Registration facade (mirror of diffICP/core/registrations.py:21-87, LDDMM part)."""
import warnings

import torch

from .LDDMM import LDDMMModel


class Registration:
    def apply(self, X: torch.Tensor):
        pass

    def backward(self, Y: torch.Tensor):
        pass

    def shoot(self, X: torch.Tensor, backward=False):
        pass


class LDDMMRegistration(Registration):
    """Apply the LDDMM diffeomorphism of (q0, a0) to external points (registrations.py:47-87)."""

    def __init__(self, LMi: LDDMMModel, q0: torch.Tensor, a0: torch.Tensor):
        self.LMi = LMi
        self.q0 = q0
        self.a0 = a0

    def shoot(self, X, backward=False, previous_forwardshoot=None):
        if not backward:
            if previous_forwardshoot is not None:
                warnings.warn("variable 'previous_forwardshoot' is useless when backward=False "
                              "[default]", RuntimeWarning)
            return self.LMi.Shoot(self.q0, self.a0, X)
        if previous_forwardshoot is None:
            previous_forwardshoot = self.shoot(None)
        q1k, a1k = previous_forwardshoot[-1][0], previous_forwardshoot[-1][1]
        return self.LMi.Shoot(q1k, -a1k, X)

    def apply(self, X):
        """Y = phi_1(X) = Shoot(q0, a0, X)[-1][3]  (registrations.py:72-77)."""
        return self.shoot(X)[-1][3]

    def backward(self, Y, previous_forwardshoot=None):
        return self.shoot(Y, backward=True, previous_forwardshoot=previous_forwardshoot)[-1][3]
