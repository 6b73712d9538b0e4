"""diff-ICP point-set registration driver (mirror of diffICP/core/PSR.py MultiPSR :42-346 and
DiffPSR :354-569), the caller of the HIP hot path.

Same attributes (x0, x1, y, N, GMMi, LMi, q0, a0, allx0, Cfe, regloss, quadloss, FE, shoot)
and methods (reinitialize_GMM, update_GMM_targets, update_quadloss, update_FE, GMM_opt,
Reg_opt, Registration, initialize_a0, update_a0, set_support_scheme, QuadLossFunctor).

MI355X addition -- frame sharding (`comm`): with a torch.distributed group of W ranks
(one process per GPU, RCCL over xGMI), rank r owns the frames {k : k mod W == r}.
Reg_opt runs only the local frames (no communication: each frame's L-BFGS is
independent, PSR.py:528-569); GMM_opt runs EM on the local points and exchanges the
per-component sufficient statistics (see core/GMM.py), so every rank holds the same GMM;
free-energy bookkeeping sums regloss / quadloss across ranks.  Frames not owned by a rank
keep their initial values there (x1, y, a0 are only meaningful on the owning rank).
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from .GMM import GaussianMixtureUnif, _comm_active, _gather_rows, _sum_ranks
from .LDDMM import LDDMMModel
from .registrations import LDDMMRegistration
from ..tools.in_out import read_point_sets
from ..tools.spec import defspec
from .support import decimated_points, grid_points, merged_v2p_args, warn_uncovered


def _rank_world(comm):
    if not _comm_active(comm):
        return 0, 1
    import torch.distributed as dist
    g = None if comm is True else comm
    return dist.get_rank(g), dist.get_world_size(g)


class MultiPSR:

    def __init__(self, x, GMMi, dataspec=defspec, compspec=defspec, comm=None):
        self.dataspec, self.compspec = dataspec, compspec
        self.printstuff = True
        self.comm = comm
        self.rank, self.world = _rank_world(comm)
        x, self.K, self.S, self.D = read_point_sets(x)
        # local frames of this rank (all frames when not sharded)
        self.frames = [k for k in range(self.K) if k % self.world == self.rank]
        self.x0 = np.empty((self.K, self.S), dtype=object)
        self.x1 = np.empty((self.K, self.S), dtype=object)
        self.y = np.empty((self.K, self.S), dtype=object)
        for k in range(self.K):
            for s in range(self.S):
                self.x0[k, s] = x[k][s].contiguous().detach().to(**self.dataspec)
                self.x1[k, s] = self.x0[k, s].clone()
                self.y[k, s] = self.x0[k, s].clone()
        self.N = np.array([[self.x0[k, s].shape[0] for s in range(self.S)] for k in range(self.K)])

        if isinstance(GMMi, GaussianMixtureUnif):
            self.GMMi = [copy.deepcopy(GMMi) for _ in range(self.S)]
        else:
            if not isinstance(GMMi, list) or len(GMMi) != self.S:
                raise ValueError("GMMi should be a single GMM model, or a list with S GMM models")
            self.GMMi = [copy.deepcopy(g) for g in GMMi]
        if any(g.spec != compspec for g in self.GMMi):
            raise ValueError("Spec (dtype+device) error : GMM 'spec' and multiPSR 'compspec' "
                             "attributes should be the same")
        for g in self.GMMi:
            g.comm = comm if self.world > 1 else None

        self.Cfe = [None] * self.S
        self.regloss = [0] * self.K
        self.quadloss = np.zeros((self.K, self.S))
        self.FE = None
        self.update_GMM_targets()
        self.shoot = [None] * self.K

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.dataspec = defspec
        self.compspec = defspec

    # ------------------------------------------------------------------------------------
    def _local_cat(self, arr, s):
        parts = tuple(arr[k, s] for k in self.frames)
        if len(parts) == 0:
            return torch.empty((0, self.D), **self.compspec)
        return torch.cat(parts, dim=0).to(**self.compspec)

    def reinitialize_GMM(self, s=None, do_mu=True, do_sigma=True):
        """mu = mean + 0.05 std randn, sigma = 0.25 std over all unwarped points (PSR.py:143-167).
        Sharded: global mean/std from per-rank sums; the randn draw is made on rank 0's
        stream of numbers and shared, so all ranks hold the same centroids."""
        slist = range(self.S) if s is None else [s]
        for s in slist:
            if self.world == 1:
                allx0s = torch.cat(tuple(self.x0[:, s]), dim=0)
                mean, std = allx0s.mean(dim=0), allx0s.std()
            else:
                parts = tuple(self.x0[k, s] for k in self.frames)
                # a rank may own no frames (K < world): it contributes zero sums
                loc = (torch.cat(parts, dim=0) if parts else
                       torch.empty((0, self.D), **self.dataspec)).double()
                n = _sum_ranks(float(loc.shape[0]), self.comm).item()
                s1 = _gather_rows(loc.sum(0).to(**self.compspec).double(), self.comm).sum(0)
                s2 = _sum_ranks((loc ** 2).sum().to(self.compspec["device"]), self.comm)
                mean = (s1 / n)
                ntot = n * self.D
                tot1 = s1.sum()
                std = torch.sqrt((s2 - tot1 ** 2 / ntot) / (ntot - 1))
                mean = mean.to(**self.dataspec)
                std = std.to(**self.dataspec)
            g = self.GMMi[s]
            if do_mu and g.to_optimize["mu"]:
                noise = torch.randn(g.C, self.D, **self.dataspec)
                if self.world > 1:
                    import torch.distributed as dist
                    nz = noise.to(self.compspec["device"])
                    dist.broadcast(nz, 0, group=None if self.comm is True else self.comm)
                    noise = nz.to(**self.dataspec)
                g.mu = (mean + 0.05 * std * noise).to(**self.compspec)
            if do_sigma and g.to_optimize["sigma"]:
                g.sigma = 0.25 * float(std)
        self.update_GMM_targets()

    def get_data_points(self, k=0, s=0):
        return self.x0[k, s]

    def get_warped_data_points(self, k=0, s=0):
        return self.x1[k, s]

    def get_template(self, s=0):
        return self.GMMi[s].mu

    # ------------------------------------------------------------------------------------
    def _assign_targets(self, s, allys):
        last = 0
        for k in self.frames:
            first, last = last, last + int(self.N[k, s])
            self.y[k, s] = allys[first:last].to(**self.dataspec)
            self.update_quadloss(k, s)

    def _row_split(self):
        """The LDDMM model's row split (core/rowsplit.py) when this PSR is not frame-sharded:
        the EM passes are then split over the same ranks by rows of the (warped) points."""
        split = getattr(getattr(self, "LMi", None), "row_split", None)
        return split if (split is not None and self.world == 1) else None

    def _em_rows(self, s, allx1s, fn):
        """Run fn(GMM, X) on this rank's row slice of X with the GMM's cross-rank statistics
        exchange switched on (the atlas code path, GMM.py comm), then all-gather the targets.
        Returns (Y (N, D), *rest of fn's result)."""
        split = self._row_split()
        if split is None:
            return fn(self.GMMi[s], allx1s)
        N = allx1s.shape[0]
        r0, n, _ = split.rows(N)
        g = self.GMMi[s]
        old = g.comm
        g.comm = True if split.group is None else split.group
        try:
            out = fn(g, allx1s[r0:r0 + n].contiguous())
        finally:
            g.comm = old
        (Y,), _ = split.gather_rows([out[0]], N)
        return (Y.contiguous(),) + tuple(out[1:])

    def update_GMM_targets(self):
        """y, Cfe, quadloss, FE from an E-step without parameter update (PSR.py:197-213)."""
        for s in range(self.S):
            allx1s = self._local_cat(self.x1, s)
            allys, self.Cfe[s], _ = self._em_rows(s, allx1s, lambda g, X: g.EM_step(X, skip_M=True))
            self._assign_targets(s, allys)
        self.update_FE()

    def update_quadloss(self, k, s):
        """quadloss[k,s] = |x1 - y|^2 / (2 sigma_s^2)  (PSR.py:217-222)."""
        self.quadloss[k, s] = ((self.x1[k, s] - self.y[k, s]) ** 2).sum() / (2 * self.GMMi[s].sigma ** 2)

    def update_FE(self, message=None):
        """FE = sum Cfe + sum regloss + sum quadloss (PSR.py:226-236); global when sharded."""
        local_reg = sum(float(self.regloss[k]) for k in self.frames)
        local_quad = float(sum(self.quadloss[k, s] for k in self.frames for s in range(self.S)))
        if self.world > 1:
            dev = self.compspec["device"]
            local_reg = float(_sum_ranks(torch.tensor(local_reg, device=dev), self.comm))
            local_quad = float(_sum_ranks(torch.tensor(local_quad, device=dev), self.comm))
        FE = float(sum(float(c) for c in self.Cfe)) + local_reg + local_quad
        if self.printstuff and message is not None and self.rank == 0:
            print(message.ljust(70) + f"Total free energy = {FE:.8}")
        if self.FE is not None and FE > self.FE and self.rank == 0:
            print("WARNING: measured increase in free energy ! Should not happen.")
        self.FE = FE

    def GMM_opt(self, max_iterations=100, tol=1e-5):
        """EM per structure on all (local) warped points, then targets back per frame
        (PSR.py:242-271)."""
        for s in range(self.S):
            allx1s = self._local_cat(self.x1, s)
            allys, self.Cfe[s], _, i = self._em_rows(
                s, allx1s, lambda g, X: g.EM_optimization(X, max_iterations=max_iterations, tol=tol))
            self._assign_targets(s, allys)
            message = f"GMM optim (structure {s}) : {i} EM steps"
            if self.GMMi[s].outliers:
                p0 = 1 / (1 + np.exp(-self.GMMi[s].outliers["eta0"]))
                message += f", p_outlier={p0:.4}"
            else:
                message += "."
            self.update_FE(message=message)

    def Reg_opt(self, tol=1e-5):
        raise NotImplementedError("function Reg_opt must be written in derived classes.")

    def Registration(self, k=0):
        if isinstance(self, DiffPSR):
            return LDDMMRegistration(self.LMi, self.q0[k], self.a0[k])
        raise NotImplementedError


class DiffPSR(MultiPSR):
    """MultiPSR with LDDMM registrations (PSR.py:354-569)."""

    def __init__(self, x, GMMi, LMi: LDDMMModel, dataspec=defspec, compspec=defspec, comm=None,
                 v2p_args=None):
        """v2p_args (extension, default None = the reference's v2p defaults): keyword arguments
        of every v2p call made by initialize_a0 / update_a0 when the caller gives none, e.g.
        {"version": "ridge_keops", "alpha": 1e-3} -- the alternative PSR.py:402 leaves
        commented out, which is the only one that scales to 50k+ support points (device CG)."""
        super().__init__(x, GMMi, dataspec=dataspec, compspec=compspec, comm=comm)
        self.v2p_args = dict(v2p_args or {})
        if LMi.Kernel.spec != compspec:
            raise ValueError("Spec (dtype+device) error : LDDMMmodel kernel 'spec' and diffPSR "
                             "'compspec' attributes should be the same")
        self.LMi = LMi
        self.allx0 = [None] * self.K
        for k in range(self.K):
            self.allx0[k] = torch.cat(tuple(self.x0[k, :]), dim=0).to(**self.compspec).contiguous()
        self.support_scheme, self.rho = None, None
        self.q0 = self.allx0
        self.a0 = [None] * self.K
        self.concurrent_frames = None   # Reg_opt host threads / HIP streams (None = automatic)
        self.batch_frames = None        # Reg_opt lockstep launch batches (opt-in: True)
        # the frames' kernel geometry (library hint "batch_share"): 0 (default) = each launch
        # sized for its share of the chip -- the concurrent frames (1 when the frames run one
        # after another) or the frames per batch group -- which picks the 4-row kernels for
        # 20k frames on 4 streams (csrc/lddmm_sym.hpp DICP_SYM_SHARE4_MIN_PAIRS); 1 = each
        # launch sized as if alone; n = for 1/n of the chip, in every mode (a sequential run
        # with n equal to the concurrent frames gives their bits: the geometry, not the
        # concurrency, decides the fp32 summation order)
        self.batch_share = 0
        self.initialize_a0()

    def initialize_a0(self, **v2p_args):
        """a0 giving zero initial speeds (PSR.py:406-413)."""
        v2p_args = v2p_args or self.v2p_args
        for k in range(self.K):
            v0 = torch.zeros(self.q0[k].shape, **self.compspec)
            self.a0[k] = self.LMi.v2p(self.q0[k], v0, **v2p_args)

    def update_a0(self, q0_prev, a0_prev=None, **v2p_args):
        """Momenta on the current support giving the previous velocity field (PSR.py:415-425)."""
        v2p_args = merged_v2p_args(self.v2p_args, v2p_args)
        if a0_prev is None:
            a0_prev = self.a0
        for k in range(self.K):
            v0 = self.LMi.v(self.q0[k], q0_prev[k], a0_prev[k])
            self.a0[k] = self.LMi.v2p(self.q0[k], v0, **v2p_args)

    def set_support_scheme(self, scheme="decim", rho=1.0, xticks=None, yticks=None, q0=None, zticks=None):
        """Support points (PSR.py:430-493): "decim" (greedy covering decimation of each
        structure, point_sets.py:102-133, device kernels), "grid" (the reference's 2D grid, and
        its 3D extension: core/support.py grid_points; zticks for the third axis) or "custom"
        (:484-487)."""
        self.rho = rho
        Rcover = rho * self.LMi.Kernel.sigma
        self.support_scheme = scheme
        q0_prev = self.q0
        if scheme == "grid":
            ticks = (xticks, yticks) if self.D == 2 else (xticks, yticks, zticks)
            self.q0 = [grid_points(self.allx0, Rcover, self.D, self.compspec, ticks)] * self.K
        elif scheme == "custom":
            assert q0 is not None, "For a custom support scheme, please specify argument q0"
            self.q0 = [q0.clone().detach().to(**self.compspec).contiguous()] * self.K
        elif scheme == "decim":
            # greedy covering decimation of every structure (PSR.py:458-470), on the device
            self.supp_ids = np.array([[None] * self.S] * self.K, dtype=object)
            self.q0 = [None] * self.K
            for k in range(self.K):
                self.q0[k], ids = decimated_points(list(self.x0[k, :]), Rcover, self.compspec)
                for s in range(self.S):
                    self.supp_ids[k, s] = ids[s]
                if self.printstuff:
                    Ndecim = self.q0[k].shape[0]
                    Pdecim = Ndecim / sum(int(self.N[k, s]) for s in range(self.S))
                    print(f"Decimation, frame {k} : {Ndecim} support points ({Pdecim:.0%} of original sets)")
        else:
            raise ValueError(f"Unknown value of support point scheme : {scheme}.")
        self.update_a0(q0_prev, rcond=1e-1)

    def QuadLossFunctor(self, k):
        """dataloss(x) = sum (x - y)^2 / (2 sigma_s^2) over frame k (PSR.py:498-516)."""
        y = torch.cat(tuple(self.y[k, :]), dim=0).to(**self.compspec).contiguous()
        sig2 = torch.cat(tuple(self.GMMi[s].sigma ** 2 * torch.ones(int(self.N[k, s]))
                               for s in range(self.S))).to(**self.compspec).contiguous()

        s2x = 2 * sig2[:, None]

        def dataloss_func(x):
            return ((x - y) ** 2 / s2x).sum()

        # the value and dL/dx without autograd (core/shooting.py shoot_loss_grad): the bits
        # autograd forms -- DivBackward 1/s2x, PowBackward (1/s2x) * (2 (x - y)) -- with the
        # forward's own ops for the value (tests/test_gpu_host_floor.py: bitwise)
        inv = torch.ones_like(s2x).div(s2x)

        def value_and_grad(x):
            if y.requires_grad or s2x.requires_grad:
                return None     # gradients into y / sigma: the autograd path
            d = x - y
            return (d ** 2 / s2x).sum(), inv * (2.0 * d)
        dataloss_func.value_and_grad = value_and_grad
        return dataloss_func

    def _optimize_frame(self, k, nmax, tol):
        if self.support_scheme is None:
            return self.LMi.Optimize(self.QuadLossFunctor(k), self.q0[k], self.a0[k], tol=tol, nmax=nmax)
        return self.LMi.Optimize(self.QuadLossFunctor(k), self.q0[k], self.a0[k], self.allx0[k],
                                 tol=tol, nmax=nmax)

    def _optimize_frames(self, nmax, tol):
        """{k: Optimize(...)} for the local frames.  With `concurrent_frames` > 1 (default on a
        HIP device: up to 4) the frames' independent L-BFGS runs are driven by that many host
        threads, each on its own HIP stream, so one frame's host-side work (L-BFGS logic,
        launches, .item() syncs) overlaps the others' kernels; every frame's computation is
        unchanged, so the results are bitwise those of the sequential loop (PSR.py:528)."""
        frames = list(self.frames)
        nconc = getattr(self, "concurrent_frames", None)
        if nconc is None:
            nconc = 4 if str(self.compspec.get("device", "cpu")).startswith("cuda") else 1
        nconc = min(int(nconc), len(frames))
        if self._batch_frames_ok(len(frames)):
            return self._optimize_frames_batched(frames, max(1, nconc), nmax, tol)
        from .. import _lib
        share = int(getattr(self, "batch_share", 0))
        if nconc <= 1 or self.LMi.row_split is not None:
            # one frame after another: alone on the chip unless a hint n > 1 is set
            with _lib.thread_option(share if share > 1 and self.LMi.row_split is None else 1,
                                    "batch_share"):
                return {k: self._optimize_frame(k, nmax, tol) for k in frames}
        import threading
        from concurrent.futures import ThreadPoolExecutor
        main = torch.cuda.current_stream()
        streams = [torch.cuda.Stream() for _ in range(nconc)]
        for st in streams:
            st.wait_stream(main)        # inputs (q0, a0, targets) were produced on `main`
        # one stream per worker THREAD (not per frame index): a thread that finishes early
        # and picks up the next frame keeps its own stream, so two frames driven by two
        # threads never share (and serialise on) one stream
        local = threading.local()
        lock = threading.Lock()
        free = list(streams)

        share = nconc if share == 0 else max(1, share)     # 0 = the concurrent frames

        def work(k):
            st = getattr(local, "stream", None)
            if st is None:
                with lock:
                    st = local.stream = free.pop()
            with torch.cuda.stream(st), _lib.thread_option(share, "batch_share"):
                out = self._optimize_frame(k, nmax, tol)
            st.synchronize()            # results are consumed on `main` afterwards
            return k, out

        from .shooting import graphs_blocked
        with graphs_blocked(), ThreadPoolExecutor(max_workers=nconc) as ex:
            return dict(ex.map(work, frames))

    def _batch_frames_ok(self, nframes):
        """Whether Reg_opt runs the local frames in lockstep launch batches (core/batching.py):
        `batch_frames` True (opt-in; None / False = off), when every frame's shooting takes the
        batchable path -- dense support (no external points), Euler, the eta = 0 models
        (classic / hybrid) on the packed kernels (fwd_alg 2/5/6, bwd_alg 3) -- on a HIP device
        with at least 2 local frames."""
        want = getattr(self, "batch_frames", None)
        if not want:     # opt-in (None = off): measured slower than per-frame streams, DESIGN §6
            return False
        ok = (nframes >= 2 and self.support_scheme is None and self.LMi.scheme == "Euler"
              and self.LMi.eta == 0 and self.LMi.row_split is None
              and not getattr(self.LMi, "try_trajcost_optim", False)
              and getattr(self.LMi, "row_orders", None) is None
              and str(self.compspec.get("device", "cpu")).startswith("cuda"))
        if ok:
            from .. import _lib
            ok = _lib.get_option("fwd_alg") in (2, 5, 6) and _lib.get_option("bwd_alg") == 3
        if want is True and not ok:
            raise ValueError("batch_frames=True needs dense support, Euler, eta = 0, fwd_alg 2, "
                             "bwd_alg 3 and >= 2 local frames on a HIP device")
        return ok

    def _optimize_frames_batched(self, frames, ngroups, nmax, tol):
        """{k: Optimize(...)}: every local frame on its own host thread, the frames split into
        `ngroups` groups (contiguous in frame order), each group on one HIP stream with one
        LaunchBatcher -- within a group the frames' shooting launches are issued as one batched
        grid per step (lockstep), while the groups overlap each other's host work.  Each
        frame's computation is unchanged: results bitwise those of the sequential loop.
        (`concurrent_frames` = the number of groups here; 1 = every local frame in one batch.)"""
        from concurrent.futures import ThreadPoolExecutor

        from .batching import LaunchBatcher, frame_thread
        main = torch.cuda.current_stream()
        per = -(-len(frames) // ngroups)
        groups = [frames[i:i + per] for i in range(0, len(frames), per)]
        batchers = []
        for g in groups:
            st = torch.cuda.Stream()
            st.wait_stream(main)
            batchers.append(LaunchBatcher(st))
        owner = {k: batchers[i] for i, g in enumerate(groups) for k in g}

        share = int(getattr(self, "batch_share", 0))
        share = per if share == 0 else max(1, share)     # 0 = the group size

        def work(k):
            b = owner[k]
            with frame_thread(b, k, share):
                out = self._optimize_frame(k, nmax, tol)
            b.stream.synchronize()       # results are consumed on `main` afterwards
            return k, out

        from .shooting import graphs_blocked
        with graphs_blocked(), ThreadPoolExecutor(max_workers=len(frames)) as ex:
            res = dict(ex.map(work, frames))
        self.batch_stats = {"groups": len(groups), "batches": sum(b.batches for b in batchers),
                            "calls": sum(b.calls for b in batchers)}
        return res

    def Reg_opt(self, nmax=10, tol=1e-3):
        """Per-frame LDDMM optimisation (PSR.py:521-569), local frames only when sharded."""
        results = self._optimize_frames(nmax, tol)
        for k in self.frames:
            self.a0[k], self.shoot[k], self.regloss[k], datal, isteps, change = results[k]
            allx1k = self.shoot[k][-1][0] if self.support_scheme is None else self.shoot[k][-1][-1]
            last = 0
            for s in range(self.S):
                first, last = last, last + int(self.N[k, s])
                self.x1[k, s] = allx1k[first:last].to(**self.dataspec)
            for s in range(self.S):
                self.update_quadloss(k, s)
            if self.support_scheme is not None:
                warn_uncovered(self.LMi.Kernel, self.shoot[k])
            chg = change if isinstance(change, str) else f"{change:.4}"
            msg = f"Frame {k} : {isteps} optim steps, loss={self.regloss[k] + datal:.4}, change={chg}."
            if self.world == 1:
                self.update_FE(message=msg)
            elif self.printstuff:
                print(f"[rank {self.rank}] " + msg)
        if self.world > 1:
            self.update_FE(message="Reg_opt (all frames)")
