"""GPEngine — tensors in, tensors out, through the C ABI of libgpx.so.

PyTorch-ROCm tensors are only device-memory containers here: every byte of arithmetic on the hot path
(Gram, Cholesky, triangular inverse, alpha, K*, the triangular sweep, acquisition, argmax) runs in the
hand-written HIP kernels of ``bayesianoptimizer_amd/csrc``.  All launches go on torch's current stream of
the engine's device, so torch events / synchronisation compose with them.

Reference surface this mirrors:
  fit       ≙ SingleTaskGP(train_X, train_Y) + exact posterior caches (optimization/Bayesian.py:89-94,
              optimization/Bayesian6.py:458-490) with FIXED hyperparameters (MLL fitting is §8f row 1)
  posterior ≙ model.posterior(X).mean / .variance (optimization/Bayesian2.py:169-171,
              optimization/Bayesian6.py:615-617)
  acquire   ≙ analytic EI/LogEI/UCB or posterior-variance sweep + argmax (optimization/Bayesian.py:96-113,
              optimization/Bayesian7.py:646-681)
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence, Union

import torch

from . import _capi
from ._capi import (ACQ_EI, ACQ_LOGEI, ACQ_UCB, ACQ_VARIANCE, KERNEL_MATERN52, KERNEL_RBF,
                    KERNEL_SCALE_LINEAR_MATERN52, AcqParamsC, GPXError, GPXTimeoutError, KernelParamsC,
                    NotPositiveDefiniteError, info_error)

KERNEL_KINDS = {"rbf": KERNEL_RBF, "matern52": KERNEL_MATERN52,
                "scale_linear_matern52": KERNEL_SCALE_LINEAR_MATERN52}
ACQ_KINDS = {"ei": ACQ_EI, "logei": ACQ_LOGEI, "ucb": ACQ_UCB, "variance": ACQ_VARIANCE}


def botorch_default_lengthscale(d: int) -> float:
    """Mode of BoTorch's dimension-scaled LogNormal(sqrt2 + log(d)/2, sqrt3) lengthscale prior [upstream]
    (the prior of the SingleTaskGP default covariance reached from optimization/Bayesian.py:91)."""
    return math.exp(math.sqrt(2.0) + 0.5 * math.log(d) - 3.0)


@dataclass
class KernelParams:
    """Fixed GP hyperparameters (the arguments of the reference's covar_module/likelihood/mean)."""

    kind: Union[str, int] = "rbf"
    lengthscale: Union[float, Sequence[float]] = 1.0
    outputscale: float = 1.0
    noise: float = 1e-4
    jitter: float = 0.0
    const_mean: float = 0.0
    linear_variance: Union[float, Sequence[float]] = 1.0
    cov_fp32: bool = False  # fp32 covariance evaluation, fp64 factorisation (BASELINE configs[4])

    @property
    def kind_id(self) -> int:
        if isinstance(self.kind, str):
            try:
                return KERNEL_KINDS[self.kind.lower()]
            except KeyError as e:
                raise ValueError(f"unknown kernel '{self.kind}', expected one of {sorted(KERNEL_KINDS)}") from e
        return int(self.kind)

    def lengthscales(self, d: int):
        ls = [float(self.lengthscale)] * d if isinstance(self.lengthscale, (int, float)) else \
            [float(v) for v in self.lengthscale]
        if len(ls) != d:
            raise ValueError(f"expected {d} lengthscales, got {len(ls)}")
        return ls

    def linear_variances(self, d: int):
        lv = [float(self.linear_variance)] * d if isinstance(self.linear_variance, (int, float)) else \
            [float(v) for v in self.linear_variance]
        if len(lv) != d:
            raise ValueError(f"expected {d} linear variances, got {len(lv)}")
        return lv

    def to_c(self, d: int) -> KernelParamsC:
        if not 1 <= d <= _capi.GPX_MAX_DIM:
            raise ValueError(f"input dimension {d} outside [1, {_capi.GPX_MAX_DIM}]")
        c = KernelParamsC()
        c.kind = self.kind_id
        c.d = d
        c.lengthscale[:d] = self.lengthscales(d)  # slice assignment: one ctypes call per array (to_c runs per fit)
        c.linear_variance[:d] = self.linear_variances(d)
        c.outputscale = float(self.outputscale)
        c.noise = float(self.noise)
        c.jitter = float(self.jitter)
        c.const_mean = float(self.const_mean)
        c.cov_fp32 = 1 if self.cov_fp32 else 0
        return c

    def replace(self, **kw) -> "KernelParams":
        d = dict(self.__dict__)
        d.update(kw)
        return KernelParams(**d)


@dataclass
class GPState:
    """Device-resident posterior caches of one exact GP (all tensors on the engine's device).

    L: padded lower Cholesky factor (only its lower triangle is defined), W = L^{-T} (upper), alpha =
    K^{-1}(Y - m) (padded_n x nrhs), Dinv: inverses of the 64x64 diagonal blocks of L.  L and W may be
    npad x npad views of larger capacity x capacity buffers (``GPEngine.append`` grows into them); their
    leading dimension is ``L.stride(0)``.  ``W_ready`` is False after a factor-only update (``GPEngine.fit`` with
    ``inverse=False``): W is then built by ``GPEngine.inverse`` the first time a sweep / posterior / gradient needs it.
    """

    X: torch.Tensor
    L: torch.Tensor
    W: torch.Tensor
    Dinv: torch.Tensor
    alpha: torch.Tensor
    info: torch.Tensor
    params: KernelParams
    n: int
    npad: int
    nrhs: int
    _batch: Optional[tuple] = field(default=None, repr=False)  # stacked tensors of a fit_batched call
    W_ready: bool = True

    @property
    def d(self) -> int:
        return self.X.shape[1]

    def pivot_failure(self) -> int:
        """0-based failing pivot, or -1 (synchronises).  A factorisation or triangular solve whose in-launch hand-off
        timed out (info = GPX_INFO_TIMEOUT) raises GPXTimeoutError: it is not a pivot, and no jitter cures it."""
        v = int(self.info.item())
        if v < 0:
            raise info_error(v)
        return v - 1 if v else -1

    def check(self, what: str = "") -> None:
        """Raise NotPositiveDefiniteError / GPXTimeoutError for a failed update (synchronises)."""
        err = info_error(int(self.info.item()), what)
        if err is not None:
            raise err


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class GPEngine:
    """One engine per device; launches on torch's current stream of that device."""

    def __init__(self, device: Union[int, str, torch.device, None] = None):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device) if not isinstance(device, torch.device) else device
        if device.type != "cuda":
            raise ValueError("GPEngine runs on a ROCm GPU device ('cuda:N'); there is no CPU path")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.lib = _capi.load()
        h = ctypes.c_void_p()
        st = self.lib.gpx_create(int(device.index), ctypes.byref(h))
        if st != _capi.GPX_OK:
            raise GPXError(st, f"gpx_create(device={device.index}) failed")
        self.handle = h
        self._ws = {}
        self._stream_ptr = None

    # -- plumbing ---------------------------------------------------------------------------------
    def __del__(self):
        try:
            if getattr(self, "handle", None) is not None and self.lib is not None:
                self.lib.gpx_destroy(self.handle)
                self.handle = None
        except Exception:
            pass

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream_ptr:
            _capi.check(self.lib.gpx_set_stream(self.handle, ctypes.c_void_p(s)), self.handle)
            self._stream_ptr = s

    def _check(self, st: int):
        _capi.check(st, self.handle)

    def workspace(self, key: str, nbytes: int) -> torch.Tensor:
        buf = self._ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            self._ws[key] = buf
        return buf

    def _as_f64(self, t, name: str) -> torch.Tensor:
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t)
        t = t.to(device=self.device, dtype=torch.float64)
        if t.dim() == 1:
            t = t.unsqueeze(-1)
        return t.contiguous()

    @staticmethod
    def padded_n(n: int) -> int:
        return ((n + _capi.GPX_TILE - 1) // _capi.GPX_TILE) * _capi.GPX_TILE

    # -- fit --------------------------------------------------------------------------------------
    def set_option(self, name: str, value: int) -> None:
        """Per-handle tuning / diagnostic option (include/gpx.h GPX_OPT_*: spin_limit, sweep_fused,
        gram_split, potrf_lazy, potrf_mode)."""
        self._check(self.lib.gpx_set_option(self.handle, _capi.OPTIONS[name], int(value)))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        self._check(self.lib.gpx_get_option(self.handle, _capi.OPTIONS[name], ctypes.byref(v)))
        return int(v.value)

    def alloc_state(self, X: torch.Tensor, nrhs: int, params: KernelParams, capacity: int = 0) -> GPState:
        """Device buffers of one GP; ``capacity`` (training points) reserves room for later ``append`` calls."""
        n = X.shape[0]
        npad = self.padded_n(n)
        cap = max(npad, self.padded_n(capacity)) if capacity else npad
        dev = self.device
        Lbuf = torch.empty((cap, cap), dtype=torch.float64, device=dev)
        Wbuf = torch.empty((cap, cap), dtype=torch.float64, device=dev)
        return GPState(
            X=X,
            L=Lbuf[:npad, :npad],
            W=Wbuf[:npad, :npad],
            Dinv=torch.empty((2 * (cap // 64), 64, 64), dtype=torch.float64, device=dev),
            alpha=torch.empty((npad, nrhs), dtype=torch.float64, device=dev),
            info=torch.zeros((1,), dtype=torch.int32, device=dev),
            params=params, n=n, npad=npad, nrhs=nrhs)

    def fit(self, X, Y, params: KernelParams, check: bool = True, out: Optional[GPState] = None,
            capacity: int = 0, inverse: bool = False) -> GPState:
        """One posterior update: Gram + blocked Cholesky + alpha for up to 8 outputs sharing X.

        ``inverse=False`` (default): alpha by the triangular solves of gpx_fit_factor_f64 and W = L^{-T} left to
        ``GPEngine.inverse``, which the sweep / posterior / gradient / append entry points call on first use (an
        update followed by another update before any sweep never pays for W).  ``inverse=True``: gpx_fit_f64 (W formed
        in the same call, alpha from W).  With ``check`` (default) synchronises and raises NotPositiveDefiniteError like
        psd_safe_cholesky would; with ``check=False`` stays asynchronous (inspect ``state.info`` later).  ``capacity``:
        training points to reserve buffer room for (later ``append`` calls grow in place up to it).
        """
        X = self._as_f64(X, "X")
        Y = self._as_f64(Y, "Y")
        n, d = X.shape
        if Y.shape[0] != n:
            raise ValueError(f"X has {n} rows but Y has {Y.shape[0]}")
        nrhs = Y.shape[1]
        if not 1 <= nrhs <= _capi.GPX_MAX_RHS:
            raise ValueError(f"number of outputs {nrhs} outside [1, {_capi.GPX_MAX_RHS}]")
        pc = params.to_c(d)
        st = out if (out is not None and out.n == n and out.nrhs == nrhs) else \
            self.alloc_state(X, nrhs, params, capacity)
        st.X, st.params = X, params
        nbytes = ctypes.c_size_t()
        self._bind_stream()
        if inverse:
            self._check(self.lib.gpx_fit_workspace_size(n, nrhs, ctypes.byref(nbytes)))
            ws = self.workspace("fit", nbytes.value)
            self._check(self.lib.gpx_fit_f64(
                self.handle, ctypes.byref(pc), n, _ptr(X), X.stride(0), _ptr(Y), Y.stride(0), nrhs,
                _ptr(st.L), st.L.stride(0), _ptr(st.Dinv), _ptr(st.W), st.W.stride(0), _ptr(st.alpha), _ptr(st.info),
                _ptr(ws), ws.numel()))
        else:
            self._check(self.lib.gpx_fit_factor_workspace_size(n, nrhs, ctypes.byref(nbytes)))
            ws = self.workspace("potrs", nbytes.value)
            self._check(self.lib.gpx_fit_factor_f64(
                self.handle, ctypes.byref(pc), n, _ptr(X), X.stride(0), _ptr(Y), Y.stride(0), nrhs,
                _ptr(st.L), st.L.stride(0), _ptr(st.Dinv), _ptr(st.alpha), _ptr(st.info), _ptr(ws), ws.numel()))
        st.W_ready = inverse
        if check:
            st.check()
        return st

    def inverse(self, state: GPState) -> GPState:
        """Build W = L^{-T} of a factor-only update (gpx_trtri_f64 from L and the diagonal-block inverses); no-op when
        it is already there.  Asynchronous."""
        if state.W_ready:
            return state
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_trtri_workspace_size(state.n, ctypes.byref(nbytes)))
        ws = self.workspace("fit", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_trtri_f64(self.handle, state.n, _ptr(state.L), state.L.stride(0), _ptr(state.Dinv),
                                           _ptr(state.W), state.W.stride(0), _ptr(ws), ws.numel()))
        state.W_ready = True
        return state

    def inverse_batched(self, states: Sequence[GPState]) -> Sequence[GPState]:
        """W for every state of one ``fit_batched`` call in the same launches (gpx_trtri_batched_f64); states that
        already have W are left alone, states of different calls fall back to ``inverse`` one by one."""
        todo = [st for st in states if not st.W_ready]
        if not todo:
            return states
        b0 = todo[0]._batch
        if b0 is None or len(todo) != len(states) or any(st._batch is not b0 for st in todo):
            for st in todo:
                self.inverse(st)
            return states
        Lb, Wb, Db, _, _ = b0
        B, npad = Lb.shape[0], Lb.shape[1]
        if B != len(states):
            for st in todo:
                self.inverse(st)
            return states
        n = states[0].n
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_trtri_batched_workspace_size(n, B, ctypes.byref(nbytes)))
        ws = self.workspace("trtri_batched", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_trtri_batched_f64(self.handle, B, n, _ptr(Lb), npad, Lb.stride(0), _ptr(Db),
                                                   Db.stride(0), _ptr(Wb), npad, Wb.stride(0), _ptr(ws), ws.numel()))
        for st in states:
            st.W_ready = True
        return states

    def potrs(self, state: GPState, Y) -> torch.Tensor:
        """alpha = K^{-1}(Y - const_mean) from the state's factor alone (gpx_potrs_f64): new targets on the same X.
        The solve reports into an info word of its own (a copy of the state's): a timed-out hand-off raises
        GPXTimeoutError here and leaves the fitted state (its L, alpha and info) valid."""
        Y = self._as_f64(Y, "Y")
        if Y.shape[0] != state.n:
            raise ValueError(f"Y must have {state.n} rows, got {Y.shape[0]}")
        nrhs = Y.shape[1]
        alpha = torch.empty((state.npad, nrhs), dtype=torch.float64, device=self.device)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_potrs_workspace_size(state.n, nrhs, ctypes.byref(nbytes)))
        ws = self.workspace("potrs", nbytes.value)
        self._bind_stream()
        info = state.info.clone()
        self._check(self.lib.gpx_potrs_f64(
            self.handle, state.n, _ptr(state.L), state.L.stride(0), _ptr(state.Dinv), _ptr(Y), Y.stride(0), nrhs,
            float(state.params.const_mean), _ptr(alpha), _ptr(info), _ptr(ws), ws.numel()))
        # a failed factor (info = pivot + 1, e.g. after fit(check=False)) leaves alpha untouched, a timed-out hand-off
        # writes GPX_INFO_TIMEOUT: both raise instead of returning the uninitialised buffer
        err = _capi.info_error(int(info.item()), "potrs")
        if err is not None:
            raise err
        return alpha

    def append(self, state: GPState, X, Y, check: bool = True, growth: float = 1.5) -> GPState:
        """Incremental posterior update: X / Y hold ALL training rows, the first ``state.n`` of them
        the ones ``state`` was fitted on (same hyperparameters).  The bordered Cholesky of the new rows
        (gpx_append_f64, O(n^2 q)) replaces the reference's refit from scratch after appending observations
        (optimization/Bayesian7.py:628-631,639; optimization/Bayesian.py:163-174).  Y may be re-standardised: alpha is
        recomputed from all of it.  Grows the buffers (by ``growth``) when the capacity is exceeded.  Returns the
        updated state (the same object when it fitted in place)."""
        X = self._as_f64(X, "X")
        Y = self._as_f64(Y, "Y")
        n_new, d = X.shape
        n_old = state.n
        if d != state.d:
            raise ValueError(f"X has {d} columns, state has d={state.d}")
        if Y.shape != (n_new, state.nrhs):
            raise ValueError(f"Y must have shape ({n_new}, {state.nrhs}), got {tuple(Y.shape)}")
        if n_new <= n_old:
            raise ValueError(f"append needs more rows than the fitted {n_old}, got {n_new}")
        self.inverse(state)  # the bordered update extends W
        npad = self.padded_n(n_new)
        ld = state.L.stride(0)
        if npad > ld or state.Dinv.shape[0] < 2 * (npad // 64) or state.W.stride(0) != ld:
            # grow: copy the kept leading block into bigger buffers (plumbing; the update itself is gpx_append_f64)
            cap = self.padded_n(max(n_new, int(growth * n_new)))
            n0 = (n_old // _capi.GPX_TILE) * _capi.GPX_TILE
            new = self.alloc_state(X, state.nrhs, state.params, cap)
            Lb = new.L.as_strided((cap, cap), (cap, 1))
            Wb = new.W.as_strided((cap, cap), (cap, 1))
            Lb[:n0, :n0].copy_(state.L[:n0, :n0])
            Wb[:n0, :n0].copy_(state.W[:n0, :n0])
            new.Dinv[: n0 // 64].copy_(state.Dinv[: n0 // 64])
            state, ld = new, cap
        Lfull = state.L.as_strided((npad, npad), (ld, 1))
        Wfull = state.W.as_strided((npad, npad), (ld, 1))
        alpha = torch.empty((npad, state.nrhs), dtype=torch.float64, device=self.device)
        pc = state.params.to_c(d)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_append_workspace_size(n_old, n_new, state.nrhs, ctypes.byref(nbytes)))
        ws = self.workspace("append", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_append_f64(
            self.handle, ctypes.byref(pc), n_old, n_new, _ptr(X), X.stride(0), _ptr(Y), Y.stride(0), state.nrhs,
            _ptr(Lfull), ld, _ptr(state.Dinv), _ptr(Wfull), ld, _ptr(alpha), _ptr(state.info), _ptr(ws), ws.numel()))
        state.X, state.L, state.W, state.alpha = X, Lfull, Wfull, alpha
        state.n, state.npad, state._batch = n_new, npad, None
        if check:
            state.check()
        return state

    def fit_batched(self, X, Y, params: Union[KernelParams, Sequence[KernelParams]], check: bool = True,
                    out: Optional[Sequence[GPState]] = None, inverse: bool = False) -> list:
        """Posterior updates of B independent problems (X: B x n x d, Y: B x n or B x n x nrhs) sharing n and d
        (restarts / seeds, BASELINE configs[3]) in the same launches (gpx_fit_factor_batched_f64, or gpx_fit_batched_f64
        with ``inverse``: W formed for every problem in the same launches).  ``params``: one KernelParams shared by all
        problems, or a sequence of B (gpx_fit_*_batched_params_f64).  Returns one GPState per problem (views into
        stacked device tensors); results equal B calls of ``fit``.  With ``check`` synchronises and raises
        NotPositiveDefiniteError for the first failing problem."""
        X = X if isinstance(X, torch.Tensor) else torch.as_tensor(X)
        Y = Y if isinstance(Y, torch.Tensor) else torch.as_tensor(Y)
        X = X.to(device=self.device, dtype=torch.float64).contiguous()
        Y = Y.to(device=self.device, dtype=torch.float64)
        if X.dim() != 3:
            raise ValueError("X must be B x n x d")
        if Y.dim() == 2:
            Y = Y.unsqueeze(-1)
        Y = Y.contiguous()
        B, n, d = X.shape
        if Y.shape[:2] != (B, n):
            raise ValueError(f"Y must be {B} x {n} (x nrhs), got {tuple(Y.shape)}")
        return self._fit_batch(X, X.stride(1), X.stride(0), Y, Y.stride(1), Y.stride(0), Y.shape[2], B, n, d, params,
                               check, out, inverse, [X[b] for b in range(B)])

    def fit_outputs(self, X, Y, params: Sequence[KernelParams], check: bool = True,
                    out: Optional[Sequence[GPState]] = None, inverse: bool = False) -> list:
        """T independent GPs on ONE training set: X n x d, Y n x T, one KernelParams per output — the reference's
        multi-output SingleTaskGP (optimization/Bayesian1.py:108-116: a batch of independent GPs on one X, each with its
        own lengthscales, outputscale, noise and constant mean [upstream]).  One call of gpx_fit_*_batched_params_f64
        with X shared (stride 0) and Y read column by column (stride 1, ldy = T): the Cholesky and solves of all T
        outputs run in the same launches.  Returns one GPState per output (nrhs = 1, X = the shared tensor)."""
        X = self._as_f64(X, "X")
        Y = self._as_f64(Y, "Y")
        n, d = X.shape
        if Y.shape[0] != n:
            raise ValueError(f"X has {n} rows but Y has {Y.shape[0]}")
        T = Y.shape[1]
        if len(params) != T:
            raise ValueError(f"expected {T} kernel parameter sets (one per output), got {len(params)}")
        return self._fit_batch(X, X.stride(0), 0, Y, Y.stride(0), 1, 1, T, n, d, list(params), check, out, inverse,
                               [X] * T)

    @staticmethod
    def batch_info(states: Sequence[GPState]):
        """The pivot-failure words of ``states`` as one host array (one synchronisation): 0, pivot + 1, or
        GPX_INFO_TIMEOUT."""
        b0 = states[0]._batch
        if b0 is not None and all(st._batch is b0 for st in states) and b0[4].numel() == len(states):
            return b0[4].cpu().numpy()
        return torch.cat([st.info for st in states]).cpu().numpy()

    def _fit_batch(self, X, ldx, sx, Y, ldy, sy, nrhs, B, n, d, params, check, out, inverse, Xviews) -> list:
        if not 1 <= nrhs <= _capi.GPX_MAX_RHS:
            raise ValueError(f"number of outputs {nrhs} outside [1, {_capi.GPX_MAX_RHS}]")
        per_problem = not isinstance(params, KernelParams)
        plist = list(params) if per_problem else [params] * B
        if len(plist) != B:
            raise ValueError(f"expected {B} kernel parameter sets, got {len(plist)}")
        pcs = (KernelParamsC * B)(*[pp.to_c(d) for pp in plist]) if per_problem else plist[0].to_c(d)
        npad = self.padded_n(n)
        nblk = npad // 64
        if out is not None and len(out) == B and all(s.n == n and s.nrhs == nrhs for s in out) and \
                out[0]._batch is not None:
            Lb, Wb, Db, Ab, Ib = out[0]._batch
        else:
            dev = self.device
            Lb = torch.empty((B, npad, npad), dtype=torch.float64, device=dev)
            Wb = torch.empty((B, npad, npad), dtype=torch.float64, device=dev)
            Db = torch.empty((B, 2 * nblk, 64, 64), dtype=torch.float64, device=dev)
            Ab = torch.empty((B, npad, nrhs), dtype=torch.float64, device=dev)
            Ib = torch.zeros((B,), dtype=torch.int32, device=dev)
        nbytes = ctypes.c_size_t()
        self._bind_stream()
        pref = pcs if per_problem else ctypes.byref(pcs)
        sfx = "_params" if per_problem else ""
        if inverse:
            self._check(self.lib.gpx_fit_batched_workspace_size(n, nrhs, B, ctypes.byref(nbytes)))
            ws = self.workspace("fit_batched", nbytes.value)
            self._check(getattr(self.lib, f"gpx_fit_batched{sfx}_f64")(
                self.handle, pref, B, n, _ptr(X), ldx, sx, _ptr(Y), ldy, sy, nrhs, _ptr(Lb), npad, Lb.stride(0),
                _ptr(Db), Db.stride(0), _ptr(Wb), npad, Wb.stride(0), _ptr(Ab), Ab.stride(0), _ptr(Ib), _ptr(ws),
                ws.numel()))
        else:
            self._check(self.lib.gpx_fit_factor_batched_workspace_size(n, nrhs, B, ctypes.byref(nbytes)))
            ws = self.workspace("potrs_batched", nbytes.value)
            self._check(getattr(self.lib, f"gpx_fit_factor_batched{sfx}_f64")(
                self.handle, pref, B, n, _ptr(X), ldx, sx, _ptr(Y), ldy, sy, nrhs, _ptr(Lb), npad, Lb.stride(0),
                _ptr(Db), Db.stride(0), _ptr(Ab), Ab.stride(0), _ptr(Ib), _ptr(ws), ws.numel()))
        states = []
        batch = (Lb, Wb, Db, Ab, Ib)  # ONE object shared by the states: inverse_batched / batch_info test identity
        for b in range(B):
            states.append(GPState(X=Xviews[b], L=Lb[b], W=Wb[b], Dinv=Db[b], alpha=Ab[b], info=Ib[b:b + 1],
                                  params=plist[b], n=n, npad=npad, nrhs=nrhs, _batch=batch, W_ready=inverse))
        if check:
            bad = Ib.cpu().numpy()
            for b in range(B):
                err = info_error(int(bad[b]), f"problem {b}")
                if err is not None:
                    raise err
        return states

    # individual stages (tests and benchmarks)
    def gram(self, X, params: KernelParams) -> torch.Tensor:
        X = self._as_f64(X, "X")
        n, d = X.shape
        npad = self.padded_n(n)
        K = torch.zeros((npad, npad), dtype=torch.float64, device=self.device)
        pc = params.to_c(d)
        self._bind_stream()
        self._check(self.lib.gpx_gram_f64(self.handle, ctypes.byref(pc), n, _ptr(X), X.stride(0), _ptr(K), npad))
        return K

    def potrf(self, K: torch.Tensor, n: int):
        """In-place Cholesky of a padded matrix; returns (Dinv, info tensor)."""
        npad = K.shape[0]
        Dinv = torch.empty((2 * (npad // 64), 64, 64), dtype=torch.float64, device=self.device)
        info = torch.zeros((1,), dtype=torch.int32, device=self.device)
        self._bind_stream()
        self._check(self.lib.gpx_potrf_f64(self.handle, n, _ptr(K), K.stride(0), _ptr(Dinv), _ptr(info)))
        return Dinv, info

    def trtri(self, L: torch.Tensor, Dinv: torch.Tensor, n: int) -> torch.Tensor:
        npad = L.shape[0]
        W = torch.zeros((npad, npad), dtype=torch.float64, device=self.device)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_trtri_workspace_size(n, ctypes.byref(nbytes)))
        ws = self.workspace("fit", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_trtri_f64(self.handle, n, _ptr(L), L.stride(0), _ptr(Dinv), _ptr(W), npad,
                                           _ptr(ws), ws.numel()))
        return W

    # -- posterior / acquisition ----------------------------------------------------------------
    def posterior(self, state: GPState, Xs, y_mean: Optional[Sequence[float]] = None,
                  y_scale: Optional[Sequence[float]] = None):
        """Posterior mean (m x nrhs) and variance (m) at Xs; (y_mean, y_scale) = Standardize untransform."""
        Xs = self._as_f64(Xs, "Xs")
        if Xs.shape[1] != state.d:
            raise ValueError(f"Xs has {Xs.shape[1]} columns, model has d={state.d}")
        m = Xs.shape[0]
        self.inverse(state)
        mean = torch.empty((m, state.nrhs), dtype=torch.float64, device=self.device)
        var = torch.empty((m,), dtype=torch.float64, device=self.device)
        if m == 0:
            return mean, var
        ym = (ctypes.c_double * state.nrhs)(*([0.0] * state.nrhs if y_mean is None else [float(v) for v in y_mean]))
        ys = (ctypes.c_double * state.nrhs)(*([1.0] * state.nrhs if y_scale is None else [float(v) for v in y_scale]))
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_sweep_workspace_size(state.n, state.nrhs, m, ctypes.byref(nbytes)))
        ws = self.workspace("sweep", nbytes.value)
        pc = state.params.to_c(state.d)
        self._bind_stream()
        self._check(self.lib.gpx_posterior_f64(
            self.handle, ctypes.byref(pc), state.n, _ptr(state.X), state.X.stride(0), _ptr(state.W), state.W.stride(0),
            _ptr(state.alpha), state.nrhs, _ptr(Xs), m, Xs.stride(0), ym, ys, _ptr(mean), state.nrhs, _ptr(var),
            _ptr(ws), ws.numel()))
        return mean, var

    def acquire(self, state: GPState, Xs, kind: Union[str, int] = "logei", best_f: float = 0.0, beta: float = 4.0,
                y_mean: float = 0.0, y_scale: float = 1.0, alpha: Optional[torch.Tensor] = None,
                index_offset: int = 0, return_scores: bool = False):
        """Score every candidate and return device scalars (best_value, best_index) (+ scores)."""
        Xs = self._as_f64(Xs, "Xs")
        if Xs.shape[1] != state.d:
            raise ValueError(f"Xs has {Xs.shape[1]} columns, model has d={state.d}")
        m = Xs.shape[0]
        if m == 0:
            raise ValueError("empty candidate set")
        self.inverse(state)
        kid = ACQ_KINDS[kind.lower()] if isinstance(kind, str) else int(kind)
        if alpha is None:
            alpha = state.alpha[:, 0]
        alpha = alpha.to(device=self.device, dtype=torch.float64).contiguous()
        if alpha.numel() != state.npad:
            raise ValueError("alpha must have padded_n entries")
        ap = AcqParamsC()
        ap.kind, ap.best_f, ap.beta, ap.y_mean, ap.y_scale = kid, float(best_f), float(beta), float(y_mean), \
            float(y_scale)
        best_val = torch.empty((1,), dtype=torch.float64, device=self.device)
        best_idx = torch.empty((1,), dtype=torch.int64, device=self.device)
        scores = torch.empty((m,), dtype=torch.float64, device=self.device) if return_scores else None
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_sweep_workspace_size(state.n, 1, m, ctypes.byref(nbytes)))
        ws = self.workspace("sweep", nbytes.value)
        pc = state.params.to_c(state.d)
        self._bind_stream()
        self._check(self.lib.gpx_acquire_argmax_f64(
            self.handle, ctypes.byref(pc), state.n, _ptr(state.X), state.X.stride(0), _ptr(state.W), state.W.stride(0),
            _ptr(alpha), _ptr(Xs), m, Xs.stride(0), ctypes.byref(ap), int(index_offset), _ptr(best_val),
            _ptr(best_idx), _ptr(scores), _ptr(ws), ws.numel()))
        if return_scores:
            return best_val, best_idx, scores
        return best_val, best_idx

    def acquire_multi(self, states: Sequence[GPState], Xs, kind: Union[str, int] = "logei", best_f: float = 0.0,
                      beta: float = 4.0, weights: Optional[Sequence[float]] = None,
                      y_mean: Optional[Sequence[float]] = None, y_scale: Optional[Sequence[float]] = None,
                      index_offset: int = 0, return_scores: bool = False):
        """Score a linear objective sum_t w_t f_t over the T independent outputs of one ``fit_outputs`` call
        (gpx_acquire_argmax_multi_f64: mean sum_t w_t (y_mean_t + y_scale_t mu_t), variance sum_t w_t^2 y_scale_t^2
        var_t) and return device scalars (best_value, best_index) (+ scores).  ``kind="variance"`` with unit weights is
        the variance-sum pool-scan score (optimization/Bayesian7.py:671)."""
        Xs = self._as_f64(Xs, "Xs")
        T = len(states)
        if T < 1:
            raise ValueError("no outputs to score")
        st0 = states[0]
        if any(st.n != st0.n or st.X.shape != st0.X.shape for st in states):
            raise ValueError("acquire_multi needs outputs fitted on the same training inputs")
        d = st0.d
        if Xs.shape[1] != d:
            raise ValueError(f"Xs has {Xs.shape[1]} columns, model has d={d}")
        m = Xs.shape[0]
        if m == 0:
            raise ValueError("empty candidate set")
        self.inverse_batched(states)
        w = [1.0] * T if weights is None else [float(v) for v in weights]
        if len(w) != T:
            raise ValueError(f"expected {T} objective weights, got {len(w)}")
        ym = [0.0] * T if y_mean is None else [float(v) for v in y_mean]
        ys = [1.0] * T if y_scale is None else [float(v) for v in y_scale]
        kid = ACQ_KINDS[kind.lower()] if isinstance(kind, str) else int(kind)
        ap = AcqParamsC()
        ap.kind, ap.best_f, ap.beta, ap.y_mean, ap.y_scale = kid, float(best_f), float(beta), 0.0, 1.0
        pcs = (KernelParamsC * T)(*[st.params.to_c(d) for st in states])
        best_val = torch.empty((1,), dtype=torch.float64, device=self.device)
        best_idx = torch.empty((1,), dtype=torch.int64, device=self.device)
        scores = torch.empty((m,), dtype=torch.float64, device=self.device) if return_scores else None
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_sweep_multi_workspace_size(states[0].n, m, ctypes.byref(nbytes)))
        ws = self.workspace("sweep_multi", nbytes.value)
        X = st0.X
        alphas = [st.alpha[:, 0].contiguous() for st in states]  # keeps the columns alive across the call
        wp = (ctypes.c_void_p * T)(*[st.W.data_ptr() for st in states])
        ldw = (ctypes.c_int64 * T)(*[st.W.stride(0) for st in states])
        ap_ = (ctypes.c_void_p * T)(*[a.data_ptr() for a in alphas])
        self._bind_stream()
        self._check(self.lib.gpx_acquire_argmax_multi_f64(
            self.handle, pcs, T, st0.n, _ptr(X), X.stride(0), wp, ldw, ap_, (ctypes.c_double * T)(*w), (ctypes.c_double * T)(*ym), (ctypes.c_double * T)(*ys), _ptr(Xs),
            m, Xs.stride(0), ctypes.byref(ap), int(index_offset), _ptr(best_val), _ptr(best_idx), _ptr(scores),
            _ptr(ws), ws.numel()))
        if return_scores:
            return best_val, best_idx, scores
        return best_val, best_idx

    def moments_grad(self, state: GPState, Xs, q: int = 1, alpha: Optional[torch.Tensor] = None):
        """Posterior mean / q-batch covariance of candidates Xs (m x d, consecutive q-batches) and their derivatives
        w.r.t. the candidates (gpx_moments_grad_f64), in the engine's standardised units:
        mean (m), dmean (m x d), cov (m x q: row a of its batch's q x q covariance), dcov (m x d x q, first-argument
        partials; see include/gpx.h for the chain rule).  ``alpha``: padded_n objective column (default output 0)."""
        Xs = self._as_f64(Xs, "Xs")
        m, d = Xs.shape
        if d != state.d:
            raise ValueError(f"Xs has {d} columns, model has d={state.d}")
        if m % q:
            raise ValueError(f"{m} candidates do not form q-batches of {q}")
        self.inverse(state)
        if alpha is None:
            alpha = state.alpha[:, 0]
        alpha = alpha.to(device=self.device, dtype=torch.float64).contiguous()
        if alpha.numel() != state.npad:
            raise ValueError("alpha must have padded_n entries")
        dev = self.device
        mean = torch.empty((m,), dtype=torch.float64, device=dev)
        dmean = torch.empty((m, d), dtype=torch.float64, device=dev)
        cov = torch.empty((m, q), dtype=torch.float64, device=dev)
        dcov = torch.empty((m, d, q), dtype=torch.float64, device=dev)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_moments_grad_workspace_size(state.n, m, ctypes.byref(nbytes)))
        ws = self.workspace("moments_grad", nbytes.value)
        pc = state.params.to_c(d)
        self._bind_stream()
        self._check(self.lib.gpx_moments_grad_f64(
            self.handle, ctypes.byref(pc), state.n, _ptr(state.X), state.X.stride(0), _ptr(state.W), state.W.stride(0),
            _ptr(alpha), _ptr(Xs), m, q, Xs.stride(0), _ptr(mean), _ptr(dmean), _ptr(cov), _ptr(dcov), _ptr(ws),
            ws.numel()))
        return mean, dmean, cov, dcov

    def argmax_combine(self, vals: torch.Tensor, idx: torch.Tensor):
        """Deterministic (max value, lowest index) over device records (after the cross-rank gather)."""
        vals = vals.to(device=self.device, dtype=torch.float64).contiguous().reshape(-1)
        idx = idx.to(device=self.device, dtype=torch.int64).contiguous().reshape(-1)
        bv = torch.empty((1,), dtype=torch.float64, device=self.device)
        bi = torch.empty((1,), dtype=torch.int64, device=self.device)
        self._bind_stream()
        self._check(self.lib.gpx_argmax_combine_f64(self.handle, _ptr(vals), _ptr(idx), vals.numel(), _ptr(bv),
                                                    _ptr(bi)))
        return bv, bi

    # -- marginal likelihood ----------------------------------------------------
    def mll_grad(self, state: GPState, Y, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """-log p(Y) and its gradient w.r.t. the shared hyperparameters of a fitted state (Y: the n x nrhs targets
        the fit used), as a device vector of MLL_NOUT doubles (layout ``_capi.MLL_*``).  Asynchronous."""
        Y = self._as_f64(Y, "Y")
        if Y.shape != (state.n, state.nrhs):
            raise ValueError(f"Y must have shape ({state.n}, {state.nrhs}), got {tuple(Y.shape)}")
        if out is None:
            out = torch.empty((_capi.MLL_NOUT,), dtype=torch.float64, device=self.device)
        self.inverse(state)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_mll_workspace_size(state.n, ctypes.byref(nbytes)))
        ws = self.workspace("mll", nbytes.value)
        pc = state.params.to_c(state.d)
        self._bind_stream()
        self._check(self.lib.gpx_mll_grad_f64(
            self.handle, ctypes.byref(pc), state.n, _ptr(state.X), state.X.stride(0), _ptr(Y), Y.stride(0),
            state.nrhs, _ptr(state.L), state.L.stride(0), _ptr(state.W), state.W.stride(0), _ptr(state.alpha), _ptr(out),
            _ptr(ws), ws.numel()))
        return out

    def mll_grad_outputs(self, states: Sequence[GPState], Y, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """-log p(y_t) and its gradient w.r.t. output t's own hyperparameters for every output of one ``fit_outputs``
        call (Y: the n x T targets it used), as a T x MLL_NOUT device tensor (gpx_mll_grad_batched_f64).  Asynchronous."""
        Y = self._as_f64(Y, "Y")
        T = len(states)
        st0 = states[0]
        if Y.shape != (st0.n, T):
            raise ValueError(f"Y must have shape ({st0.n}, {T}), got {tuple(Y.shape)}")
        b0 = st0._batch
        if b0 is None or any(st._batch is not b0 for st in states) or b0[0].shape[0] != T:
            raise ValueError("mll_grad_outputs needs the states of one fit_outputs call, in order")
        self.inverse_batched(states)
        Lb, Wb, Db, Ab, Ib = b0
        if out is None:
            out = torch.empty((T, _capi.MLL_NOUT), dtype=torch.float64, device=self.device)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_mll_workspace_size(st0.n, ctypes.byref(nbytes)))
        ws = self.workspace("mll", nbytes.value)
        pcs = (KernelParamsC * T)(*[st.params.to_c(st0.d) for st in states])
        npad = st0.npad
        self._bind_stream()
        self._check(self.lib.gpx_mll_grad_batched_f64(
            self.handle, pcs, T, st0.n, _ptr(st0.X), st0.X.stride(0), 0, _ptr(Y), Y.stride(0), 1, 1, _ptr(Lb), npad,
            Lb.stride(0), _ptr(Wb), npad, Wb.stride(0), _ptr(Ab), Ab.stride(0), _ptr(out), _ptr(ws), ws.numel()))
        return out

    def mll_value_grad_outputs(self, X, Y, params: Sequence[KernelParams],
                               jitters: Sequence[float] = (0.0, 1e-8, 1e-7, 1e-6),
                               states: Optional[Sequence[GPState]] = None):
        """``mll_value_grad`` for T independent outputs on one X (Y: n x T, one KernelParams each), all of them in
        one batched fit + one batched gradient per jitter attempt.  A failing output retries with the next jitter of
        the ladder while the others keep theirs (psd_safe_cholesky adds jitter only to the failing batch members
        [upstream]).  Returns (list of T host dicts, states).  Synchronises."""
        X = self._as_f64(X, "X")
        Y = self._as_f64(Y, "Y")
        T = Y.shape[1]
        level = [0] * T
        while True:
            pj = [p.replace(jitter=p.jitter + jitters[level[t]]) for t, p in enumerate(params)]
            states = self.fit_outputs(X, Y, pj, check=False, out=states, inverse=True)
            out = self.mll_grad_outputs(states, Y)
            v = out.cpu().numpy()
            info = states[0]._batch[4].cpu().numpy()
            bad = [t for t in range(T) if info[t] != 0]
            for t in bad:
                if info[t] < 0:
                    raise info_error(int(info[t]), f"output {t}")
            if not bad:
                break
            for t in bad:
                level[t] += 1
                if level[t] >= len(jitters):
                    raise NotPositiveDefiniteError(int(info[t]) - 1, f"output {t}: not positive definite at pivot "
                                                                     f"{int(info[t]) - 1} through the jitter ladder")
        d = X.shape[1]
        res = []
        for t in range(T):
            r = v[t]
            res.append({
                "nll": float(r[_capi.MLL_NLL]), "quad": float(r[_capi.MLL_QUAD]), "logdet": float(r[_capi.MLL_LOGDET]),
                "noise": float(r[_capi.MLL_D_NOISE]), "outputscale": float(r[_capi.MLL_D_OUTPUTSCALE]),
                "const_mean": float(r[_capi.MLL_D_MEAN]),
                "lengthscale": r[_capi.MLL_D_LENGTHSCALE:_capi.MLL_D_LENGTHSCALE + d].copy(),
                "linear_variance": r[_capi.MLL_D_LINVAR:_capi.MLL_D_LINVAR + d].copy(),
            })
        return res, states

    def mll_value_grad(self, X, y, params: KernelParams, jitters: Sequence[float] = (0.0, 1e-8, 1e-7, 1e-6),
                       state: Optional[GPState] = None):
        """Fit at ``params`` (retrying with the psd_safe_cholesky jitter ladder [upstream] on NOT_PD) and return
        (host dict of -log p(Y) and its gradient w.r.t. the natural hyperparameters, state).  Y: n or n x T
        (T outputs sharing the hyperparameters).  Synchronises."""
        X = self._as_f64(X, "X")
        y = self._as_f64(y, "y")
        # The gradient is queued right behind the fit and the pivot-failure word is read after both (one host round
        # trip per evaluation instead of two; a gradient computed on a failed factor is discarded).
        piv = -1
        for jit in jitters:
            # inverse=True: the gradient needs W = L^{-T}; the fused fit forms it from potrf's diagonal inverses and takes
            # alpha from it (no triangular solve whose alpha the gradient would not use)
            state = self.fit(X, y, params.replace(jitter=params.jitter + jit), check=False, out=state, inverse=True)
            out = self.mll_grad(state, y)
            v = out.cpu().numpy()
            piv = state.pivot_failure()
            if piv < 0:
                break
        else:
            raise NotPositiveDefiniteError(piv)
        d = X.shape[1]
        res = {
            "nll": float(v[_capi.MLL_NLL]), "quad": float(v[_capi.MLL_QUAD]), "logdet": float(v[_capi.MLL_LOGDET]),
            "noise": float(v[_capi.MLL_D_NOISE]), "outputscale": float(v[_capi.MLL_D_OUTPUTSCALE]),
            "const_mean": float(v[_capi.MLL_D_MEAN]),
            "lengthscale": v[_capi.MLL_D_LENGTHSCALE:_capi.MLL_D_LENGTHSCALE + d].copy(),
            "linear_variance": v[_capi.MLL_D_LINVAR:_capi.MLL_D_LINVAR + d].copy(),
        }
        return res, state

    # -- SVGP predictive + pool-scan selection --------------------------------
    def svgp_prepare(self, params: Sequence[KernelParams], Z, vmean, vchol, jitter: float = 1e-4):
        """Factor K_ZZ + jitter I per task and build the predictive caches of a trained batched SVGP
        (gpx_svgp_prepare_f64).  Z: T x M x d, vmean: T x M, vchol: T x M x M (lower triangle used).  Returns a dict
        of device tensors (W, W2, alpha, info, Z) consumed by ``svgp_predict``; raises NotPositiveDefiniteError."""
        Z = torch.as_tensor(Z).to(device=self.device, dtype=torch.float64).contiguous()
        vmean = torch.as_tensor(vmean).to(device=self.device, dtype=torch.float64).contiguous()
        vchol = torch.as_tensor(vchol).to(device=self.device, dtype=torch.float64).contiguous()
        T, M, d = Z.shape
        if vmean.shape != (T, M) or vchol.shape != (T, M, M):
            raise ValueError("vmean must be T x M and vchol T x M x M")
        if len(params) != T:
            raise ValueError(f"expected {T} kernel parameter sets, got {len(params)}")
        pcs = (KernelParamsC * T)(*[pp.to_c(d) for pp in params])
        Mpad = self.padded_n(M)
        W = torch.empty((T, Mpad, Mpad), dtype=torch.float64, device=self.device)
        W2 = torch.empty((T, Mpad, Mpad), dtype=torch.float64, device=self.device)
        alpha = torch.empty((T, Mpad), dtype=torch.float64, device=self.device)
        info = torch.zeros((T,), dtype=torch.int32, device=self.device)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_svgp_prepare_workspace_size(M, T, ctypes.byref(nbytes)))
        ws = self.workspace("svgp_prep", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_svgp_prepare_f64(
            self.handle, pcs, T, M, float(jitter), _ptr(Z), Z.stride(1), Z.stride(0), _ptr(vmean), vmean.stride(0),
            _ptr(vchol), vchol.stride(1), vchol.stride(0), _ptr(W), _ptr(W2), _ptr(alpha), _ptr(info), _ptr(ws),
            ws.numel()))
        bad = info.cpu().numpy()
        for t in range(T):
            err = info_error(int(bad[t]), f"task {t}: K_ZZ")
            if err is not None:
                raise err
        return {"Z": Z, "W": W, "W2": W2, "alpha": alpha, "params": list(params), "M": M}

    def svgp_predict(self, prep: dict, Xs, min_var: float = 1e-10, want=("mean", "var", "score")):
        """Predictive mean / variance (m x T, likelihood noise included) and the pool-scan score (m, sum over tasks
        of the variance) at input-transformed points Xs (gpx_svgp_predict_f64)."""
        Xs = self._as_f64(Xs, "Xs")
        Z = prep["Z"]
        T, M, d = Z.shape
        if Xs.shape[1] != d:
            raise ValueError(f"Xs has {Xs.shape[1]} columns, model has d={d}")
        m = Xs.shape[0]
        mean = torch.empty((m, T), dtype=torch.float64, device=self.device) if "mean" in want else None
        var = torch.empty((m, T), dtype=torch.float64, device=self.device) if "var" in want else None
        score = torch.empty((m,), dtype=torch.float64, device=self.device) if "score" in want else None
        pcs = (KernelParamsC * T)(*[pp.to_c(d) for pp in prep["params"]])
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_svgp_predict_workspace_size(M, m, ctypes.byref(nbytes)))
        ws = self.workspace("svgp_pred", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_svgp_predict_f64(
            self.handle, pcs, T, M, _ptr(Z), Z.stride(1), Z.stride(0), _ptr(prep["W"]), _ptr(prep["W2"]),
            _ptr(prep["alpha"]), _ptr(Xs), m, Xs.stride(0), float(min_var), _ptr(mean), T, _ptr(var), T, _ptr(score),
            _ptr(ws), ws.numel()))
        return mean, var, score

    def topk(self, scores: torch.Tensor, k: int):
        """(values, indices) of the k largest scores, descending, ties -> lower index first (gpx_topk_f64)."""
        scores = scores.to(device=self.device, dtype=torch.float64).contiguous().reshape(-1)
        m = scores.numel()
        idx = torch.empty((k,), dtype=torch.int64, device=self.device)
        val = torch.empty((k,), dtype=torch.float64, device=self.device)
        nbytes = ctypes.c_size_t()
        self._check(self.lib.gpx_topk_workspace_size(m, ctypes.byref(nbytes)))
        ws = self.workspace("topk", nbytes.value)
        self._bind_stream()
        self._check(self.lib.gpx_topk_f64(self.handle, _ptr(scores), m, int(k), _ptr(idx), _ptr(val), _ptr(ws),
                                          ws.numel()))
        return val, idx

    def fps(self, X, k: int, start: int) -> torch.Tensor:
        """Indices (selection order) of k farthest-point-sampled rows of X starting at row ``start`` (gpx_fps_f64)."""
        X = self._as_f64(X, "X")
        m, d = X.shape
        idx = torch.empty((k,), dtype=torch.int64, device=self.device)
        self._bind_stream()
        self._check(self.lib.gpx_fps_f64(self.handle, _ptr(X), m, d, X.stride(0), int(k), int(start), _ptr(idx)))
        return idx

    # -- instrumentation ------------------------------------------------------------------------
    def timing_enable(self, timers: Sequence[str] = ("trmm",)):
        mask = 0
        for t in timers:
            mask |= 1 << _capi.TIMERS[t]
        self._check(self.lib.gpx_timing_enable(self.handle, mask))

    def timing_disable(self):
        self._check(self.lib.gpx_timing_enable(self.handle, 0))

    def timing_reset(self):
        self._check(self.lib.gpx_timing_reset(self.handle))

    def timing_query(self, timer: str):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        self._check(self.lib.gpx_timing_query(self.handle, _capi.TIMERS[timer], ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value
