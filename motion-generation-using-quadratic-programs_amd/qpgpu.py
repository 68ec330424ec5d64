"""qpgpu — Python host mirror of the batched solve_quadprog() C-ABI (include/qpgpu.h).

The reference interface this mirrors is the solver call at reference src/mgqp.cpp:708
(``solve_quadprog(G, g0, t(CE), ce0, t(CI), ci0, x)``, declared at
include/QuadProgpp/QuadProg++.hh:69-72), batched: the same argument meanings, the same sign
convention (``CE^T x + ce0 = 0``, ``CI^T x + ci0 >= 0``), the same "G is overwritten" option,
and the same error outcomes, reported per QP as status codes instead of exceptions
(``solve_quadprog`` in this module re-raises them exactly like the reference for one QP).

Every solve runs on the gfx950 HIP kernels in ``lib/libqpgpu.so``.  If that library is missing
this module raises at import time; there is no CPU fallback.

Also hosts the synthetic problem generator of SURVEY.md §8(d): a counter-based SplitMix64
stream keyed by (seed, qp_index, stream, element), so any shard of a batch can be generated
independently and identically on every rank.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
LIB_PATH = os.environ.get("QPGPU_LIB_PATH") or os.path.join(LIB_DIR, "libqpgpu.so")  # env: A/B builds only
DROPIN_PATH = os.path.join(LIB_DIR, "libquadprog_amd.so")

# per-QP status codes (include/qpgpu.h)
QP_OK = 0
QP_INFEASIBLE = 1
QP_NOT_POSITIVE_DEFINITE = 2
QP_DEPENDENT = 3
QP_MAX_ITER = 4
STATUS_NAMES = {0: "ok", 1: "infeasible", 2: "not_positive_definite", 3: "dependent", 4: "max_iter"}

# API return codes
SUCCESS = 0
ERR_INVALID_ARGUMENT = 1
ERR_UNSUPPORTED_SHAPE = 2
ERR_HIP = 3
ERR_NO_DEVICE = 4

FLAG_WRITE_FACTOR = 0x1
FLAG_EXACT = 0x2  # reference operation order for n > 64 too (no MFMA panel setup)
FLAG_FAST = 0x4  # lane-kernel shapes: fused multiply-adds, shared reciprocals (1e-10, not bitwise)
FLAG_FORCE_LANE = 0x100
FLAG_FORCE_SUBGROUP = 0x200
FLAG_FORCE_WAVE = 0x400
FLAG_FORCE_GENERIC = 0x800  # any shape: the generic workspace kernel (qp_generic.hip)
FAMILY_FLAGS = {None: 0, "auto": 0, "lane": FLAG_FORCE_LANE, "subgroup": FLAG_FORCE_SUBGROUP,
                "wave": FLAG_FORCE_WAVE, "generic": FLAG_FORCE_GENERIC}
LAYOUT_QP_MAJOR = 0
LAYOUT_TILED64 = 1
LAYOUTS = {None: 0, "qp_major": LAYOUT_QP_MAJOR, "tiled64": LAYOUT_TILED64}

EXPORTED_SYMBOLS = (
    "qpgpu_solve_batched",
    "qpgpu_solve_batched_eq",
    "qpgpu_solve_batched_host",
    "qpgpu_max_n",
    "qpgpu_max_m",
    "qpgpu_kernel_name",
    "qpgpu_kernel_name_flags",
    "qpgpu_last_error",
    "qpgpu_device_count",
    "qpgpu_abi_version",
    "qpgpu_relayout",
    "qpgpu_solve_batched_multi",
)


class QpgpuError(RuntimeError):
    pass


class ProblemDesc(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32),
        ("p", ctypes.c_int32),
        ("m", ctypes.c_int32),
        ("max_iter", ctypes.c_int32),
        ("batch", ctypes.c_int64),
        ("flags", ctypes.c_uint32),
        ("layout", ctypes.c_uint32),
    ]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"qpgpu: {LIB_PATH} is missing; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp = ctypes.c_void_p
    lib.qpgpu_solve_batched.argtypes = [ctypes.POINTER(ProblemDesc)] + [vp] * 11
    lib.qpgpu_solve_batched.restype = ctypes.c_int
    lib.qpgpu_solve_batched_eq.argtypes = [ctypes.POINTER(ProblemDesc)] + [vp] * 14
    lib.qpgpu_solve_batched_eq.restype = ctypes.c_int
    lib.qpgpu_solve_batched_host.argtypes = [ctypes.POINTER(ProblemDesc)] + [vp] * 10
    lib.qpgpu_solve_batched_host.restype = ctypes.c_int
    lib.qpgpu_solve_batched_multi.argtypes = [ctypes.POINTER(ProblemDesc), ctypes.c_int32, vp] + [vp] * 10
    lib.qpgpu_solve_batched_multi.restype = ctypes.c_int
    lib.qpgpu_kernel_name.argtypes = [ctypes.c_int32] * 3
    lib.qpgpu_kernel_name.restype = ctypes.c_char_p
    lib.qpgpu_kernel_name_flags.argtypes = [ctypes.c_int32] * 3 + [ctypes.c_uint32]
    lib.qpgpu_kernel_name_flags.restype = ctypes.c_char_p
    lib.qpgpu_last_error.restype = ctypes.c_char_p
    lib.qpgpu_max_n.restype = ctypes.c_int
    lib.qpgpu_max_m.restype = ctypes.c_int
    lib.qpgpu_device_count.restype = ctypes.c_int
    lib.qpgpu_abi_version.restype = ctypes.c_int
    lib.qpgpu_relayout.argtypes = [ctypes.c_int64, ctypes.c_int32, vp, vp, ctypes.c_int32, vp]
    lib.qpgpu_relayout.restype = ctypes.c_int
    return lib


LIB = _load()


def build_provenance() -> dict:
    """Which sources the loaded libqpgpu.so was built from: the md5 of the library, the sha256 the
    Makefile recorded over its sources at link time (lib/libqpgpu.sources), the sha256 of those
    files now, and whether they match (False: the library is older than its sources — rebuild;
    None: the record or the sources are absent, e.g. an A/B library)."""
    import hashlib

    rec = os.path.join(os.path.dirname(LIB_PATH), "libqpgpu.sources")
    out = {"lib": os.path.relpath(LIB_PATH, os.path.dirname(LIB_DIR)),
           "lib_md5": hashlib.md5(open(LIB_PATH, "rb").read()).hexdigest(),
           "sources_sha256_at_build": None, "sources_sha256_now": None, "matches_sources": None}
    try:
        files, sha = open(rec).read().split("\n")[:2]
    except (OSError, ValueError):
        return out
    out["sources_sha256_at_build"] = sha.strip()
    pkg = os.path.dirname(LIB_DIR)
    try:
        h = hashlib.sha256()
        for f in files.split():
            h.update(open(os.path.join(pkg, f), "rb").read())
        out["sources_sha256_now"] = h.hexdigest()
        out["matches_sources"] = out["sources_sha256_now"] == out["sources_sha256_at_build"]
    except OSError:
        pass
    return out


def kernel_name(n: int, p: int, m: int, fast: bool = False) -> str:
    if fast:
        return LIB.qpgpu_kernel_name_flags(n, p, m, FLAG_FAST).decode()
    return LIB.qpgpu_kernel_name(n, p, m).decode()


# the n > 64 default path's certification: a QP whose decisions the tolerance mode
# cannot certify carries STATUS_RESOLVE | reasons << 9 until the EXACT re-solve rewrites it
STATUS_RESOLVE = 0x100
UNC_REASONS = ("dependent", "setup", "max_iter", "step_tie", "zz", "t_t2", "select_tie", "psi",
               "f_cancel", "x_cancel", "non_finite", "t1_tie", "givens")


def set_resolve(on: bool) -> None:
    """Test / diagnostic hook: False skips the EXACT re-solve of uncertified n > 64 QPs and leaves
    their marks in the status words (see unc_reasons)."""
    fn = LIB.qpgpu_debug_set_resolve
    fn.argtypes = [ctypes.c_int]
    fn(1 if on else 0)


def set_shadow(on: bool) -> None:
    """Test / diagnostic hook: False makes the n > 64 default path's l1 scans fp64-only instead of
    reading the fp32 copy of CI first; results are the same bit for bit."""
    fn = LIB.qpgpu_debug_set_shadow
    fn.argtypes = [ctypes.c_int]
    fn(1 if on else 0)


def shadow_stats(reset: bool = True) -> tuple:
    """(l1 scans of the n > 64 default path that tried the fp32 copy of CI, scans it settled, fp64
    re-evaluations of candidates in those) since the last reset; synchronises the device."""
    fn = LIB.qpgpu_debug_shadow_stats
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    fn.restype = ctypes.c_int
    out = (ctypes.c_uint64 * 3)()
    rc = fn(out, 1 if reset else 0)
    if rc:
        raise QpgpuError(f"qpgpu_debug_shadow_stats: {rc} {LIB.qpgpu_last_error().decode()}")
    return int(out[0]), int(out[1]), int(out[2])


def unc_reasons(status: np.ndarray) -> dict:
    """Counts of each certification reason in status words returned with set_resolve(False)."""
    st = np.asarray(status, dtype=np.int64)
    marked = (st & STATUS_RESOLVE) != 0
    out = {"marked": int(marked.sum())}
    for k, name in enumerate(UNC_REASONS):
        c = int((marked & (((st >> 9) >> k) & 1).astype(bool)).sum())
        if c:
            out[name] = c
    return out


def device_count() -> int:
    return int(LIB.qpgpu_device_count())


def _check(rc: int, what: str):
    if rc != SUCCESS:
        detail = LIB.qpgpu_last_error().decode() if rc in (ERR_HIP, ERR_NO_DEVICE) else ""
        raise QpgpuError(f"{what} failed with code {rc} {detail}".strip())


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


# ----------------------------------------------------------------------------------------------
# problem container
# ----------------------------------------------------------------------------------------------
@dataclass
class Problems:
    """A batch of QPs in the include/qpgpu.h layout (numpy float64, QP-major, row-major)."""

    n: int
    p: int
    m: int
    G: np.ndarray  # (B, n, n)
    g0: np.ndarray  # (B, n)
    CE: np.ndarray  # (B, n, p)
    ce0: np.ndarray  # (B, p)
    CI: np.ndarray  # (B, n, m)
    ci0: np.ndarray  # (B, m)

    @property
    def batch(self) -> int:
        return int(self.G.shape[0])

    def slice(self, b0: int, b1: int) -> "Problems":
        return Problems(self.n, self.p, self.m, self.G[b0:b1].copy(), self.g0[b0:b1].copy(),
                        self.CE[b0:b1].copy(), self.ce0[b0:b1].copy(), self.CI[b0:b1].copy(),
                        self.ci0[b0:b1].copy())

    def arrays(self):
        return (self.G, self.g0, self.CE, self.ce0, self.CI, self.ci0)


def to_tiled64(a: np.ndarray) -> np.ndarray:
    """(B, ...) per-QP blocks -> TILED64 flat array of ceil(B/64) tiles (include/qpgpu.h)."""
    B = a.shape[0]
    E = int(np.prod(a.shape[1:])) if a.ndim > 1 else 1
    BB = (B + 63) // 64 * 64
    pad = np.zeros((BB, E), dtype=np.float64)
    pad[:B] = a.reshape(B, E)
    return np.ascontiguousarray(pad.reshape(BB // 64, 64, E).transpose(0, 2, 1)).reshape(-1)


def from_tiled64(flat: np.ndarray, B: int, shape) -> np.ndarray:
    """Inverse of to_tiled64: returns (B, *shape)."""
    E = int(np.prod(shape)) if len(shape) else 1
    BB = (B + 63) // 64 * 64
    t = np.asarray(flat).reshape(BB // 64, E, 64).transpose(0, 2, 1).reshape(BB, E)
    return np.ascontiguousarray(t[:B]).reshape((B,) + tuple(shape))


def rel_error_per_qp(x, x_ref, f, f_ref, tiny: float = np.finfo(np.float64).tiny, f_scale=None):
    """north_star's parity measure ("primal/objective within 1e-10 relative"), per QP:
    ex_i = ||x_i - xref_i||_inf / max(||xref_i||_inf, tiny), ef_i = |f_i - fref_i| / max(|fref_i|, tiny).
    With f_scale (per QP, objective_term_scale()), ef_i is relative to max(|fref_i|, f_scale_i): the
    magnitude of the objective's terms, which is the scale f is determined to when its two terms
    cancel.  Entries that are equal (inf == inf included) or NaN in both count as 0.  Returns the
    arrays (ex, ef) so callers can report max, percentiles and the worst QP."""
    if len(f) == 0:
        return np.zeros(0), np.zeros(0)
    x = np.asarray(x, dtype=np.float64).reshape(len(f), -1)
    xr = np.asarray(x_ref, dtype=np.float64).reshape(len(f_ref), -1)
    f = np.asarray(f, dtype=np.float64)
    fr = np.asarray(f_ref, dtype=np.float64)
    with np.errstate(invalid="ignore", over="ignore"):
        dx = np.abs(x - xr)
        dx[(x == xr) | (np.isnan(x) & np.isnan(xr))] = 0.0
        nx = np.max(np.abs(np.where(np.isnan(xr), 0.0, xr)), axis=1) if xr.shape[1] else np.zeros(len(xr))
        ex = (np.max(dx, axis=1) if xr.shape[1] else np.zeros(len(xr))) / np.maximum(nx, tiny)
        df = np.abs(f - fr)
        df[(f == fr) | (np.isnan(f) & np.isnan(fr))] = 0.0
        den = np.maximum(np.abs(np.where(np.isnan(fr), 0.0, fr)), tiny)
        if f_scale is not None:
            den = np.maximum(den, np.where(np.isfinite(f_scale), f_scale, 0.0))
        ef = df / den
    ex[np.isnan(ex)] = np.inf  # one side NaN only
    ef[np.isnan(ef)] = np.inf
    return ex, ef


def objective_term_scale(G, g0, x):
    """Per QP, 0.5 |x^T G x| + |g0^T x|: the magnitudes of the two terms whose sum is the objective
    f = 0.5 x^T G x + g0^T x (G the original matrix, x the reference solution).  When they cancel,
    f itself is only determined to ~eps times this scale (the reference's own rounding), so the
    objective's relative error is measured against max(|f|, this)."""
    G = np.asarray(G, dtype=np.float64)
    if G.shape[0] == 0:
        return np.zeros(0)
    x = np.asarray(x, dtype=np.float64).reshape(G.shape[0], -1)
    g0 = np.asarray(g0, dtype=np.float64).reshape(G.shape[0], -1)
    with np.errstate(invalid="ignore", over="ignore"):
        return 0.5 * np.abs(np.einsum("bi,bij,bj->b", x, G, x)) + np.abs(np.einsum("bi,bi->b", g0, x))


def algorithmic_bytes_per_qp(n: int, p: int, m: int) -> int:
    """read G, g0, CE, ce0, CI, ci0; write x and f (status excluded)."""
    return 8 * (n * n + n + n * p + p + n * m + m) + 8 * (n + 1)


# ----------------------------------------------------------------------------------------------
# host-pointer solve (numpy in, numpy out) — copies through the C-ABI's host entry point
# ----------------------------------------------------------------------------------------------
def _host_call(d, arrs, outs, devices):
    """qpgpu_solve_batched_host, or qpgpu_solve_batched_multi over `devices` (device ids)."""
    if devices is None:
        return LIB.qpgpu_solve_batched_host(ctypes.byref(d), *[_ptr(a) for a in arrs], *[_ptr(o) for o in outs])
    dv = np.ascontiguousarray(devices, dtype=np.int32)
    return LIB.qpgpu_solve_batched_multi(ctypes.byref(d), len(dv), _ptr(dv), *[_ptr(a) for a in arrs],
                                         *[_ptr(o) for o in outs])


def solve_batched_host(pr: Problems, write_factor: bool = False, max_iter: int = 0, family=None,
                       layout=None, exact: bool = False, fast: bool = False, devices=None):
    """Solve every QP of `pr` on the GPU.  Returns (x, f, status, iters).

    With write_factor=True, pr.G is overwritten with each QP's Cholesky factor, as the
    reference overwrites G (QuadProg++.hh:42-45).  layout="tiled64" sends the batch in the
    TILED64 layout (converted here on the host) and converts x / G back.  exact=True keeps the
    reference's operation order for n > 64 as well (QPGPU_FLAG_EXACT); fast=True runs the lane
    kernel's fast build (QPGPU_FLAG_FAST: within 1e-10, not bitwise).  devices=[d0, d1, ...]
    splits the batch into contiguous shards over those GPUs (qpgpu_solve_batched_multi)."""
    B, n, p, m = pr.batch, pr.n, pr.p, pr.m
    xflags = FAMILY_FLAGS[family] | (FLAG_EXACT if exact else 0) | (FLAG_FAST if fast else 0)
    if LAYOUTS[layout] == LAYOUT_TILED64:
        arrs = [to_tiled64(np.asarray(a, dtype=np.float64)) for a in pr.arrays()]
        xt = np.zeros((B + 63) // 64 * 64 * n, dtype=np.float64)
        f = np.zeros(B, dtype=np.float64)
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros(B, dtype=np.int32)
        d = ProblemDesc(n, p, m, max_iter, B,
                        (FLAG_WRITE_FACTOR if write_factor else 0) | xflags, LAYOUT_TILED64)
        rc = _host_call(d, arrs, (xt, f, st, it), devices)
        _check(rc, "qpgpu_solve_batched_host")
        if write_factor:
            pr.G[...] = from_tiled64(arrs[0], B, (n, n))
        return from_tiled64(xt, B, (n,)), f, st, it
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in pr.arrays()]
    if write_factor:
        if not (pr.G.flags.c_contiguous and pr.G.dtype == np.float64):
            raise ValueError("write_factor needs a C-contiguous float64 G")
        arrs[0] = pr.G
    x = np.zeros((B, n), dtype=np.float64)
    f = np.zeros(B, dtype=np.float64)
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    d = ProblemDesc(n, p, m, max_iter, B, (FLAG_WRITE_FACTOR if write_factor else 0) | xflags, 0)
    rc = _host_call(d, arrs, (x, f, st, it), devices)
    _check(rc, "qpgpu_solve_batched_host")
    return x, f, st, it


# ----------------------------------------------------------------------------------------------
# device-pointer solve (torch tensors already resident in HBM)
# ----------------------------------------------------------------------------------------------
class DeviceBatch:
    """Device-resident inputs/outputs for repeated solves (torch tensors on one GPU)."""

    def __init__(self, pr: Problems, device, with_iters: bool = True, layout=None):
        import torch

        self.n, self.p, self.m, self.batch = pr.n, pr.p, pr.m, pr.batch
        self.layout = LAYOUTS[layout]
        conv = to_tiled64 if self.layout == LAYOUT_TILED64 else (lambda a: a)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(conv(np.asarray(a, dtype=np.float64)))).to(device)
        self.G, self.g0, self.CE, self.ce0, self.CI, self.ci0 = (t(a) for a in pr.arrays())
        rows = (self.batch + 63) // 64 * 64 if self.layout == LAYOUT_TILED64 else self.batch
        self.x = torch.zeros((rows, self.n), dtype=torch.float64, device=device)
        self.f = torch.zeros(self.batch, dtype=torch.float64, device=device)
        self.status = torch.zeros(self.batch, dtype=torch.int32, device=device)
        self.iters = torch.zeros(self.batch, dtype=torch.int32, device=device) if with_iters else None

    def solve(self, stream=None, max_iter: int = 0, write_factor: bool = False, family=None,
              eq_out=None, exact: bool = False, fast: bool = False):
        """Enqueue one batched solve on `stream` (a torch.cuda.Stream, default current).
        eq_out=(x_eq, f_eq, status_eq) tensors also receive the m = 0 answer
        (qpgpu_solve_batched_eq)."""
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(self.x.device)
        d = ProblemDesc(self.n, self.p, self.m, max_iter, self.batch,
                        (FLAG_WRITE_FACTOR if write_factor else 0) | FAMILY_FLAGS[family]
                        | (FLAG_EXACT if exact else 0) | (FLAG_FAST if fast else 0), self.layout)
        vp = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
        args = [ctypes.byref(d), vp(self.G), vp(self.g0), vp(self.CE), vp(self.ce0), vp(self.CI),
                vp(self.ci0), vp(self.x), vp(self.f), vp(self.status), vp(self.iters)]
        if eq_out is None:
            rc = LIB.qpgpu_solve_batched(*args, ctypes.c_void_p(stream.cuda_stream))
        else:
            rc = LIB.qpgpu_solve_batched_eq(*args, *[vp(t) for t in eq_out],
                                            ctypes.c_void_p(stream.cuda_stream))
        _check(rc, "qpgpu_solve_batched")

    def launcher(self, stream, max_iter: int = 0, family=None, exact: bool = False, fast: bool = False):
        """A zero-argument callable that enqueues this batch's solve on `stream` with every ctypes
        argument prebuilt (for tight launch loops: ~2 us of host time per launch)."""
        d = ProblemDesc(self.n, self.p, self.m, max_iter, self.batch,
                        FAMILY_FLAGS[family] | (FLAG_EXACT if exact else 0) | (FLAG_FAST if fast else 0),
                        self.layout)
        vp = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
        args = (ctypes.byref(d), vp(self.G), vp(self.g0), vp(self.CE), vp(self.ce0), vp(self.CI),
                vp(self.ci0), vp(self.x), vp(self.f), vp(self.status), vp(self.iters),
                ctypes.c_void_p(stream.cuda_stream))
        fn = LIB.qpgpu_solve_batched

        def launch():
            rc = fn(*args)
            if rc != SUCCESS:
                _check(rc, "qpgpu_solve_batched")

        launch._keep = (d, self)
        return launch

    def results(self):
        it = None if self.iters is None else self.iters.cpu().numpy()
        x = self.x.cpu().numpy()
        if self.layout == LAYOUT_TILED64:
            x = from_tiled64(x.reshape(-1), self.batch, (self.n,))
        return x, self.f.cpu().numpy(), self.status.cpu().numpy(), it


def relayout(src, dst, batch: int, elems: int, to_tiled: bool, stream=None):
    """Device conversion of one per-QP array between layouts (torch tensors)."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(src.device)
    rc = LIB.qpgpu_relayout(batch, elems, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                            1 if to_tiled else 0, ctypes.c_void_p(stream.cuda_stream))
    _check(rc, "qpgpu_relayout")


# ----------------------------------------------------------------------------------------------
# synthetic problems, counter-based so shards regenerate identically
# ----------------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform01(seed: int, idx: np.ndarray, stream: int, count: int) -> np.ndarray:
    """(len(idx), count) uniforms in (0, 1], keyed by (seed, qp index, stream, element)."""
    idx = idx.astype(np.uint64)[:, None]
    k = np.arange(count, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ np.uint64(0x5851F42D4C957F2D * (stream + 1) & 0xFFFFFFFFFFFFFFFF))
        c = (idx << np.uint64(24)) + k
        bits = _splitmix64(_splitmix64(c) ^ key)
    return ((bits >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)


def _normal(seed: int, idx: np.ndarray, stream: int, count: int) -> np.ndarray:
    u1 = _uniform01(seed, idx, 2 * stream, count)
    u2 = _uniform01(seed, idx, 2 * stream + 1, count)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


def make_problems(kind: str, n: int, p: int, m: int, b0: int, b1: int, seed: int = 2026,
                  threads: int = 0) -> Problems:
    """Generate QPs [b0, b1) of a synthetic batch.

    kind="general" (C1, C3, C4, C5): G = M^T M + n I, g0 ~ 10 N(0,1), feasible point
        x_f ~ 0.1 N(0,1), CE ~ N(0,1), ce0 = -CE^T x_f, CI ~ N(0,1), ci0 = -CI^T x_f + |N(0,1)|.
    kind="box" (C2, mgqp joint-limit ordering, reference src/mgqp.cpp:1111-1112): same G, g0, CE;
        CI = [-I, +I] (m = 2n), ci0 = [hi; -lo] with hi = -lo = 1.

    Every QP depends only on (seed, its global index), so large ranges are generated in chunks
    on `threads` host threads (0 = up to 8; numpy releases the GIL) with identical results.
    """
    B = b1 - b0
    chunk = 8192
    if threads == 0:
        threads = min(8, os.cpu_count() or 1)
    if threads > 1 and B > 2 * chunk:
        from concurrent.futures import ThreadPoolExecutor

        cuts = list(range(b0, b1, chunk)) + [b1]
        with ThreadPoolExecutor(threads) as ex:
            parts = list(ex.map(lambda c: _make_range(kind, n, p, m, c[0], c[1], seed),
                                zip(cuts[:-1], cuts[1:])))
        cat = lambda k: np.concatenate([getattr(q, k) for q in parts])
        return Problems(n, p, m, cat("G"), cat("g0"), cat("CE"), cat("ce0"), cat("CI"), cat("ci0"))
    return _make_range(kind, n, p, m, b0, b1, seed)


def _make_range(kind: str, n: int, p: int, m: int, b0: int, b1: int, seed: int) -> Problems:
    idx = np.arange(b0, b1, dtype=np.uint64)
    B = b1 - b0
    M = _normal(seed, idx, 0, n * n).reshape(B, n, n)
    G = np.einsum("bki,bkj->bij", M, M) + n * np.eye(n)[None]
    g0 = 10.0 * _normal(seed, idx, 1, n)
    xf = 0.1 * _normal(seed, idx, 2, n)
    CE = _normal(seed, idx, 3, n * p).reshape(B, n, p)
    ce0 = -np.einsum("bnp,bn->bp", CE, xf)
    if kind == "general":
        CI = _normal(seed, idx, 4, n * m).reshape(B, n, m)
        ci0 = -np.einsum("bnm,bn->bm", CI, xf) + np.abs(_normal(seed, idx, 5, m))
    elif kind == "box":
        if m != 2 * n:
            raise ValueError("box problems need m = 2n")
        eye = np.eye(n)
        CI = np.broadcast_to(np.concatenate([-eye, eye], axis=1), (B, n, m)).copy()
        ci0 = np.ones((B, m))
    else:
        raise ValueError(kind)
    return Problems(n, p, m, np.ascontiguousarray(G), np.ascontiguousarray(g0),
                    np.ascontiguousarray(CE), np.ascontiguousarray(ce0), np.ascontiguousarray(CI),
                    np.ascontiguousarray(ci0))


# ----------------------------------------------------------------------------------------------
# one QP, reference semantics (exceptions instead of status codes)
# ----------------------------------------------------------------------------------------------
def solve_quadprog(G: np.ndarray, g0, CE, ce0, CI, ci0):
    """Single-QP mirror of the reference call: returns (f, x); overwrites G with its Cholesky
    factor; raises ValueError/RuntimeError where the reference raises logic_error/runtime_error.
    CE is n x p and CI is n x m (the t(CE) / t(CI) mgqp passes)."""
    G = np.asarray(G)
    n = G.shape[1]
    CE = np.asarray(CE, dtype=np.float64).reshape(n, -1) if np.size(CE) else np.zeros((n, 0))
    CI = np.asarray(CI, dtype=np.float64).reshape(n, -1) if np.size(CI) else np.zeros((n, 0))
    p, m = CE.shape[1], CI.shape[1]
    if G.shape[0] != n:
        raise ValueError(f"The matrix G is not a squared matrix ({G.shape[0]} x {G.shape[1]})")
    ce0 = np.asarray(ce0, dtype=np.float64).reshape(-1)
    ci0 = np.asarray(ci0, dtype=np.float64).reshape(-1)
    if ce0.size != p:
        raise ValueError(f"The vector ce0 is incompatible (incorrect dimension {ce0.size}, expecting {p})")
    if ci0.size != m:
        raise ValueError(f"The vector ci0 is incompatible (incorrect dimension {ci0.size}, expecting {m})")
    Gc = np.ascontiguousarray(G, dtype=np.float64).reshape(1, n, n).copy()
    pr = Problems(n, p, m, Gc, np.asarray(g0, dtype=np.float64).reshape(1, n), CE.reshape(1, n, p),
                  ce0.reshape(1, p), CI.reshape(1, n, m), ci0.reshape(1, m))
    x, f, st, _ = solve_batched_host(pr, write_factor=True)
    if G.dtype == np.float64 and G.flags.c_contiguous:
        G[...] = Gc[0]
    s = int(st[0])
    if s == QP_NOT_POSITIVE_DEFINITE:
        raise ValueError(f"Error in cholesky decomposition, sum: {f[0]:g}")
    if s == QP_DEPENDENT:
        raise RuntimeError("Constraints are linearly dependent")
    if s == QP_MAX_ITER:
        raise RuntimeError("qpgpu: active-set step cap reached")
    return float(f[0]), x[0]
