"""ctypes front end of oracle/selective_scan_ref.c (float64 selective scan forward + backward).

TEST INFRASTRUCTURE ONLY (the checker of tests/ at config-E lengths; parity unpinned at the
mamba_ssm level, pinned to oracle/selective_scan_ref.py by tests/test_selective_scan_oracle.py).
build() compiles the C file with gcc into oracle/lib/ (git-ignored, travels to the GPU box with
the snapshot like dna_amd/lib); __graft_entry__.build() calls it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "selective_scan_ref.c")
LIB = os.path.join(HERE, "lib", "libssref.so")
_lib = None


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", LIB, SRC, "-lm"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        for f in (_lib.ssref_fwd, _lib.ssref_bwd):
            f.restype = ctypes.c_int
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f64(a):
    return None if a is None else np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def scan_fwd(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False):
    """-> (out [b,d,l], last_state [b,d,n]) in float64 (numpy inputs of any float dtype)."""
    u, delta, A, B, C, D, z, delta_bias = map(_f64, (u, delta, A, B, C, D, z, delta_bias))
    b, d, l = u.shape
    n = A.shape[1]
    out = np.empty((b, d, l))
    last = np.empty((b, d, n))
    rc = lib().ssref_fwd(_p(u), _p(delta), _p(A), _p(B), _p(C), _p(D), _p(z), _p(delta_bias),
                         int(bool(delta_softplus)), b, d, l, n, _p(out), _p(last))
    if rc:
        raise MemoryError("ssref_fwd")
    return out, last


def scan_bwd(u, delta, A, B, C, dout, D=None, z=None, delta_bias=None, delta_softplus=False):
    """-> dict of float64 gradients: u, delta, A, B, C (+ D, z, delta_bias when given)."""
    u, delta, A, B, C, D, z, delta_bias, dout = map(_f64, (u, delta, A, B, C, D, z, delta_bias, dout))
    b, d, l = u.shape
    n = A.shape[1]
    g = {"u": np.empty_like(u), "delta": np.empty_like(u), "A": np.empty_like(A),
         "B": np.empty_like(B), "C": np.empty_like(C)}
    if D is not None:
        g["D"] = np.empty_like(D)
    if z is not None:
        g["z"] = np.empty_like(z)
    if delta_bias is not None:
        g["delta_bias"] = np.empty_like(delta_bias)
    rc = lib().ssref_bwd(_p(u), _p(delta), _p(A), _p(B), _p(C), _p(D), _p(z), _p(delta_bias),
                         int(bool(delta_softplus)), b, d, l, n, _p(dout), _p(g["u"]),
                         _p(g["delta"]), _p(g["A"]), _p(g["B"]), _p(g["C"]), _p(g.get("D")),
                         _p(g.get("z")), _p(g.get("delta_bias")))
    if rc:
        raise MemoryError("ssref_bwd")
    return g


class _ScanC:
    """torch.autograd.Function over scan_fwd / scan_bwd (float64 CPU tensors)."""
    fn = None


def _make_fn():
    import torch

    class ScanC(torch.autograd.Function):
        @staticmethod
        def forward(ctx, u, delta, A, B, C, D, z, delta_bias, softplus):
            np_in = [None if t is None else t.detach().double().numpy()
                     for t in (u, delta, A, B, C, D, z, delta_bias)]
            out, _ = scan_fwd(*np_in[:5], D=np_in[5], z=np_in[6], delta_bias=np_in[7],
                              delta_softplus=softplus)
            ctx.np_in, ctx.softplus = np_in, softplus
            ctx.has = [t is not None for t in (D, z, delta_bias)]
            return torch.from_numpy(out)

        @staticmethod
        def backward(ctx, dout):
            u, delta, A, B, C, D, z, bias = ctx.np_in
            g = scan_bwd(u, delta, A, B, C, dout.detach().double().numpy(), D=D, z=z,
                         delta_bias=bias, delta_softplus=ctx.softplus)
            t = lambda k: torch.from_numpy(g[k]) if k in g else None
            return t("u"), t("delta"), t("A"), t("B"), t("C"), t("D"), t("z"), t("delta_bias"), None

    return ScanC


def selective_scan_c(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                     return_last_state=False):
    """Drop-in for oracle.selective_scan_ref.selective_scan_ref (float64, autograd through the C
    backward) at lengths the Python loop cannot reach."""
    if return_last_state:
        raise NotImplementedError("selective_scan_c: return_last_state (use scan_fwd)")
    if _ScanC.fn is None:
        _ScanC.fn = _make_fn()
    return _ScanC.fn.apply(u, delta, A, B, C, D, z, delta_bias, bool(delta_softplus))
