"""The RCPS restatement (oracle/caduceus_ref.py rcps_*) against the reference's own RCPS modules
(tests/golden/rcps_golden.npz, written by tests/golden/make_rcps_golden.py from
/root/reference/src/models/caduceus/modeling_rcps.py): outputs and every input / parameter
gradient, float64, CPU."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import caduceus_ref as C
from tests.conftest import GOLDEN

Z = np.load(os.path.join(GOLDEN, "rcps_golden.npz"))
T = lambda k, grad=False: torch.tensor(Z[k]).requires_grad_(grad)


def _close(a, k, tol=1e-12):
    ref = Z[k]
    a = a.detach().numpy()
    assert a.shape == ref.shape, (k, a.shape, ref.shape)
    err = np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-30)
    assert err <= tol, (k, err)


def _grad(outs, gouts, ts):
    return torch.autograd.grad(outs, ts, gouts)


def test_rcps_embedding():
    W = T("emb_W", True)
    y = C.rcps_embedding(W, torch.tensor(Z["complement"]), torch.tensor(Z["emb_ids"]))
    _close(y, "emb_out")
    (dW,) = _grad(y, T("emb_gout"), [W])
    _close(dW, "emb_dW")


def test_rcps_wrapper():
    x, W, b = T("wrap_x", True), T("wrap_W", True), T("wrap_b", True)
    y = C.rcps_wrapper(lambda t: F.linear(t, W, b), x)
    _close(y, "wrap_out")
    for g, k in zip(_grad(y, T("wrap_gout"), [x, W, b]), ("wrap_dx", "wrap_dW", "wrap_db")):
        _close(g, k)


@pytest.mark.parametrize("tag", ["an0", "an"])
def test_rcps_add_norm(tag):
    x, g, b = T(f"{tag}_x", True), T(f"{tag}_g", True), T(f"{tag}_beta", True)
    res = T(f"{tag}_res", True) if f"{tag}_res" in Z else None
    y, r = C.rcps_add_norm(lambda t: F.layer_norm(t, (t.shape[-1],), g, b, 1e-5), x, res)
    _close(y, f"{tag}_y")
    _close(r, f"{tag}_res_out")
    ts = [x, g, b] + ([res] if res is not None else [])
    grads = _grad((y, r), (T(f"{tag}_gy"), T(f"{tag}_gres")), ts)
    for gr, k in zip(grads, ("dx", "dg", "dbeta", "dres")):
        _close(gr, f"{tag}_{k}")


@pytest.mark.parametrize("tag", ["blk0", "blk"])
def test_rcps_block_nonfused(tag):
    h = T(f"{tag}_h", True)
    ng, nb = T(f"{tag}_norm_g", True), T(f"{tag}_norm_b", True)
    mW, mb = T(f"{tag}_mix_W", True), T(f"{tag}_mix_b", True)
    res = T(f"{tag}_res", True) if f"{tag}_res" in Z else None
    hh, rr = C.rcps_block(lambda t: F.layer_norm(t, (t.shape[-1],), ng, nb, 1e-5),
                          lambda t: F.linear(t, mW, mb), h, res, fused_add_norm=False,
                          residual_in_fp32=True)
    _close(hh, f"{tag}_h_out")
    _close(rr, f"{tag}_res_out")
    ts = [h, ng, nb, mW, mb] + ([res] if res is not None else [])
    grads = _grad((hh, rr), (T(f"{tag}_gh"), T(f"{tag}_gres")), ts)
    for gr, k in zip(grads, ("dh", "dnorm_g", "dnorm_b", "dmix_W", "dmix_b", "dres")):
        _close(gr, f"{tag}_{k}")


def test_rcps_lm_head():
    x, W = T("head_x", True), T("head_W", True)
    y = C.rcps_lm_head(W, torch.tensor(Z["complement"]), x)
    _close(y, "head_out")
    for g, k in zip(_grad(y, T("head_gout"), [x, W]), ("head_dx", "head_dW")):
        _close(g, k)
