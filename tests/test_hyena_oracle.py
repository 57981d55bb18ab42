"""CPU: the FFT long-conv oracle (oracle/hyena_ref.py) against fixtures produced by the
reference's own fftconv_ref (tests/golden/make_hyena_golden.py), and against the O(L^2) definition."""
import os

import numpy as np
import pytest
import torch

from oracle import hyena_ref as H

GOLD = os.path.join(os.path.dirname(__file__), "golden", "fftconv_golden.npz")


def _cases():
    z = np.load(GOLD)
    for c in range(int(z["ncases"])):
        p = f"c{c}_"
        B, D, L, bi = (int(v) for v in z[p + "shape"])
        yield c, B, D, L, bool(bi), {k[len(p):]: z[k] for k in z.files if k.startswith(p)}


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: f"c{c[0]}_B{c[1]}D{c[2]}L{c[3]}bi{int(c[4])}")
def test_oracle_matches_reference_fixture(case):
    _, B, D, L, bi, f = case
    u = f["u"].reshape(B, D, L)
    bias = f["bias"].reshape(D, 1)
    y = H.fftconv_fwd(u, f["k"], bias, bi)
    np.testing.assert_allclose(y, f["y64"].reshape(B, D, L), rtol=0, atol=1e-12 * np.abs(y).max())
    du, dk, db = H.fftconv_bwd(f["dy"].reshape(B, D, L), u, f["k"], bias, bi)
    np.testing.assert_allclose(du, f["du"].reshape(B, D, L), rtol=0, atol=1e-12 * np.abs(du).max())
    np.testing.assert_allclose(dk, f["dk"], rtol=0, atol=1e-12 * np.abs(dk).max())
    np.testing.assert_allclose(db.reshape(-1), f["dbias"].reshape(-1), rtol=0, atol=1e-10)
    # the reference's own fp32 output agrees with its fp64 output to fp32 FFT precision
    assert np.abs(f["y32"] - f["y64"]).max() < 1e-5 * np.abs(f["y64"]).max()


@pytest.mark.parametrize("bi", [False, True])
def test_oracle_fft_equals_direct_definition(bi):
    rng = np.random.default_rng(1)
    u = rng.standard_normal((2, 3, 64))
    k = rng.standard_normal((3, 64))
    bias = rng.standard_normal((3, 1))
    np.testing.assert_allclose(H.fftconv_fwd(u, k, bias, bi), H.fftconv_direct(u, k, bias, bi), atol=1e-12)


def test_pad_before_matches_reference_formula():
    # hyena.py:70-72: padded = L + 2*(L//2); pad_before = padded//2 - L//2
    assert H.pad_before(64, True) == 32 and H.pad_before(65, True) == 32 and H.pad_before(64, False) == 0


def _op_fixture():
    d = np.load(os.path.join(os.path.dirname(GOLD), "hyena_op_golden.npz"), allow_pickle=False)
    sd = {k[3:]: torch.tensor(d[k]) for k in d.files if k.startswith("sd/")}
    return d, sd


def test_operator_oracle_matches_reference_fixture():
    """oracle/hyena_operator_ref.py vs the reference HyenaOperator run (hyena_op_golden.npz)."""
    from oracle import hyena_operator_ref as H
    d, sd = _op_fixture()
    k = H.hyena_filter(sd, 64)
    assert torch.allclose(k, torch.tensor(d["filter_k"]), rtol=0, atol=1e-12)
    y = H.hyena_operator(sd, torch.tensor(d["x"]), 16, order=2, l_max=64)
    assert torch.allclose(y, torch.tensor(d["y"]), rtol=0, atol=1e-12)
    z, t = H.positional_embedding(3, 64)
    assert torch.equal(z.double(), sd["filter_fn.pos_emb.z"]) and torch.equal(t.double(), sd["filter_fn.pos_emb.t"])


def test_operator_module_state_dict_matches_reference():
    """dna_amd.hyena.HyenaOperator has the reference's module tree: the fixture's state_dict
    (saved from the reference operator) loads strictly; a CPU forward raises (no fallback)."""
    from dna_amd.hyena import HyenaOperator
    d, sd = _op_fixture()
    op = HyenaOperator(d_model=16, l_max=64, order=2, filter_order=16).double()
    assert sorted(op.state_dict()) == sorted(sd)
    op.load_state_dict(sd, strict=True)
    with pytest.raises(RuntimeError):
        op(torch.tensor(d["x"]))
