#!/usr/bin/env python
"""Golden fixtures for the HyenaDNA FFT long-conv path, produced by running the REFERENCE code.

Run from the repo root:  python tests/golden/make_hyena_golden.py
Imports /root/reference/src/models/sequence/hyena.py by path (read-only, never copied) with
stand-ins for packages this image lacks (SURVEY §8c recipe 4: pytorch_lightning.rank_zero_only,
hydra.utils.get_method, omegaconf DictConfig/ListConfig, opt_einsum.contract). Writes:

  fftconv_golden.npz  `fftconv_ref` (hyena.py:60-92), causal and bidirectional, on fp32 inputs:
                      y in float64 (inputs upcast) and float32 (the reference's own dtype), and
                      float64 autograd grads du, dk, dbias for a random upstream dy.
  hyena_op_golden.npz tiny `HyenaFilter.filter` (hyena.py:240-251) and `HyenaOperator.forward`
                      (:421-509) outputs with their state_dicts (fp64).
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_shims():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules.setdefault(name, m)
        return m

    pl = mod("pytorch_lightning")
    util = mod("pytorch_lightning.utilities", rank_zero_only=lambda f: f)
    pl.utilities = util
    hydra = mod("hydra")
    def get_method(path):
        m, name = path.rsplit(".", 1)
        return getattr(importlib.import_module(m), name)

    hydra.utils = mod("hydra.utils", get_method=get_method, instantiate=lambda *a, **k: None)

    class _DC(dict):
        pass

    mod("omegaconf", DictConfig=_DC, ListConfig=list,
        OmegaConf=types.SimpleNamespace(to_container=lambda c, **k: dict(c)))
    mod("opt_einsum", contract=lambda *a, **k: torch.einsum(*a))
    sys.path.insert(0, REF)
    os.environ.setdefault("PROJECT_ROOT", REF)


def fftconv_cases(hy):
    rng = np.random.default_rng(2222)
    cases = [(2, 3, 64, False), (2, 3, 64, True), (3, 4, 1024, False), (2, 2, 1024, True),
             (1, 2, 4096, True), (1, 3, 4096, False), (2, 1, 16384, True)]
    out = {}
    for ci, (B, D, L, bi) in enumerate(cases):
        u = rng.standard_normal((B, 1, D, 1, L)).astype(np.float32)
        # filters decay like the implicit Hyena filters (ExponentialModulation)
        k = (rng.standard_normal((D, L)) * np.exp(-np.linspace(0, 4, L))[None]).astype(np.float32)
        bias = rng.standard_normal((1, D, 1)).astype(np.float32)
        dy = rng.standard_normal((B, 1, D, 1, L)).astype(np.float32)
        ut = torch.tensor(u, dtype=torch.float64, requires_grad=True)
        kt = torch.tensor(k, dtype=torch.float64, requires_grad=True)
        bt = torch.tensor(bias, dtype=torch.float64, requires_grad=True)
        y = hy.fftconv_ref(ut, kt, bt, dropout_mask=None, gelu=False, bidirectional=bi)
        y.backward(torch.tensor(dy, dtype=torch.float64))
        y32 = hy.fftconv_ref(torch.tensor(u), torch.tensor(k), torch.tensor(bias), dropout_mask=None,
                             gelu=False, bidirectional=bi)
        p = f"c{ci}_"
        out[p + "shape"] = np.array([B, D, L, int(bi)])
        out[p + "u"], out[p + "k"], out[p + "bias"], out[p + "dy"] = u, k, bias, dy
        out[p + "y64"] = y.detach().numpy()
        out[p + "y32"] = y32.numpy()
        out[p + "du"] = ut.grad.numpy()
        out[p + "dk"] = kt.grad.numpy()
        out[p + "dbias"] = bt.grad.numpy()
    out["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "fftconv_golden.npz"), **out)
    print("fftconv cases:", cases)


def operator_case(hy):
    torch.manual_seed(7)
    d_model, L = 16, 64
    op = hy.HyenaOperator(d_model=d_model, l_max=L, order=2, filter_order=16,
                          filter_args={"emb_dim": 5}).double()
    sd = {k: v.detach().numpy() for k, v in op.state_dict().items()}
    x = torch.randn(2, L, d_model, dtype=torch.float64)
    y = op(x)
    k = op.filter_fn.filter(L)
    out = {"x": x.numpy(), "y": y.detach().numpy(), "filter_k": k.detach().numpy()}
    out.update({"sd/" + k: v for k, v in sd.items()})
    np.savez_compressed(os.path.join(HERE, "hyena_op_golden.npz"), **out)
    print("operator state keys:", sorted(sd))


def main():
    _install_shims()
    hy = importlib.import_module("src.models.sequence.hyena")
    fftconv_cases(hy)
    operator_case(hy)


if __name__ == "__main__":
    main()
