#!/usr/bin/env python
"""Golden fixtures for Caduceus' reverse-complement parameter-sharing layers, produced by running
the REFERENCE code (VERDICT r4 "missing 1").

Run from the repo root:  python tests/golden/make_rcps_golden.py
Loads /root/reference/src/models/caduceus/modeling_rcps.py by path (read-only, never copied; its
only mamba_ssm import is guarded by try/except, :12-15, so it imports without mamba_ssm) and runs
each RCPS class in float64 with plain torch submodules -- nn.Linear as the mixer, nn.LayerNorm as
the norm -- on seeded inputs, recording outputs and the gradients of every input and parameter
under a seeded upstream cotangent. Writes rcps_golden.npz:

  emb_*    RCPSEmbedding (:18-64)              ids -> [fwd | flip_{L,C}(emb(rc(ids)))]
  wrap_*   RCPSWrapper(nn.Linear) (:67-96)
  an0_*    RCPSAddNormWrapper(nn.LayerNorm) (:99-127), residual=None, prenorm=True
  an_*     the same with a residual
  blk0_*   RCPSMambaBlock(fused_add_norm=False, residual_in_fp32=True) (:130-203), first layer
  blk_*    the same with a residual
  head_*   RCPSLMHead (:206-243)

Not covered (they need mamba_ssm, absent here): the fused_add_norm block (layer_norm_fn /
rms_norm_fn), RMSNorm, and the Mamba mixer itself -- those stay "parity unpinned".
"""
import importlib.util
import os

import numpy as np
import torch
from torch import nn

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

B, L, D, V = 2, 16, 64, 12
# special ids 0-6 complement to themselves, A=7 <-> T=10, C=8 <-> G=9, N=11 -> N
COMPLEMENT = {i: i for i in range(V)}
COMPLEMENT.update({7: 10, 10: 7, 8: 9, 9: 8})


def load_rcps():
    path = os.path.join(REF, "src", "models", "caduceus", "modeling_rcps.py")
    spec = importlib.util.spec_from_file_location("ref_modeling_rcps", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class LinearMixer(nn.Linear):
    """nn.Linear(dim, dim) built as mixer_cls(dim), taking the mixer call's inference_params
    keyword (RCPSMambaBlock.forward passes it through RCPSWrapper)."""

    def __init__(self, dim):
        super().__init__(dim, dim)

    def forward(self, x, inference_params=None):
        return super().forward(x)


def _set(mod, g, **shapes):
    with torch.no_grad():
        for name, p in mod.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.5
                    + (1.0 if name.endswith("weight") and p.dim() == 1 else 0.0))


def _grads(out, gouts, tensors):
    outs = out if isinstance(out, tuple) else (out,)
    gs = torch.autograd.grad(outs, tensors, gouts, allow_unused=True)
    return [torch.zeros_like(t) if g is None else g for t, g in zip(tensors, gs)]


def main():
    torch.set_default_dtype(torch.float64)
    R = load_rcps()
    g = torch.Generator().manual_seed(2222)
    rnd = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)
    out = {"complement": np.array([COMPLEMENT[i] for i in range(V)], dtype=np.int64)}

    # RCPSEmbedding
    emb = R.RCPSEmbedding(V, D, COMPLEMENT)
    _set(emb, g)
    ids = torch.randint(0, V, (B, L), generator=g)
    y = emb(ids)
    gy = rnd(*y.shape)
    (dW,) = _grads(y, gy, [emb.embedding.weight])
    out.update(emb_ids=ids.numpy(), emb_W=emb.embedding.weight.detach().numpy(),
               emb_gout=gy.numpy(), emb_out=y.detach().numpy(), emb_dW=dW.numpy())

    # RCPSWrapper over nn.Linear
    lin = nn.Linear(D, D)
    _set(lin, g)
    wrap = R.RCPSWrapper(lin)
    x = rnd(B, L, 2 * D).requires_grad_(True)
    y = wrap(x)
    gy = rnd(*y.shape)
    dx, dW, db = _grads(y, gy, [x, lin.weight, lin.bias])
    out.update(wrap_x=x.detach().numpy(), wrap_W=lin.weight.detach().numpy(),
               wrap_b=lin.bias.detach().numpy(), wrap_gout=gy.numpy(), wrap_out=y.detach().numpy(),
               wrap_dx=dx.numpy(), wrap_dW=dW.numpy(), wrap_db=db.numpy())

    # RCPSAddNormWrapper over nn.LayerNorm, without and with a residual (prenorm=True)
    for tag, with_res in (("an0", False), ("an", True)):
        ln = nn.LayerNorm(D)
        _set(ln, g)
        an = R.RCPSAddNormWrapper(ln)
        x = rnd(B, L, 2 * D).requires_grad_(True)
        res = rnd(B, L, 2 * D).requires_grad_(True) if with_res else None
        yy, rr = an(x, residual=res, prenorm=True)
        gy, gr = rnd(*yy.shape), rnd(*rr.shape)
        ts = [x, ln.weight, ln.bias] + ([res] if with_res else [])
        grads = _grads((yy, rr), (gy, gr), ts)
        out.update({f"{tag}_x": x.detach().numpy(), f"{tag}_g": ln.weight.detach().numpy(),
                    f"{tag}_beta": ln.bias.detach().numpy(), f"{tag}_gy": gy.numpy(),
                    f"{tag}_gres": gr.numpy(), f"{tag}_y": yy.detach().numpy(),
                    f"{tag}_res_out": rr.detach().numpy(), f"{tag}_dx": grads[0].numpy(),
                    f"{tag}_dg": grads[1].numpy(), f"{tag}_dbeta": grads[2].numpy()})
        if with_res:
            out.update({f"{tag}_res": res.detach().numpy(), f"{tag}_dres": grads[3].numpy()})

    # RCPSMambaBlock (non-fused add + norm, residual in fp32) with a Linear mixer
    for tag, with_res in (("blk0", False), ("blk", True)):
        blk = R.RCPSMambaBlock(D, LinearMixer, norm_cls=nn.LayerNorm, fused_add_norm=False,
                               residual_in_fp32=True)
        _set(blk, g)
        h = rnd(B, L, 2 * D).requires_grad_(True)
        res = rnd(B, L, 2 * D).requires_grad_(True) if with_res else None
        hh, rr = blk(h, residual=res)
        gh, gr = rnd(*hh.shape), rnd(*rr.shape)
        ln, mix = blk.norm.submodule, blk.mixer.submodule
        ts = [h, ln.weight, ln.bias, mix.weight, mix.bias] + ([res] if with_res else [])
        grads = _grads((hh, rr), (gh, gr), ts)
        out.update({f"{tag}_h": h.detach().numpy(), f"{tag}_norm_g": ln.weight.detach().numpy(),
                    f"{tag}_norm_b": ln.bias.detach().numpy(), f"{tag}_mix_W": mix.weight.detach().numpy(),
                    f"{tag}_mix_b": mix.bias.detach().numpy(), f"{tag}_gh": gh.numpy(),
                    f"{tag}_gres": gr.numpy(), f"{tag}_h_out": hh.detach().numpy(),
                    f"{tag}_res_out": rr.detach().numpy(), f"{tag}_dh": grads[0].numpy(),
                    f"{tag}_dnorm_g": grads[1].numpy(), f"{tag}_dnorm_b": grads[2].numpy(),
                    f"{tag}_dmix_W": grads[3].numpy(), f"{tag}_dmix_b": grads[4].numpy()})
        if with_res:
            out.update({f"{tag}_res": res.detach().numpy(), f"{tag}_dres": grads[5].numpy()})

    # RCPSLMHead
    head = R.RCPSLMHead(D, V, COMPLEMENT)
    _set(head, g)
    x = rnd(B, L, 2 * D).requires_grad_(True)
    y = head(x)
    gy = rnd(*y.shape)
    dx, dW = _grads(y, gy, [x, head.lm_head.weight])
    out.update(head_x=x.detach().numpy(), head_W=head.lm_head.weight.detach().numpy(),
               head_gout=gy.numpy(), head_out=y.detach().numpy(), head_dx=dx.numpy(),
               head_dW=dW.numpy())

    path = os.path.join(HERE, "rcps_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays")


if __name__ == "__main__":
    main()
