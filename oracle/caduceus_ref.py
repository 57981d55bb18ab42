"""CPU restatement of the Caduceus MLM forward (torch, float64) -- test infrastructure.

Follows CaduceusMixerModel.forward / CaduceusForMaskedLM.forward (reference
src/models/caduceus/modeling_caduceus.py:197-257, :430-470) over the mamba_ssm Block
(add -> norm -> mixer) and the BiMamba oracle (oracle/mamba_block_ref.py). With rcps=True it
follows the RC-parameter-sharing modules of src/models/caduceus/modeling_rcps.py: RCPSEmbedding
(:51-64), RCPSWrapper (:82-96), RCPSAddNormWrapper (:104-127), RCPSMambaBlock.forward with and
without fused_add_norm (:157-197), the rcps final norm (modeling_caduceus.py:214-243) and
RCPSLMHead (:230-243). PARITY UNPINNED: mamba_ssm is absent, so no reference output exists.
"""
import torch
import torch.nn.functional as F

from .mamba_block_ref import bimamba_forward


def _norm(x, sd, prefix, rms, eps):
    if rms:
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * sd[prefix + "weight"]
    return F.layer_norm(x, (x.shape[-1],), sd[prefix + "weight"], sd[prefix + "bias"], eps)


def _flip_lc(x):
    return torch.flip(x, dims=[-2, -1])


def mlm_logits(sd, ids, n_layer, d_state, d_conv, dt_rank, rms_norm=True, eps=1e-5,
               strategy="add", scan=None, rcps=False, fused_add_norm=True):
    p0 = "caduceus.backbone."
    kw = {} if scan is None else {"scan": scan}
    if not rcps:
        h = F.embedding(ids, sd[p0 + "embeddings.word_embeddings.weight"])
        residual = None
        for i in range(n_layer):
            p = f"{p0}layers.{i}."
            residual = h if residual is None else h + residual
            x = _norm(residual, sd, p + "norm.", rms_norm, eps)
            msd = {k[len(p + "mixer."):]: v for k, v in sd.items() if k.startswith(p + "mixer.")}
            h = bimamba_forward(msd, x, d_state, d_conv, dt_rank, strategy=strategy, **kw)
        residual = h + residual
        h = _norm(residual, sd, p0 + "norm_f.", rms_norm, eps)
        return F.linear(h, sd["lm_head.weight"])

    W = sd[p0 + "embeddings.word_embeddings.embedding.weight"]
    cm = sd[p0 + "embeddings.word_embeddings.complement_map"]
    D = W.shape[1]
    rc_ids = cm[ids.flip(-1)]
    h = torch.cat([F.embedding(ids, W), _flip_lc(F.embedding(rc_ids, W))], -1)
    residual = None
    for i in range(n_layer):
        p = f"{p0}layers.{i}."
        np_ = p + ("norm." if fused_add_norm else "norm.submodule.")
        # which half of (h, residual) feeds the forward-strand norm: the fused block takes the
        # second half (modeling_rcps.py:170-186), the non-fused wrapper the first (:116-125)
        a, b = (slice(D, None), slice(None, D)) if fused_add_norm else (slice(None, D), slice(D, None))
        r_f = h[..., a] if residual is None else h[..., a] + residual[..., a]
        r_r = _flip_lc(h[..., b]) if residual is None else _flip_lc(h[..., b]) + _flip_lc(residual[..., b])
        x = torch.cat([_norm(r_f, sd, np_, rms_norm, eps), _flip_lc(_norm(r_r, sd, np_, rms_norm, eps))], -1)
        residual = torch.cat([r_f, _flip_lc(r_r)], -1)
        mp = p + "mixer.submodule."
        msd = {k[len(mp):]: v for k, v in sd.items() if k.startswith(mp)}
        y_f = bimamba_forward(msd, x[..., :D], d_state, d_conv, dt_rank, strategy=strategy, **kw)
        y_r = bimamba_forward(msd, _flip_lc(x[..., D:]), d_state, d_conv, dt_rank, strategy=strategy, **kw)
        h = torch.cat([y_f, _flip_lc(y_r)], -1)
    nf = p0 + ("norm_f." if fused_add_norm else "norm_f.submodule.")
    out_f = _norm(h[..., :D] + residual[..., :D], sd, nf, rms_norm, eps)
    out_r = _norm(_flip_lc(h[..., D:]) + _flip_lc(residual[..., D:]), sd, nf, rms_norm, eps)
    h = torch.cat([out_f, _flip_lc(out_r)], -1)
    Wl = sd["lm_head.lm_head.weight"]
    return F.linear(h[..., :D], Wl) + F.linear(torch.flip(h[..., D:], dims=[-1]), Wl[sd["lm_head.complement_map"]])
