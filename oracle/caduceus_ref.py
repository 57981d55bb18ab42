"""CPU restatement of the Caduceus MLM forward (torch, float64) -- test infrastructure.

Follows CaduceusMixerModel.forward / CaduceusForMaskedLM.forward (reference
src/models/caduceus/modeling_caduceus.py:197-257, :430-470) over the mamba_ssm Block
(add -> norm -> mixer) and the BiMamba oracle (oracle/mamba_block_ref.py). With rcps=True it
follows the RC-parameter-sharing modules of src/models/caduceus/modeling_rcps.py: RCPSEmbedding
(:51-64), RCPSWrapper (:82-96), RCPSAddNormWrapper (:104-127), RCPSMambaBlock.forward with and
without fused_add_norm (:157-197), the rcps final norm (modeling_caduceus.py:214-243) and
RCPSLMHead (:230-243). The RCPS layers (rcps_* below) are PINNED to the reference module itself
(tests/golden/rcps_golden.npz, made by tests/golden/make_rcps_golden.py from modeling_rcps.py with
nn.Linear / nn.LayerNorm submodules); the Mamba mixer, RMSNorm and the fused add + norm branch need
mamba_ssm, which is absent: that part stays PARITY UNPINNED.
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


# ---- the RCPS layers one at a time (modeling_rcps.py), pinned by tests/golden/rcps_golden.npz
def rcps_embedding(W, cm, ids):
    """RCPSEmbedding.forward (:51-64): [emb(ids) | flip_{L,C}(emb(cm[flip_L(ids)]))]."""
    return torch.cat([F.embedding(ids, W), _flip_lc(F.embedding(cm[ids.flip(-1)], W))], -1)


def rcps_wrapper(f, x):
    """RCPSWrapper.forward (:82-96): f on the first half and on rc(second half), rc'd back."""
    D = x.shape[-1] // 2
    return torch.cat([f(x[..., :D]), _flip_lc(f(_flip_lc(x[..., D:])))], -1)


def rcps_add_norm(norm, x, residual=None):
    """RCPSAddNormWrapper.forward(prenorm=True) (:104-127): (norm per half, residual) with the
    halves kept in place; residual=None normalises x itself."""
    D = x.shape[-1] // 2
    r_f = x[..., :D] if residual is None else x[..., :D] + residual[..., :D]
    r_r = _flip_lc(x[..., D:]) if residual is None else _flip_lc(x[..., D:]) + _flip_lc(residual[..., D:])
    y = torch.cat([norm(r_f), _flip_lc(norm(r_r))], -1)
    return y, (x if residual is None else torch.cat([r_f, _flip_lc(r_r)], -1))


def rcps_block(norm, mixer, h, residual=None, fused_add_norm=False, residual_in_fp32=False):
    """RCPSMambaBlock.forward (:157-197) -> (mixer output, residual). Non-fused: the add + norm
    wrapper above; fused: the second half feeds the forward-strand norm (:170-186), so the halves
    trade places (restated; mamba_ssm's layer_norm_fn is not importable, that branch is unpinned)."""
    if fused_add_norm:
        D = h.shape[-1] // 2
        h = torch.cat([h[..., D:], h[..., :D]], -1)
        residual = None if residual is None else torch.cat([residual[..., D:], residual[..., :D]], -1)
        # after the swap the wrapper's per-half arithmetic is the fused block's
    x, residual = rcps_add_norm(norm, h, residual)
    if residual_in_fp32:  # :162-163 (the float64 model oracle keeps float64: False there)
        residual = residual.to(torch.float32)
    return rcps_wrapper(mixer, x), residual


def rcps_lm_head(W, cm, x):
    """RCPSLMHead.forward (:230-243): W x_fwd + W[cm] flip_C(x_rc)."""
    D = x.shape[-1] // 2
    return F.linear(x[..., :D], W) + F.linear(torch.flip(x[..., D:], dims=[-1]), W[cm])


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
    h = rcps_embedding(W, cm, ids)
    residual = None
    for i in range(n_layer):
        p = f"{p0}layers.{i}."
        np_ = p + ("norm." if fused_add_norm else "norm.submodule.")
        mp = p + "mixer.submodule."
        msd = {k[len(mp):]: v for k, v in sd.items() if k.startswith(mp)}
        h, residual = rcps_block(
            lambda t: _norm(t, sd, np_, rms_norm, eps),
            lambda t: bimamba_forward(msd, t, d_state, d_conv, dt_rank, strategy=strategy, **kw),
            h, residual, fused_add_norm=fused_add_norm)
    # the final norm keeps the halves in place, fused or not (modeling_caduceus.py:214-243)
    nf = p0 + ("norm_f." if fused_add_norm else "norm_f.submodule.")
    h, _ = rcps_add_norm(lambda t: _norm(t, sd, nf, rms_norm, eps), h, residual)
    return rcps_lm_head(sd["lm_head.lm_head.weight"], sd["lm_head.complement_map"], h)
