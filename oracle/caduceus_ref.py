"""CPU restatement of the Caduceus MLM forward (rcps=False; torch, float64) -- test infrastructure.

Follows CaduceusMixerModel.forward / CaduceusForMaskedLM.forward (reference
src/models/caduceus/modeling_caduceus.py:194-216, :440-470) over the mamba_ssm Block
(add -> norm -> mixer) and the BiMamba oracle (oracle/mamba_block_ref.py). PARITY UNPINNED:
mamba_ssm is absent, so no reference output exists.
"""
import torch
import torch.nn.functional as F

from .mamba_block_ref import bimamba_forward


def _norm(x, sd, prefix, rms, eps):
    if rms:
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * sd[prefix + "weight"]
    return F.layer_norm(x, (x.shape[-1],), sd[prefix + "weight"], sd[prefix + "bias"], eps)


def mlm_logits(sd, ids, n_layer, d_state, d_conv, dt_rank, rms_norm=True, eps=1e-5,
               strategy="add", scan=None):
    p0 = "caduceus.backbone."
    h = F.embedding(ids, sd[p0 + "embeddings.word_embeddings.weight"])
    residual = None
    for i in range(n_layer):
        p = f"{p0}layers.{i}."
        residual = h if residual is None else h + residual
        x = _norm(residual, sd, p + "norm.", rms_norm, eps)
        msd = {k[len(p + "mixer."):]: v for k, v in sd.items() if k.startswith(p + "mixer.")}
        kw = {} if scan is None else {"scan": scan}
        h = bimamba_forward(msd, x, d_state, d_conv, dt_rank, strategy=strategy, **kw)
    residual = h + residual
    h = _norm(residual, sd, p0 + "norm_f.", rms_norm, eps)
    return F.linear(h, sd["lm_head.weight"])
