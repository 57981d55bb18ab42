"""CPU restatement of the HyenaDNA LM backbone (torch, float64) -- test infrastructure only.

Backbone semantics follow the reference's LMBackbone / BertLMHeadModel
(src/models/sequence/long_conv_lm.py:516-576, :665-682) with flash_attn's pre-norm Block and Mlp
(not installed: restated from flash_attn's published code -- parity unpinned beyond the Hyena
operator, which oracle/hyena_operator_ref.py pins to the reference). Eval mode (no dropout).
"""
import torch.nn.functional as F

from .hyena_operator_ref import hyena_operator


def lm_logits(sd, ids, d_model, n_layer, order=2, l_max=None, bidirectional=False, eps=1e-5):
    h = F.embedding(ids, sd["backbone.embeddings.word_embeddings.weight"])
    residual = None
    for i in range(n_layer):
        p = f"backbone.layers.{i}."
        residual = h if residual is None else h + residual
        x = F.layer_norm(residual, (d_model,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
        lsd = {k[len(p + "mixer."):]: v for k, v in sd.items() if k.startswith(p + "mixer.")}
        x = hyena_operator(lsd, x, d_model, order=order, l_max=l_max, bidirectional=bidirectional)
        residual = x + residual
        x = F.layer_norm(residual, (d_model,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
        x = F.linear(x, sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"])
        h = F.linear(F.gelu(x, approximate="tanh"), sd[p + "mlp.fc2.weight"], sd[p + "mlp.fc2.bias"])
    residual = h + residual
    h = F.layer_norm(residual, (d_model,), sd["backbone.ln_f.weight"], sd["backbone.ln_f.bias"], eps)
    return F.linear(h, sd["backbone.embeddings.word_embeddings.weight"])
