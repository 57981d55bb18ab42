"""CPU restatement of the HyenaDNA operator around the long convolution (torch, float64).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker; the product path
(dna_amd.hyena.HyenaOperator) runs the FFT long convolution on the HIP kernels.

Restates, as plain functions over a state_dict, what the reference computes in
  * `PositionalEmbedding` (src/models/sequence/hyena.py:113-137): z = [t, Re, Im of
    exp(-i f w)], t = linspace(0, 1, L), w = 2 pi (0..L-1) / L, f = linspace(1e-4, bands-1, bands);
  * `Sin` (:100-110): sin(freq * x) with one shared `freq` for every activation of the MLP;
  * `ExponentialModulation` (:140-163): h * (exp(-t |deltas|) + shift);
  * `HyenaFilter.filter` (:240-251): implicit MLP on z, then the modulation;
  * `HyenaFilter.forward` (:253-280) -> `fftconv_ref` (:60-92): the long conv with bias `D`;
  * `HyenaOperator.forward` (:421-509) with num_heads = num_blocks = inner_factor = 1,
    outer_mixing = post_order_ffn = False, activation "id", dropout 0: in_proj -> depthwise
    causal short conv (kernel `short_filter_order`, padding k-1, first L outputs) -> split into
    x_0 .. x_{order-1}, v -> for each x_i in reversed(x[1:]): v = long_conv(v * x_i) ->
    out_proj(v * x_0).
Pinned by tests/golden/hyena_op_golden.npz (the reference operator run in this container by
tests/golden/make_hyena_golden.py: output y and filter k for a state_dict). Autograd through
these float64 ops is the reference for gradients.
"""
import math

import torch
import torch.nn.functional as F

from .hyena_ref import pad_before


def positional_embedding(emb_dim, seq_len):
    """(z [1, L, emb_dim], t [1, L, 1]) as hyena.py:113-137 builds them (float32, as torch does)."""
    t = torch.linspace(0, 1, seq_len)[None, :, None]
    bands = (emb_dim - 1) // 2
    t_rescaled = torch.linspace(0, seq_len - 1, seq_len)[None, :, None]
    w = 2 * math.pi * t_rescaled / seq_len
    f = torch.linspace(1e-4, bands - 1, bands)[None, None]
    z = torch.exp(-1j * f * w)
    return torch.cat([t, z.real, z.imag], dim=-1), t


def fftconv_torch(u, k, bias, bidirectional=False):
    """fftconv_ref (hyena.py:60-92) in torch float64 (autograd-capable): u [..., D, L] with the
    channel at dim -3 for 5-D inputs, k [D, L], bias as the reference receives it (it adds
    u * bias.unsqueeze(-1), :86)."""
    L = u.shape[-1]
    N = 2 * L
    pb = pad_before(L, bidirectional)
    up = F.pad(u, (pb, N - L - pb))
    kf = torch.fft.rfft(k, n=N) / N
    uf = torch.fft.rfft(up, n=N)
    if u.dim() > 3:
        kf = kf[:, None, :]  # [D, 1, N/2+1] against [..., D, 1, N/2+1]
    y = torch.fft.irfft(uf * kf, n=N, norm="forward")[..., :L]
    return y + u * bias.unsqueeze(-1)


def implicit_filter(sd, prefix, z):
    """nn.Sequential(Linear, Sin, [Linear, Sin]*, Linear(no bias)) of HyenaFilter (:216-228)."""
    i = 0
    h = z
    while f"{prefix}{i}.weight" in sd:
        w = sd[f"{prefix}{i}.weight"]
        b = sd.get(f"{prefix}{i}.bias")
        h = F.linear(h, w, b)
        if f"{prefix}{i + 1}.freq" in sd:
            h = torch.sin(sd[f"{prefix}{i + 1}.freq"] * h)
            i += 2
        else:
            i += 1
    return h


def hyena_filter(sd, L, prefix="filter_fn.", modulate=True, normalized=False, shift=0.0):
    """HyenaFilter.filter(L) (:240-251) -> k [1, L, d_filter]."""
    z = sd[prefix + "pos_emb.z"][:, :L]
    t = sd[prefix + "pos_emb.t"][:, :L]
    h = implicit_filter(sd, prefix + "implicit_filter.", z)
    if modulate:
        h = h * (torch.exp(-t * sd[prefix + "modulation.deltas"].abs()) + shift)
    if normalized:
        h = h / torch.norm(h, dim=-1, p=1, keepdim=True)
    return h


def hyena_operator(sd, x, d_model, order=2, l_max=None, short_filter_order=3,
                   bidirectional=False, modulate=True, normalized=False, shift=0.0):
    """HyenaOperator.forward (:421-509) on x [b, l, d_model] -> [b, l, d_model]."""
    b, l, _ = x.shape
    l_filter = min(l, l_max) if l_max else l
    u = F.linear(x, sd["in_proj.weight"], sd["in_proj.bias"]).transpose(1, 2)  # [b, (o+1)d, l]
    C = u.shape[1]
    uc = F.conv1d(u, sd["short_filter.weight"], sd["short_filter.bias"],
                  padding=short_filter_order - 1, groups=C)[..., :l_filter]
    uc = uc.reshape(b, 1, C, 1, l_filter)               # b ho v z l with ho = z = 1
    *xs, v = uc.split(d_model, dim=2)
    k = hyena_filter(sd, l_filter, modulate=modulate, normalized=normalized, shift=shift)
    # "c l (v o) -> c o v l", v = d_model, o = order - 1
    k = k[0].reshape(l_filter, d_model, order - 1).permute(2, 1, 0)
    bias = sd["filter_fn.bias"].reshape(d_model, order - 1).t()  # "(v o) -> o v"
    for o, x_i in enumerate(reversed(xs[1:])):
        v = v * x_i
        v = fftconv_torch(v, k[o], bias[o][None, :, None], bidirectional)
    y = (v * xs[0]).reshape(b, d_model, l_filter).transpose(1, 2)  # b (z l) (h v)
    return F.linear(y, sd["out_proj.weight"], sd["out_proj.bias"])
