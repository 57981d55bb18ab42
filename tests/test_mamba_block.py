"""CPU: the Caduceus BiMamba mixer's module structure (mamba_ssm 1.x Mamba parameters, the
reference BiMambaWrapper's weight tying) and a property of the float64 oracle. Parity of the GPU
path against the oracle is tests/test_gpu_mamba_block.py; mamba_ssm itself is absent (parity
unpinned, oracle/mamba_block_ref.py)."""
import math

import pytest
import torch

from oracle import mamba_block_ref as MB


def test_mamba_parameters_and_init():
    from dna_amd.mamba import Mamba
    torch.manual_seed(0)
    m = Mamba(d_model=64, d_state=16, d_conv=4, expand=2)
    E, R = 128, math.ceil(64 / 16)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes == {"A_log": (E, 16), "D": (E,), "in_proj.weight": (2 * E, 64),
                      "conv1d.weight": (E, 1, 4), "conv1d.bias": (E,),
                      "x_proj.weight": (R + 32, E), "dt_proj.weight": (E, R), "dt_proj.bias": (E,),
                      "out_proj.weight": (64, E)}
    assert torch.allclose(m.A_log, torch.log(torch.arange(1, 17).float()).repeat(E, 1))
    dt = torch.nn.functional.softplus(m.dt_proj.bias)  # inverse-softplus init of dt in [dt_min, dt_max]
    assert dt.min() >= 1e-3 - 1e-7 and dt.max() <= 0.1 + 1e-6
    with pytest.raises(RuntimeError):  # no CPU fallback
        m(torch.randn(1, 8, 64))


def test_bimamba_weight_tie():
    from dna_amd.mamba import BiMambaWrapper
    w = BiMambaWrapper(d_model=64, bidirectional=True, bidirectional_weight_tie=True)
    assert w.mamba_rev.in_proj.weight is w.mamba_fwd.in_proj.weight
    assert w.mamba_rev.out_proj.weight is w.mamba_fwd.out_proj.weight
    assert w.mamba_rev.x_proj.weight is not w.mamba_fwd.x_proj.weight
    keys = set(w.state_dict())
    assert {"mamba_fwd.A_log", "mamba_rev.A_log", "mamba_rev.in_proj.weight"} <= keys
    with pytest.raises(NotImplementedError):
        BiMambaWrapper(d_model=64, bidirectional_strategy="concat")
    assert BiMambaWrapper(d_model=64, bidirectional=False).mamba_rev is None


def test_oracle_bimamba_flip_symmetry():
    """Tied directions with identical per-direction weights: on a palindromic input the 'add'
    output is symmetric under a flip of the sequence."""
    from dna_amd.mamba import BiMambaWrapper
    torch.manual_seed(1)
    w = BiMambaWrapper(d_model=32, d_state=8).double()
    sd = {k: v.detach() for k, v in w.state_dict().items()}
    for k in list(sd):
        if k.startswith("mamba_rev."):
            sd[k] = sd["mamba_fwd." + k[len("mamba_rev."):]]
    h = torch.randn(1, 9, 32, dtype=torch.float64)
    h = torch.cat([h, h.flip(1)[:, 1:]], dim=1)  # palindrome, L = 17
    out = MB.bimamba_forward(sd, h, 8, 4, w.mamba_fwd.dt_rank)
    assert torch.allclose(out, out.flip(1), atol=1e-12)
