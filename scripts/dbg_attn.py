"""GPU debug helper: forward errors of the default attention kernel per (batch, head, query
block) against the fp32 reference, for a few shapes with/without pads."""
import sys
import torch
sys.path.insert(0, '.')
from tests.test_gpu_kernels import _qkv, _ref_attention
from dna_amd import functional as DF
from dna_amd.config import alibi_slopes
for (b, S, H, pads) in [(2, 128, 2, []), (2, 128, 2, [(1, 77)]), (3, 64, 1, []), (2, 256, 4, [(0, 200)]),
                        (1, 512, 12, []), (2, 512, 12, [(0, 400)])]:
    qkv, kv = _qkv(b, S, H, torch.bfloat16, pads, seed=3)
    slopes = torch.tensor(alibi_slopes(H), device='cuda')
    o1 = DF.alibi_attention(qkv, kv, slopes, b, S, H)
    ref = _ref_attention(qkv.float(), kv, H, b, S)
    e = (o1.float() - ref).abs() * kv[:, None].float()
    e = e.view(b, S // 32, 32, H, 64).amax(dim=(2, 4))  # [b, qblock, H]
    bad = (e > 3e-2).nonzero().tolist()
    print(b, S, H, pads, 'max err', e.max().item(), 'bad (b,qblk,h):', bad[:12], flush=True)
