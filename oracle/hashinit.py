"""Stateless hash initialiser for DNABERT-2 parameter tensors (TEST INFRASTRUCTURE).

This file is part of the oracle: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it. It lets the golden-fixture generator and the parity tests
build the SAME weights for a model without committing the weights themselves: every element
is a pure function of (parameter name, flat index) through splitmix64.

Distribution choices mimic `BertPreTrainedModel._init_weights` (normal(0, 0.02) for Linear /
Embedding, LayerNorm weight 1 / bias 0; reference `bert_layers.py:716` calls `post_init`),
except that biases and LayerNorm affine parameters get small NON-trivial values so that every
bias / affine path is actually exercised by the parity tests.
"""
import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def hash_uniform(name: str, n: int, salt: int = 0) -> np.ndarray:
    """n float64 values uniform in [0, 1), a pure function of (name, index, salt)."""
    key = np.uint64(zlib.crc32(name.encode()) | (salt << 32))
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _splitmix64(idx ^ (key * np.uint64(0x2545F4914F6CDD1D) & _M64))
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def hash_tensor(name: str, shape, salt: int = 0) -> np.ndarray:
    """Deterministic fp32 value for parameter `name` (state_dict key) of `shape`."""
    n = int(np.prod(shape))
    u = hash_uniform(name, n, salt) * 2.0 - 1.0  # uniform [-1, 1)
    leaf = name.rsplit(".", 1)[-1]
    is_ln = "LayerNorm" in name or "layernorm" in name
    if is_ln and leaf == "weight":
        v = 1.0 + 0.1 * u
    elif is_ln and leaf == "bias":
        v = 0.05 * u
    elif leaf == "bias":
        v = 0.02 * u
    else:
        # uniform with std 0.02 (sqrt(3) * 0.02 half-width)
        v = 0.0346410161513775 * u
    return v.astype(np.float32).reshape(shape)


def hash_state_dict(named_shapes):
    """{name: np.float32 array} for an iterable of (name, shape)."""
    return {n: hash_tensor(n, s) for n, s in named_shapes}
