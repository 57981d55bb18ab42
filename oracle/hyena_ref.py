"""CPU restatement of the HyenaDNA FFT long convolution, forward and backward (numpy, float64).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product path (dna_amd.hyena runs the HIP kernels
and fails loudly without them).

Follows `fftconv_ref` (reference src/models/sequence/hyena.py:60-92) as called by
`HyenaFilter.forward` (:253-280: dropout_mask=None, gelu=False, bias = per-channel `D`):
    N = 2L,  k_f = rfft(k, N) / N
    causal:        u~ = u zero-padded at the end to N
    bidirectional: u~ = [0]*pad_before ++ u ++ [0]*pad_after, pad_before = (L + 2*(L//2))//2 - L//2
    y = irfft(rfft(u~, N) * k_f, N, norm="forward")[..., :L] + u * D
i.e. y[t] = sum_j k[j] u~[(t - j) mod N] + D u[t]  (t < L): a circular convolution of length N.
Backward (what torch autograd of that expression gives; pinned by tests/golden/fftconv_golden.npz,
produced from the reference by tests/golden/make_hyena_golden.py):
    du~ = irfft(rfft(dy padded to N) * conj(k_f), N, norm="forward");  du = du~[pad_before:+L] + D dy
    dk[j] = sum_rows sum_t dy[t] u~[(t - j) mod N]   (j < L),   dD = sum_rows sum_t dy[t] u[t]
"""
import numpy as np


def pad_before(L, bidirectional):
    if not bidirectional:
        return 0
    padded = L + 2 * (L // 2)
    return padded // 2 - L // 2


def _padded(u, L, bidirectional):
    N = 2 * L
    pb = pad_before(L, bidirectional)
    out = np.zeros(u.shape[:-1] + (N,), dtype=np.float64)
    out[..., pb:pb + L] = u
    return out


def fftconv_fwd(u, k, bias, bidirectional=False):
    """u [..., D, L]; k [D, L]; bias broadcastable to u[..., :1] per channel -> y like u (float64)."""
    u = np.asarray(u, np.float64)
    k = np.asarray(k, np.float64)
    L = u.shape[-1]
    N = 2 * L
    kf = np.fft.rfft(k, n=N) / N
    uf = np.fft.rfft(_padded(u, L, bidirectional), n=N)
    y = np.fft.irfft(uf * kf, n=N, norm="forward")[..., :L]
    return y + u * np.asarray(bias, np.float64)


def fftconv_bwd(dy, u, k, bias, bidirectional=False):
    """Gradients (du, dk, dbias) of sum(dy * fftconv_fwd(u, k, bias)); dbias shaped like bias."""
    dy = np.asarray(dy, np.float64)
    u = np.asarray(u, np.float64)
    k = np.asarray(k, np.float64)
    bias = np.asarray(bias, np.float64)
    L = u.shape[-1]
    N = 2 * L
    pb = pad_before(L, bidirectional)
    kf = np.fft.rfft(k, n=N) / N
    dyf = np.fft.rfft(dy, n=N)
    dut = np.fft.irfft(dyf * np.conj(kf), n=N, norm="forward")
    du = dut[..., pb:pb + L] + dy * bias
    uf = np.fft.rfft(_padded(u, L, bidirectional), n=N)
    corr = np.fft.irfft(dyf * np.conj(uf), n=N, norm="forward")[..., :L] / N
    D = k.shape[0]
    dk = corr.reshape(-1, D, L) if corr.ndim == 3 else corr.reshape(-1, *corr.shape[-2:])
    dk = dk.reshape(-1, D, L).sum(0)
    prod = (dy * u).sum(-1, keepdims=True)
    dbias = prod.reshape(-1, D).sum(0).reshape(bias.shape)
    return du, dk, dbias


def fftconv_direct(u, k, bias, bidirectional=False):
    """O(L^2) direct circular convolution (small L only): the definition the FFT path computes."""
    u = np.asarray(u, np.float64)
    k = np.asarray(k, np.float64)
    L = u.shape[-1]
    N = 2 * L
    ut = _padded(u, L, bidirectional)
    y = np.zeros_like(u)
    j = np.arange(L)
    for t in range(L):
        y[..., t] = (k * ut[..., (t - j) % N]).sum(-1)
    return y + u * np.asarray(bias, np.float64)
