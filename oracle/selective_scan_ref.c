/* Float64 CPU restatement of the Mamba selective scan, forward AND backward, for the long-sequence
 * checks of BASELINE config E (Caduceus, L = 131,072).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ (ctypes) as the checker; nothing in dna_amd/ links
 * or calls it. PARITY UNPINNED at the mamba_ssm level (mamba_ssm is not vendored in
 * /root/reference nor installed here -- see oracle/selective_scan_ref.py); this file restates the
 * same published `selective_scan_ref` math as that Python restatement, and tests/
 * test_selective_scan_oracle.py pins it to the Python float64 restatement (torch autograd for
 * the gradients) at small sizes. The Python/autograd form needs > 15 min at L = 131,072; this
 * one a fraction of a second per channel.
 *
 * Semantics (mamba_ssm/ops/selective_scan_interface.py selective_scan_ref, Mamba-1 call made by
 * Mamba.forward, reference src/models/caduceus/modeling_caduceus.py:68-121):
 *   d'    = softplus(delta + delta_bias)   (softplus if delta_softplus, bias if given)
 *   x_t   = exp(d'_t A[n]) x_{t-1} + d'_t B_t[n] u_t            per channel d, state n
 *   y_t   = sum_n C_t[n] x_t[n] + D u_t ;  out_t = y_t silu(z_t)  (z optional)
 * Backward (reverse sweep, g_t[n] = dL/dx_t[n]):
 *   g_t = dy_t C_t + exp(d'_{t+1} A) g_{t+1}
 *   dd'_t = sum_n g_t[n] (A[n] exp(d'_t A[n]) x_{t-1}[n] + B_t[n] u_t)
 *   dA[n] += g_t[n] d'_t exp(d'_t A[n]) x_{t-1}[n]; dB_t[n] += g_t[n] d'_t u_t (over channels);
 *   dC_t[n] += dy_t x_t[n]; du_t = dy_t D + sum_n g_t[n] d'_t B_t[n]; dD += dy_t u_t;
 *   ddelta = dd' sigmoid(delta + bias) (softplus); dbias += ddelta.
 * Layouts (all float64, contiguous): u, delta, z, out, du, ddelta, dz [b][d][l]; A, dA [d][n];
 * B, C, dB, dC [b][n][l]; D, delta_bias, dD, ddelta_bias [d]; last [b][d][n].
 * Gradient outputs are overwritten (not accumulated into). Returns 0, or -1 on allocation failure.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

static double softplus(double x) { return x > 20.0 ? x : log1p(exp(x)); }
static double sigmoid(double x) { return 1.0 / (1.0 + exp(-x)); }

/* effective step d'_t for channel (bi, di) into dd[l] */
static void deltas(const double* delta, const double* delta_bias, int softplus_on, int di, int l,
                   double* dd) {
  const double bias = delta_bias ? delta_bias[di] : 0.0;
  for (int t = 0; t < l; ++t) {
    const double v = delta[t] + bias;
    dd[t] = softplus_on ? softplus(v) : v;
  }
}

int ssref_fwd(const double* u, const double* delta, const double* A, const double* B,
              const double* C, const double* D, const double* z, const double* delta_bias,
              int delta_softplus, int b, int d, int l, int n, double* out, double* last) {
  double* dd = (double*)malloc(sizeof(double) * (size_t)l);
  double* x = (double*)malloc(sizeof(double) * (size_t)n);
  if (!dd || !x) { free(dd); free(x); return -1; }
  for (int bi = 0; bi < b; ++bi)
    for (int di = 0; di < d; ++di) {
      const size_t row = ((size_t)bi * d + di) * l;
      const double* Bb = B + (size_t)bi * n * l;
      const double* Cb = C + (size_t)bi * n * l;
      deltas(delta + row, delta_bias, delta_softplus, di, l, dd);
      memset(x, 0, sizeof(double) * (size_t)n);
      for (int t = 0; t < l; ++t) {
        const double ut = u[row + t];
        double y = 0.0;
        for (int s = 0; s < n; ++s) {
          x[s] = exp(dd[t] * A[(size_t)di * n + s]) * x[s] + dd[t] * Bb[(size_t)s * l + t] * ut;
          y += Cb[(size_t)s * l + t] * x[s];
        }
        if (D) y += D[di] * ut;
        if (z) {
          const double zt = z[row + t];
          y *= zt * sigmoid(zt);
        }
        out[row + t] = y;
      }
      if (last)
        for (int s = 0; s < n; ++s) last[((size_t)bi * d + di) * n + s] = x[s];
    }
  free(dd);
  free(x);
  return 0;
}

int ssref_bwd(const double* u, const double* delta, const double* A, const double* B,
              const double* C, const double* D, const double* z, const double* delta_bias,
              int delta_softplus, int b, int d, int l, int n, const double* dout, double* du,
              double* ddelta, double* dA, double* dB, double* dC, double* dD, double* dz,
              double* ddelta_bias) {
  double* dd = (double*)malloc(sizeof(double) * (size_t)l);
  double* xs = (double*)malloc(sizeof(double) * (size_t)(l + 1) * n);  /* x_{-1} = 0 .. x_{l-1} */
  double* g = (double*)malloc(sizeof(double) * (size_t)n);
  double* dy = (double*)malloc(sizeof(double) * (size_t)l);
  if (!dd || !xs || !g || !dy) { free(dd); free(xs); free(g); free(dy); return -1; }
  memset(dA, 0, sizeof(double) * (size_t)d * n);
  memset(dB, 0, sizeof(double) * (size_t)b * n * l);
  memset(dC, 0, sizeof(double) * (size_t)b * n * l);
  if (dD) memset(dD, 0, sizeof(double) * (size_t)d);
  if (ddelta_bias) memset(ddelta_bias, 0, sizeof(double) * (size_t)d);
  for (int bi = 0; bi < b; ++bi)
    for (int di = 0; di < d; ++di) {
      const size_t row = ((size_t)bi * d + di) * l;
      const double* Bb = B + (size_t)bi * n * l;
      const double* Cb = C + (size_t)bi * n * l;
      double* dBb = dB + (size_t)bi * n * l;
      double* dCb = dC + (size_t)bi * n * l;
      const double* Ad = A + (size_t)di * n;
      deltas(delta + row, delta_bias, delta_softplus, di, l, dd);
      /* forward sweep: keep every state */
      memset(xs, 0, sizeof(double) * (size_t)n);
      for (int t = 0; t < l; ++t)
        for (int s = 0; s < n; ++s)
          xs[(size_t)(t + 1) * n + s] = exp(dd[t] * Ad[s]) * xs[(size_t)t * n + s] +
                                        dd[t] * Bb[(size_t)s * l + t] * u[row + t];
      /* dy and dz need y */
      for (int t = 0; t < l; ++t) {
        double y = 0.0;
        for (int s = 0; s < n; ++s) y += Cb[(size_t)s * l + t] * xs[(size_t)(t + 1) * n + s];
        if (D) y += D[di] * u[row + t];
        if (z) {
          const double zt = z[row + t], sg = sigmoid(zt);
          dy[t] = dout[row + t] * zt * sg;
          dz[row + t] = dout[row + t] * y * sg * (1.0 + zt * (1.0 - sg));
        } else {
          dy[t] = dout[row + t];
        }
      }
      /* reverse sweep */
      memset(g, 0, sizeof(double) * (size_t)n);
      double dDd = 0.0, dbias = 0.0;
      for (int t = l - 1; t >= 0; --t) {
        const double ut = u[row + t];
        double ddp = 0.0, dut = D ? dy[t] * D[di] : 0.0;
        for (int s = 0; s < n; ++s) {
          const size_t k = (size_t)s * l + t;
          /* g_t = dy_t C_t + a_{t+1} g_{t+1}: the a_{t+1} factor was applied at step t+1 */
          g[s] += dy[t] * Cb[k];
          const double xt = xs[(size_t)(t + 1) * n + s], xp = xs[(size_t)t * n + s];
          const double a = exp(dd[t] * Ad[s]);
          dCb[k] += dy[t] * xt;
          ddp += g[s] * (Ad[s] * a * xp + Bb[k] * ut);
          dA[(size_t)di * n + s] += g[s] * dd[t] * a * xp;
          dBb[k] += g[s] * dd[t] * ut;
          dut += g[s] * dd[t] * Bb[k];
          g[s] *= a;  /* becomes a_t g_t for step t-1 */
        }
        du[row + t] = dut;
        if (D) dDd += dy[t] * ut;
        double dlt = ddp;
        if (delta_softplus) dlt *= sigmoid(delta[row + t] + (delta_bias ? delta_bias[di] : 0.0));
        ddelta[row + t] = dlt;
        dbias += dlt;
      }
      if (dD) dD[di] += dDd;
      if (ddelta_bias) ddelta_bias[di] += dbias;
    }
  free(dd);
  free(xs);
  free(g);
  free(dy);
  return 0;
}
