// float64 mode of the MLP / GMP path (train.py:20-40 "double"/"float64": every parameter and
// activation in fp64). CDNA4 has no fp64 MFMA shape that fits the bf16 kernels' tiles, and this
// precision serves validation runs, not the headline, so these are plain LDS-tiled FMA kernels:
//   agn_f64_gemm       out = epilogue(sum_seg A_seg . B_seg): Linear forward (B = W^T) and input
//                      gradient (B = W), gathered A rows, bias / addends / ReLU / ReLU-mask epilogue
//   agn_f64_wgrad      dW = G^T X (+ db = colsum G), row splits reduced in a fixed order
//   agn_f64_layernorm_{fwd,bwd}   torch.nn.LayerNorm (biased variance), residual add, fixed-order
//                      parameter-gradient reduction
// Everything is deterministic (no atomics).
#include "common.hpp"
#include "aerognn.h"

namespace {

inline int status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// ------------------------------------------------------------------------------ GEMM
constexpr int GT = 64;   // output tile edge
constexpr int GK = 16;   // k chunk
constexpr int GTHR = 256;

// MLP hidden activations in float64 (AGN_ACT_*; torch's formulas, as common.hpp act_fwd / act_bwd)
AGN_DEV double act_fwd64(int k, double x) {
  if (k == AGN_ACT_GELU) return x * 0.5 * (1.0 + erf(x * 0.70710678118654752440));
  if (k == AGN_ACT_SILU) return x / (1.0 + exp(-x));
  if (k == AGN_ACT_TANH) return tanh(x);
  return x > 0.0 ? x : 0.0;
}
AGN_DEV double act_bwd64(int k, double x, double dy) {
  if (k == AGN_ACT_GELU) {
    const double cdf = 0.5 * (1.0 + erf(x * 0.70710678118654752440));
    const double pdf = exp(-0.5 * x * x) * 0.39894228040143267794;
    return dy * (cdf + x * pdf);
  }
  if (k == AGN_ACT_SILU) {
    const double sg = 1.0 / (1.0 + exp(-x));
    return dy * sg * (1.0 + x * (1.0 - sg));
  }
  if (k == AGN_ACT_TANH) {
    const double y = tanh(x);
    return dy * (1.0 - y * y);
  }
  return x > 0.0 ? dy : 0.0;
}

__global__ __launch_bounds__(GTHR) void f64_gemm_kernel(const agn_f64_gemm_args a) {
  __shared__ double As[GK][GT + 1];
  __shared__ double Bs[GK][GT + 1];
  const int r0 = blockIdx.x * GT, n0 = blockIdx.y * GT;
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int s = 0; s < a.nseg; ++s) {
    const agn_f64_seg& sg = a.seg[s];
    for (int k0 = 0; k0 < sg.k; k0 += GK) {
      __syncthreads();
      // A chunk: 64 rows x 16 k (4 per thread), B chunk: 16 k x 64 n (4 per thread)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = threadIdx.x + q * GTHR;
        const int rr = e >> 4, kk = e & 15;
        const int row = r0 + rr, kc = k0 + kk;
        double v = 0.0;
        if (row < a.rows && kc < sg.k) {
          const long ar = sg.aidx ? sg.aidx[row] : row;
          v = sg.a[ar * (long)sg.lda + kc];
        }
        As[kk][rr] = v;
        // (a transposed W is read along k: consecutive threads take consecutive k)
        const int kk2 = sg.transw ? (e & 15) : (e >> 6), nn = sg.transw ? (e >> 4) : (e & 63);
        const int n = n0 + nn, kc2 = k0 + kk2;
        double w = 0.0;
        if (n < a.n && kc2 < sg.k) w = sg.transw ? sg.w[(long)n * sg.ldw + kc2] : sg.w[(long)kc2 * sg.ldw + n];
        Bs[kk2][nn] = w;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < GK; ++kk) {
        double av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = As[kk][tr + 16 * i];
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tc + 16 * j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fma(av[i], bv[j], acc[i][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = r0 + tr + 16 * i;
    if (row >= a.rows) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tc + 16 * j;
      if (n >= a.n) continue;
      double v = acc[i][j];
      if (a.bias) v += a.bias[n];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (a.add[q]) {
          const long ar = a.add_idx[q] ? a.add_idx[q][row] : row;
          v += a.add[q][ar * (long)a.add_ld[q] + n];
        }
      if (a.mask) {
        const double m = a.mask[(long)row * a.mask_ld + n];
        if (a.mask_act == 0) {
          if (!(m > 0.0)) v = 0.0;  // ReLU backward on the saved activation
        } else {
          v = act_bwd64(a.mask_act - 1, m, v);  // f'(pre-activation)
        }
      }
      if (a.pre_out) a.pre_out[(long)row * a.pre_ld + n] = v;
      if (a.relu == 1) v = v > 0.0 ? v : 0.0;
      else if (a.relu > 1) v = act_fwd64(a.relu - 1, v);
      a.out[(long)row * a.out_ld + n] = v;
    }
  }
}

// ------------------------------------------------------------------------------ dW = G^T X
// grid (m blocks, k blocks, splits): block (mb, kb, s) sums rows [s*per, (s+1)*per) into the
// partial slab [s][mpad][kpad]; f64_wgrad_reduce adds the splits in order.
__global__ __launch_bounds__(GTHR) void f64_wgrad_kernel(const agn_f64_wgrad_args a, int per, double* part,
                                                         double* bpart) {
  __shared__ double Gs[GK][GT + 1];
  __shared__ double Xs[GK][GT + 1];
  const int m0 = blockIdx.x * GT, k0 = blockIdx.y * GT, s = blockIdx.z;
  const int mpad = gridDim.x * GT, kpad = gridDim.y * GT;
  const int rb = s * per, re = min(a.rows, rb + per);
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  double bsum = 0.0;  // threads 0..63 of the kb == 0 blocks: column m0 + tid of G
  for (int r = rb; r < re; r += GK) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = threadIdx.x + q * GTHR;
      const int rr = e >> 6, cc = e & 63;
      const int row = r + rr;
      double g = 0.0, x = 0.0;
      if (row < re) {
        if (m0 + cc < a.m) g = a.g[(long)row * a.ldg + m0 + cc];
        if (k0 + cc < a.k) {
          const long xr = a.xidx ? a.xidx[row] : row;
          x = a.x[xr * (long)a.ldx + k0 + cc];
        }
      }
      Gs[rr][cc] = g;
      Xs[rr][cc] = x;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      double gv[4], xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) gv[i] = Gs[kk][tr + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = Xs[kk][tc + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fma(gv[i], xv[j], acc[i][j]);
    }
    if (bpart && blockIdx.y == 0 && threadIdx.x < GT) {
#pragma unroll
      for (int kk = 0; kk < GK; ++kk) bsum += Gs[kk][threadIdx.x];
    }
  }
  double* P = part + (size_t)s * mpad * kpad;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) P[(size_t)(m0 + tr + 16 * i) * kpad + k0 + tc + 16 * j] = acc[i][j];
  if (bpart && blockIdx.y == 0 && threadIdx.x < GT) bpart[(size_t)s * mpad + m0 + threadIdx.x] = bsum;
}

__global__ __launch_bounds__(256) void f64_wgrad_reduce(const agn_f64_wgrad_args a, int nsplit, int mpad, int kpad,
                                                        const double* part, const double* bpart) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nw = (long)a.m * a.k;
  if (t < nw) {
    const int m = (int)(t / a.k), k = (int)(t - (long)m * a.k);
    double v = 0.0;
    for (int s = 0; s < nsplit; ++s) v += part[(size_t)s * mpad * kpad + (size_t)m * kpad + k];
    a.dw[(long)m * a.ldw + k] = v;
  } else if (a.db && t < nw + a.m) {
    const int m = (int)(t - nw);
    double v = 0.0;
    for (int s = 0; s < nsplit; ++s) v += bpart[(size_t)s * mpad + m];
    a.db[m] = v;
  }
}

void wgrad_plan(const agn_f64_wgrad_args& a, int& mb, int& kb, int& ns, int& per) {
  mb = (a.m + GT - 1) / GT;
  kb = (a.k + GT - 1) / GT;
  const int target = 1024;  // blocks
  ns = max(1, min((a.rows + 255) / 256, target / (mb * kb)));
  per = ((a.rows + ns - 1) / ns + GK - 1) / GK * GK;
  ns = max(1, (a.rows + per - 1) / per);
}

// ------------------------------------------------------------------------------ LayerNorm
// one wave per row; lane l holds features l, l + 64, ... (n <= 64 * LN_PER)
constexpr int LN_PER = 16;

AGN_DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void f64_ln_fwd_kernel(int rows, int n, const double* x, int ldx, const double* g,
                                                         const double* b, const double* resid, int ldr, double* y,
                                                         int ldy, double* mean_o, double* rstd_o, double eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  double v[LN_PER];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < LN_PER; ++i) {
    const int f = lane + 64 * i;
    v[i] = f < n ? x[(long)row * ldx + f] : 0.0;
    s += v[i];
  }
  const double mean = wave_sum(s) / n;
  double q = 0.0;
#pragma unroll
  for (int i = 0; i < LN_PER; ++i)
    if (lane + 64 * i < n) q += (v[i] - mean) * (v[i] - mean);
  const double rstd = 1.0 / sqrt(wave_sum(q) / n + eps);
#pragma unroll
  for (int i = 0; i < LN_PER; ++i) {
    const int f = lane + 64 * i;
    if (f >= n) continue;
    double o = (v[i] - mean) * rstd * (g ? g[f] : 1.0) + (b ? b[f] : 0.0);
    if (resid) o += resid[(long)row * ldr + f];
    y[(long)row * ldy + f] = o;
  }
  if (lane == 0) {
    mean_o[row] = mean;
    rstd_o[row] = rstd;
  }
}

// dx = rstd (dxhat - mean(dxhat) - xhat mean(dxhat xhat)), dxhat = dy gamma; per block partials of
// dgamma = sum dy xhat and dbeta = sum dy over its LN_RB rows, reduced in block order afterwards
constexpr int LN_RB = 64;
__global__ __launch_bounds__(256) void f64_ln_bwd_kernel(int rows, int n, const double* dy, int lddy, const double* x,
                                                         int ldx, const double* mean_i, const double* rstd_i,
                                                         const double* g, double* dx, int lddx, double* part) {
  __shared__ double red[4][2][64 * 4];  // per wave, n <= 256 in the partial staging (larger n: 4 passes)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double pg[LN_PER], pb[LN_PER];
#pragma unroll
  for (int i = 0; i < LN_PER; ++i) pg[i] = pb[i] = 0.0;
  const int rb = blockIdx.x * LN_RB, re = min(rows, rb + LN_RB);
  for (int row = rb + w; row < re; row += 4) {
    const double mean = mean_i[row], rstd = rstd_i[row];
    double xh[LN_PER], d[LN_PER];
    double c1 = 0.0, c2 = 0.0;
#pragma unroll
    for (int i = 0; i < LN_PER; ++i) {
      const int f = lane + 64 * i;
      if (f < n) {
        const double gy = dy[(long)row * lddy + f];
        xh[i] = (x[(long)row * ldx + f] - mean) * rstd;
        d[i] = gy * (g ? g[f] : 1.0);
        c1 += d[i];
        c2 += d[i] * xh[i];
        pg[i] += gy * xh[i];
        pb[i] += gy;
      } else {
        xh[i] = d[i] = 0.0;
      }
    }
    c1 = wave_sum(c1) / n;
    c2 = wave_sum(c2) / n;
#pragma unroll
    for (int i = 0; i < LN_PER; ++i) {
      const int f = lane + 64 * i;
      if (f < n) dx[(long)row * lddx + f] = rstd * (d[i] - c1 - xh[i] * c2);
    }
  }
  if (!part) return;
  // the four waves' partials in wave order, 256 features per pass
  for (int p0 = 0; p0 < LN_PER; p0 += 4) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      red[w][0][lane + 64 * i] = pg[p0 + i];
      red[w][1][lane + 64 * i] = pb[p0 + i];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 2 * 256; t += 256) {
      const int q = t >> 8, fl = t & 255, f = 64 * p0 + fl;
      if (f < n) {
        const double v = ((red[0][q][fl] + red[1][q][fl]) + red[2][q][fl]) + red[3][q][fl];
        part[(size_t)blockIdx.x * 2 * n + q * n + f] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void f64_colsum_kernel(const double* part, int nblk, int n2, double* out0,
                                                         double* out1, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n2) return;
  double v = 0.0;
  for (int b = 0; b < nblk; ++b) v += part[(size_t)b * n2 + t];
  if (t < n) {
    if (out0) out0[t] = v;
  } else if (out1) {
    out1[t - n] = v;
  }
}

}  // namespace

extern "C" {

int agn_f64_gemm(const agn_f64_gemm_args* a, void* stream) {
  if (!a || a->rows < 0 || a->n < 1 || a->nseg < 0 || a->nseg > 3 || !a->out) return AGN_E_ARG;
  for (int s = 0; s < a->nseg; ++s)
    if (a->seg[s].k < 0 || (a->seg[s].k > 0 && (!a->seg[s].a || !a->seg[s].w))) return AGN_E_ARG;
  if (a->rows == 0) return 0;
  const dim3 grid((a->rows + GT - 1) / GT, (a->n + GT - 1) / GT);
  hipLaunchKernelGGL(f64_gemm_kernel, grid, dim3(GTHR), 0, (hipStream_t)stream, *a);
  return status();
}

size_t agn_f64_wgrad_scratch_bytes(const agn_f64_wgrad_args* a) {
  if (!a || a->rows <= 0) return 0;
  int mb, kb, ns, per;
  wgrad_plan(*a, mb, kb, ns, per);
  return (size_t)ns * (mb * GT) * ((size_t)kb * GT + 1) * sizeof(double);
}

int agn_f64_wgrad(const agn_f64_wgrad_args* a, void* scratch, void* stream) {
  if (!a || a->rows < 0 || a->m < 1 || a->k < 1 || !a->dw) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (a->rows == 0) {
    for (int m = 0; m < a->m; ++m)
      if (hipMemsetAsync(a->dw + (size_t)m * a->ldw, 0, sizeof(double) * a->k, st) != hipSuccess) return AGN_E_ARG;
    if (a->db && hipMemsetAsync(a->db, 0, sizeof(double) * a->m, st) != hipSuccess) return AGN_E_ARG;
    return status();
  }
  if (!scratch) return AGN_E_ARG;
  int mb, kb, ns, per;
  wgrad_plan(*a, mb, kb, ns, per);
  double* part = reinterpret_cast<double*>(scratch);
  double* bpart = a->db ? part + (size_t)ns * (mb * GT) * (kb * GT) : nullptr;
  hipLaunchKernelGGL(f64_wgrad_kernel, dim3(mb, kb, ns), dim3(GTHR), 0, st, *a, per, part, bpart);
  const long tot = (long)a->m * a->k + (a->db ? a->m : 0);
  hipLaunchKernelGGL(f64_wgrad_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, *a, ns, mb * GT, kb * GT,
                     part, bpart);
  return status();
}

int agn_f64_layernorm_fwd(int rows, int n, const double* x, int ldx, const double* gamma, const double* beta,
                          const double* resid, int ldr, double* y, int ldy, double* mean, double* rstd, double eps,
                          void* stream) {
  if (rows < 0 || n < 1 || n > 64 * LN_PER || !x || !y || !mean || !rstd) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(f64_ln_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, n, x, ldx,
                     gamma, beta, resid, ldr, y, ldy, mean, rstd, eps);
  return status();
}

size_t agn_f64_layernorm_bwd_scratch_bytes(int rows, int n) {
  return (size_t)((rows + LN_RB - 1) / LN_RB) * 2 * n * sizeof(double);
}

int agn_f64_layernorm_bwd(int rows, int n, const double* dy, int lddy, const double* x, int ldx, const double* mean,
                          const double* rstd, const double* gamma, double* dx, int lddx, double* dgamma,
                          double* dbeta, void* scratch, void* stream) {
  if (rows < 0 || n < 1 || n > 64 * LN_PER || !dy || !x || !mean || !rstd || !dx) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const bool pgrad = dgamma || dbeta;
  if (rows == 0) {
    if (dgamma && hipMemsetAsync(dgamma, 0, sizeof(double) * n, st) != hipSuccess) return AGN_E_ARG;
    if (dbeta && hipMemsetAsync(dbeta, 0, sizeof(double) * n, st) != hipSuccess) return AGN_E_ARG;
    return status();
  }
  if (pgrad && !scratch) return AGN_E_ARG;
  const int nblk = (rows + LN_RB - 1) / LN_RB;
  hipLaunchKernelGGL(f64_ln_bwd_kernel, dim3(nblk), dim3(256), 0, st, rows, n, dy, lddy, x, ldx, mean, rstd, gamma,
                     dx, lddx, pgrad ? reinterpret_cast<double*>(scratch) : nullptr);
  if (pgrad)
    hipLaunchKernelGGL(f64_colsum_kernel, dim3((2 * n + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const double*>(scratch), nblk, 2 * n, dgamma, dbeta, n);
  return status();
}

}  // extern "C"
