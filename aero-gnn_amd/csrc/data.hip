// Device-side data preparation of the aero meshes: edge / node feature
// construction and normalisation (dataset.py:39-106, :358-409) and the PyG collate of a batch of
// meshes (train.py:50-51; torch_geometric Batch.from_data_list). The reference runs these in
// Python on the host per mesh; here they are single passes over the device arrays.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

// edge e (output row i; e = perm ? perm[i] : i): d = pos[dst] - pos[src], |d| (dataset.py:52-62),
// then optionally (v - mean) / std per column (dataset.py:403). The norm accumulates the squares
// with fused multiply-adds in component order, sqrt in fp32 (torch's CPU reduction order; it can
// differ from torch CPU by one ulp where its vectorised path regroups).
__global__ void edge_features_kernel(int ne, int64_t e_total, int pdim, const int64_t* __restrict__ ei,
                                     const float* __restrict__ pos,
                                     int pos_ld, const int64_t* __restrict__ perm, const float* __restrict__ mean,
                                     const float* __restrict__ std, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ne) return;
  const int64_t e = perm ? perm[i] : i;
  const int64_t s = ei[e], d = ei[e_total + e];  // row 1 of the [2][e_total] edge_index
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  float acc = 0.f;
  for (int c = 0; c < pdim; ++c) {
    v[c] = __fsub_rn(pos[d * pos_ld + c], pos[s * pos_ld + c]);
    acc = c == 0 ? __fmul_rn(v[c], v[c]) : __builtin_fmaf(v[c], v[c], acc);
  }
  v[pdim] = sqrtf(acc);
  float* o = out + (size_t)i * (pdim + 1);
  for (int c = 0; c <= pdim; ++c) o[c] = mean ? __fdiv_rn(__fsub_rn(v[c], mean[c]), std[c]) : v[c];
}

// out = (x - mean) / std per column, any row stride; in place allowed
__global__ void normalize_kernel(int n, int k, const float* __restrict__ x, int ld, const float* __restrict__ mean,
                                 const float* __restrict__ std, float* __restrict__ out, int out_ld, int inverse) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n * k) return;
  const int r = (int)(t / k), c = (int)(t - (long)r * k);
  const float v = x[(size_t)r * ld + c];
  float o;
  if (inverse) {
    // separately rounded multiply and add (no FMA contraction): torch's v * std + mean on the host
#pragma clang fp contract(off)
    o = v * std[c] + mean[c];
  } else {
    o = (v - mean[c]) / std[c];
  }
  out[(size_t)r * out_ld + c] = o;
}

// column statistics (torch.std_mean(x, dim=0), unbiased, dataset.py:371-373), deterministic:
// pass 1 per-block fp64 partial sums, pass 2 (one block per column) fixed-order totals -> mean;
// pass 3 partial sums of squared deviations, pass 4 -> std = sqrt(ss / (n - 1)), clamped >= eps
constexpr int ST_ROWS = 4096;
__global__ void colsum64_kernel(int n, int k, const float* __restrict__ x, int ld, const double* __restrict__ mean,
                                double* __restrict__ part) {
  const int c = threadIdx.x;
  if (c >= k) return;
  const int r0 = blockIdx.x * ST_ROWS, r1 = min(n, r0 + ST_ROWS);
  double s = 0.0;
  for (int r = r0; r < r1; ++r) {
    const double v = x[(size_t)r * ld + c];
    s += mean ? (v - mean[c]) * (v - mean[c]) : v;
  }
  part[(size_t)blockIdx.x * k + c] = s;
}
__global__ void colfinish_kernel(int n, int k, int nb, const double* __restrict__ part, double* __restrict__ mean64,
                                 float* __restrict__ mean, float* __restrict__ std, float eps, int second) {
  const int c = threadIdx.x;
  if (c >= k) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[(size_t)b * k + c];
  if (!second) {
    mean64[c] = s / (double)n;
    mean[c] = (float)(s / (double)n);
  } else {
    // torch.std_mean (unbiased: n = 1 gives NaN) then clamp(min=eps), which keeps a NaN
    const float sd = (float)sqrt(s / (double)(n - 1));
    std[c] = sd != sd ? sd : fmaxf(sd, eps);
  }
}

// PyG collate of B meshes already concatenated row-wise: edge e of mesh g gets its node ids
// offset by node_off[g]; batch[v] = g for the nodes of mesh g. edge_off / node_off: exclusive
// prefix sums [B + 1]. edge_index is [2][E] (row 0 = source), int64, updated in place.
__global__ void collate_kernel(int B, int64_t ne, int64_t nn, const int64_t* __restrict__ edge_off,
                               const int64_t* __restrict__ node_off, int64_t* __restrict__ ei,
                               int64_t* __restrict__ batch) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto mesh_of = [&](const int64_t* off, int64_t i) {
    int lo = 0, hi = B;  // last g with off[g] <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= i) lo = mid;
      else hi = mid;
    }
    return lo;
  };
  if (t < ne) {
    const int64_t o = node_off[mesh_of(edge_off, t)];
    ei[t] += o;
    ei[ne + t] += o;
  }
  if (t < nn) batch[t] = mesh_of(node_off, t);
}

inline int status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

int agn_edge_features(int ne, int64_t e_total, int pdim, const int64_t* edge_index, const float* pos, int pos_ld,
                      const int64_t* perm, const float* mean, const float* std, float* out, void* stream) {
  if (ne < 0 || e_total < 0 || pdim < 1 || pdim > 3 || (!mean) != (!std)) return AGN_E_ARG;
  if (!perm && ne > e_total) return AGN_E_SHAPE;
  if (ne == 0) return 0;
  hipLaunchKernelGGL(edge_features_kernel, dim3((ne + 255) / 256), dim3(256), 0, (hipStream_t)stream, ne, e_total,
                     pdim, edge_index, pos, pos_ld, perm, mean, std, out);
  return status();
}

int agn_normalize(int n, int k, const float* x, int ld, const float* mean, const float* std, float* out, int out_ld,
                  int inverse, void* stream) {
  if (n < 0 || k < 1 || !mean || !std) return AGN_E_ARG;
  if (n == 0) return 0;
  const long t = (long)n * k;
  hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, k, x,
                     ld, mean, std, out, out_ld, inverse);
  return status();
}

size_t agn_col_stats_temp_bytes(int n, int k) {
  const int nb = (n + ST_ROWS - 1) / ST_ROWS;
  return sizeof(double) * ((size_t)(nb > 0 ? nb : 1) * k + k);
}

int agn_col_stats(int n, int k, const float* x, int ld, float* mean, float* std, float eps, void* scratch,
                  void* stream) {
  if (n < 1 || k < 1 || k > 256 || !mean || !std || !scratch) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (n + ST_ROWS - 1) / ST_ROWS;
  double* part = reinterpret_cast<double*>(scratch);
  double* m64 = part + (size_t)nb * k;
  hipLaunchKernelGGL(colsum64_kernel, dim3(nb), dim3(256), 0, st, n, k, x, ld, nullptr, part);
  hipLaunchKernelGGL(colfinish_kernel, dim3(1), dim3(256), 0, st, n, k, nb, part, m64, mean, std, eps, 0);
  hipLaunchKernelGGL(colsum64_kernel, dim3(nb), dim3(256), 0, st, n, k, x, ld, m64, part);
  hipLaunchKernelGGL(colfinish_kernel, dim3(1), dim3(256), 0, st, n, k, nb, part, m64, mean, std, eps, 1);
  return status();
}

int agn_collate(int B, int64_t ne, int64_t nn, const int64_t* edge_off, const int64_t* node_off, int64_t* edge_index,
                int64_t* batch, void* stream) {
  if (B < 1 || ne < 0 || nn < 0) return AGN_E_ARG;
  const int64_t t = ne > nn ? ne : nn;
  if (t == 0) return 0;
  hipLaunchKernelGGL(collate_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B, ne, nn,
                     edge_off, node_off, edge_index, batch);
  return status();
}

}  // extern "C"
