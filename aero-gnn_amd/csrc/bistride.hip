// BSMS-GNN bi-stride operators (gfx950): the stale `models/bistride_ops` + old `bsms_mgn`
// design recovered in SURVEY Appendix A — BFS hop distances, even-level (bi-stride) node
// selection, sub-graph extraction, row scatter for Unpool, and the fused WeightedEdgeConv.
//
// Determinism: BFS distances are order-independent; selections/sub-graphs are order-preserving
// compactions (scan); WeightedEdgeConv sums walk CSC (by receiver) / CSR (by sender) groups in
// edge order, and its parameter-gradient partials are reduced in a fixed order. No float atomics.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
inline dim3 grid1(long n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

// ------------------------------------------------------------------------------ BFS
__global__ void fill_i32_kernel(int32_t* p, int n, int v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void bfs_init_kernel(int32_t* dist, int32_t* frontier, int32_t* cnt, int seed) {
  dist[seed] = 0;
  frontier[0] = seed;
  cnt[0] = 1;
  cnt[1] = 0;
  cnt[2] = 0;
}

// Expand one BFS level: every frontier node u visits its out-neighbours (edge_index[0] -> [1],
// bistride_ops @21); an unvisited v gets dist = level + 1 (first writer wins; every writer
// writes the same value, so the distances do not depend on the order) and joins the next
// frontier. Counters rotate over 3 slots: in = cnt[L%3], out = cnt[(L+1)%3], and the slot
// two levels ahead is cleared here for the next launch.
__global__ __launch_bounds__(256) void bfs_expand_kernel(const int32_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ nbr, int32_t* dist,
                                                         const int32_t* __restrict__ fin, int32_t* fout,
                                                         int32_t* cnt, int level) {
  const int nin = cnt[level % 3];
  int32_t* nout = cnt + (level + 1) % 3;
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(level + 2) % 3] = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nin; i += gridDim.x * blockDim.x) {
    const int u = fin[i];
    for (int j = rowptr[u]; j < rowptr[u + 1]; ++j) {
      const int v = nbr[j];
      if (atomicCAS(&dist[v], -1, level + 1) == -1) {
        const int p = atomicAdd(nout, 1);
        fout[p] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------ seeds
// argmin over n of |pos_i - mean(pos)|_2 (first index on ties), bistride_ops @56: one block.
__global__ __launch_bounds__(1024) void center_seed_kernel(const float* __restrict__ pos, int n, int pdim, int ld,
                                                           int32_t* seed) {
  __shared__ double red[1024];
  __shared__ float mean[4];
  __shared__ float bv[1024];
  __shared__ int bi[1024];
  for (int d = 0; d < pdim; ++d) {
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += 1024) s += (double)pos[(size_t)i * ld + d];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) mean[d] = (float)(red[0] / (double)n);
    __syncthreads();
  }
  float best = INFINITY;
  int besti = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 1024) {
    float q = 0.f;
    for (int d = 0; d < pdim; ++d) {
      const float t = pos[(size_t)i * ld + d] - mean[d];
      q += t * t;
    }
    const float r = sqrtf(q);
    if (r < best) { best = r; besti = i; }  // i increases: first index kept on ties
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const float o = bv[threadIdx.x + w];
      const int oi = bi[threadIdx.x + w];
      if (o < bv[threadIdx.x] || (o == bv[threadIdx.x] && oi < bi[threadIdx.x])) {
        bv[threadIdx.x] = o;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *seed = bi[0] == 0x7fffffff ? 0 : bi[0];
}

// argmax_i (rowptr[i+1] - rowptr[i]) = argmax bincount(edge_index[0]) (first index on ties)
__global__ __launch_bounds__(1024) void maxdeg_seed_kernel(const int32_t* __restrict__ rowptr, int n, int32_t* seed) {
  __shared__ int bv[1024];
  __shared__ int bi[1024];
  int best = -1, besti = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const int d = rowptr[i + 1] - rowptr[i];
    if (d > best) { best = d; besti = i; }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const int o = bv[threadIdx.x + w], oi = bi[threadIdx.x + w];
      if (o > bv[threadIdx.x] || (o == bv[threadIdx.x] && oi < bi[threadIdx.x])) {
        bv[threadIdx.x] = o;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *seed = bi[0] == 0x7fffffff ? 0 : bi[0];
}

// ------------------------------------------------------------------------------ compactions
__global__ void select_flags_kernel(const int32_t* __restrict__ dist, int n, int even_only, int32_t* flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = dist[i];
  flags[i] = even_only ? (d >= 0 && (d % 2) == 0) : (d >= 0);
}

__global__ void compact_index_kernel(const int32_t* __restrict__ flags, const int32_t* __restrict__ pos, int n,
                                     int32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flags[i]) out[pos[i]] = i;
}

__global__ void index_map_kernel(const int32_t* __restrict__ sel, int nsel, int32_t* map) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nsel) map[sel[j]] = j;
}

__global__ void subgraph_flags_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int e,
                                      const int32_t* __restrict__ map, int32_t* flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e) return;
  const int a = map[src[i]], b = map[dst[i]];
  flags[i] = (a >= 0 && b >= 0 && a != b);
}

__global__ void subgraph_emit_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int e,
                                     const int32_t* __restrict__ map, const int32_t* __restrict__ flags,
                                     const int32_t* __restrict__ pos, int64_t* osrc, int64_t* odst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e || !flags[i]) return;
  osrc[pos[i]] = map[src[i]];
  odst[pos[i]] = map[dst[i]];
}

// out[idx[j]] = src[j] (16 B per thread)
template <typename T>
__global__ __launch_bounds__(256) void scatter_rows_kernel(int rows, int k, const int32_t* __restrict__ idx,
                                                           const T* __restrict__ src, int src_ld, T* out, int out_ld) {
  constexpr int PER = 16 / sizeof(T);
  const int sub = threadIdx.x & 15;
  const int r = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (r >= rows) return;
  const T* s = src + (size_t)r * src_ld;
  T* o = out + (size_t)idx[r] * out_ld;
  for (int f = sub * PER; f < k; f += 16 * PER) {
    if (f + PER <= k && ((src_ld | out_ld) % PER) == 0 && ((((uintptr_t)s) | ((uintptr_t)o)) & 15) == 0) {
      *reinterpret_cast<uint4*>(o + f) = *reinterpret_cast<const uint4*>(s + f);
    } else {
      for (int e = 0; e < PER && f + e < k; ++e) o[f + e] = s[f + e];
    }
  }
}

// ------------------------------------------------------------------------------ WeightedEdgeConv
// bistride_ops @131-210: w_e = sigmoid(w2 . relu(W1 [x_src, x_dst, |pos_dst - pos_src|] + b1) + b2),
// out_v = sum_{e: dst_e = v} (T x + b_T)[src_e] * w_e   ('mean': / max(deg, 1)).
// W1 x is split per node (sum trick): P_a = x W1a^T, P_b = x W1b^T + b1 ([n][hid] each, one node
// GEMM), so an edge costs a 64-wide dot product on VALU. 16 lanes own one receiver: each lane
// holds OUT/16 output features and HID/16 = 4 hidden units; all sums fp32, in CSC edge order.
constexpr int WEC_G = 16;
constexpr int WEC_HID = 64;
constexpr int WEC_HL = WEC_HID / WEC_G;  // 4 hidden units per lane

AGN_DEV float red16(float v) {
  v += __shfl_xor(v, 8, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 1, 16);
  return v;
}

template <typename T, int N>
AGN_DEV void ldv(float (&o)[N], const T* p) {
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    const f32x4 x = load4(p + i);
    o[i] = x[0]; o[i + 1] = x[1]; o[i + 2] = x[2]; o[i + 3] = x[3];
  }
}
template <typename T, int N>
AGN_DEV void stv(T* p, const float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; i += 4) store4(p + i, f32x4{v[i], v[i + 1], v[i + 2], v[i + 3]});
}

AGN_DEV float edge_len(const float* pos, int ld, int pdim, int u, int v) {
  float q = 0.f;
  for (int d = 0; d < pdim; ++d) {
    const float t = pos[(size_t)v * ld + d] - pos[(size_t)u * ld + d];
    q += t * t;
  }
  return sqrtf(q);
}

// recompute the edge weight: returns fp32 sigmoid; h[] = relu pre-activations, len
template <typename T>
AGN_DEV float wec_weight(const agn_wec_args& a, int u, int v, const float (&pb)[WEC_HL], const float (&w1c)[WEC_HL],
                         const float (&w2)[WEC_HL], int sub, float (&h)[WEC_HL], float& len) {
  float pa[WEC_HL];
  ldv<T, WEC_HL>(pa, reinterpret_cast<const T*>(a.pab) + (size_t)u * (2 * WEC_HID) + WEC_HL * sub);
  len = edge_len(a.pos, a.pos_ld, a.pos_dim, u, v);
  float part = 0.f;
#pragma unroll
  for (int k = 0; k < WEC_HL; ++k) {
    h[k] = fmaxf(pa[k] + pb[k] + len * w1c[k], 0.f);
    part += h[k] * w2[k];
  }
  const float logit = red16(part) + a.w2[WEC_HID];  // w2 = [w2 | b2]
  return 1.f / (1.f + __expf(-logit));
}

template <typename T, int OUT>
__global__ __launch_bounds__(256) void wec_fwd_kernel(const agn_wec_args a) {
  constexpr int OL = OUT / WEC_G;
  const int sub = threadIdx.x & (WEC_G - 1);
  const int v = blockIdx.x * (256 / WEC_G) + threadIdx.x / WEC_G;
  if (v >= a.n) return;  // whole 16-lane group leaves together
  const bool compute = a.w_in == nullptr;
  float pb[WEC_HL], w1c[WEC_HL], w2[WEC_HL];
  if (compute) {
    ldv<T, WEC_HL>(pb, reinterpret_cast<const T*>(a.pab) + (size_t)v * (2 * WEC_HID) + WEC_HID + WEC_HL * sub);
#pragma unroll
    for (int k = 0; k < WEC_HL; ++k) { w1c[k] = a.w1c[WEC_HL * sub + k]; w2[k] = a.w2[WEC_HL * sub + k]; }
  }
  float acc[OL];
#pragma unroll
  for (int i = 0; i < OL; ++i) acc[i] = 0.f;
  const int beg = a.rowptr[v], end = a.rowptr[v + 1];
  for (int j = beg; j < end; ++j) {
    const int u = a.src[j];
    float s;
    if (compute) {
      float h[WEC_HL], len;
      s = round_t<T>(wec_weight<T>(a, u, v, pb, w1c, w2, sub, h, len));
      if (sub == 0 && a.w_out) reinterpret_cast<T*>(a.w_out)[a.perm[j]] = from_f<T>(s);
    } else {
      s = to_f(reinterpret_cast<const T*>(a.w_in)[a.perm[j]]);
    }
    if (a.out) {
      float tx[OL];
      ldv<T, OL>(tx, reinterpret_cast<const T*>(a.tx) + (size_t)u * OUT + OL * sub);
#pragma unroll
      for (int i = 0; i < OL; ++i) acc[i] += round_t<T>(tx[i] * s);  // message m = Tx[src] * w (dtype)
    }
  }
  if (!a.out) return;  // compute_edge_weights alone
  if (a.mean) {
    const float c = (float)max(end - beg, 1);
#pragma unroll
    for (int i = 0; i < OL; ++i) acc[i] /= c;
  }
  stv<T, OL>(reinterpret_cast<T*>(a.out) + (size_t)v * OUT + OL * sub, acc);
}

// backward, receiver side: ds_e = <Tx[src], dout[dst]>, then through the sigmoid / ReLU of the
// weight MLP: dh_e (kept fp32 per CSC edge for the sender-side sum), dP_b[v] = sum dh_e, and the
// per-block partials of dw2, dw1c, db2 (fixed-order reduced on the host side by agn_colsum).
template <typename T, int OUT>
__global__ __launch_bounds__(256) void wec_bwd_dst_kernel(const agn_wec_args a) {
  constexpr int OL = OUT / WEC_G;
  constexpr int NG = 256 / WEC_G;
  __shared__ float red[NG][2 * WEC_HID + 1];
  const int sub = threadIdx.x & (WEC_G - 1);
  const int grp = threadIdx.x / WEC_G;
  const int v = blockIdx.x * NG + grp;
  const bool compute = a.w_in == nullptr;
  float dw2p[WEC_HL], dw1p[WEC_HL], db2p = 0.f;
#pragma unroll
  for (int k = 0; k < WEC_HL; ++k) { dw2p[k] = 0.f; dw1p[k] = 0.f; }
  if (v < a.n) {
    float pb[WEC_HL], w1c[WEC_HL], w2[WEC_HL];
    if (compute) {
      ldv<T, WEC_HL>(pb, reinterpret_cast<const T*>(a.pab) + (size_t)v * (2 * WEC_HID) + WEC_HID + WEC_HL * sub);
#pragma unroll
      for (int k = 0; k < WEC_HL; ++k) { w1c[k] = a.w1c[WEC_HL * sub + k]; w2[k] = a.w2[WEC_HL * sub + k]; }
    }
    const int beg = a.rowptr[v], end = a.rowptr[v + 1];
    float dv[OL];
    ldv<T, OL>(dv, reinterpret_cast<const T*>(a.dout) + (size_t)v * OUT + OL * sub);
    if (a.mean) {
      const float c = (float)max(end - beg, 1);
#pragma unroll
      for (int i = 0; i < OL; ++i) dv[i] /= c;
    }
    float dpb[WEC_HL];
#pragma unroll
    for (int k = 0; k < WEC_HL; ++k) dpb[k] = 0.f;
    for (int j = beg; j < end; ++j) {
      const int u = a.src[j];
      float tx[OL];
      ldv<T, OL>(tx, reinterpret_cast<const T*>(a.tx) + (size_t)u * OUT + OL * sub);
      float part = 0.f;
#pragma unroll
      for (int i = 0; i < OL; ++i) part += tx[i] * dv[i];
      const float ds = red16(part);
      const long pe = a.perm[j];
      if (compute) {
        float h[WEC_HL], len;
        const float s = wec_weight<T>(a, u, v, pb, w1c, w2, sub, h, len);
        if (sub == 0) a.s_csc[j] = round_t<T>(s);
        const float gs = ds + (a.gw ? to_f(reinterpret_cast<const T*>(a.gw)[pe]) : 0.f);
        const float dl = gs * s * (1.f - s);
        float dh[WEC_HL];
#pragma unroll
        for (int k = 0; k < WEC_HL; ++k) {
          dh[k] = h[k] > 0.f ? dl * w2[k] : 0.f;
          dpb[k] += dh[k];
          dw2p[k] += dl * h[k];
          dw1p[k] += dh[k] * len;
        }
        db2p += dl;
        *reinterpret_cast<f32x4*>(a.dh + (size_t)j * WEC_HID + WEC_HL * sub) = f32x4{dh[0], dh[1], dh[2], dh[3]};
      } else {
        if (sub == 0) {
          a.s_csc[j] = to_f(reinterpret_cast<const T*>(a.w_in)[pe]);
          if (a.dw_in) reinterpret_cast<T*>(a.dw_in)[pe] = from_f<T>(ds);
        }
      }
    }
    if (compute) stv<T, WEC_HL>(reinterpret_cast<T*>(a.dpb) + (size_t)v * WEC_HID + WEC_HL * sub, dpb);
  }
  if (!compute || !a.partial) return;
#pragma unroll
  for (int k = 0; k < WEC_HL; ++k) {
    red[grp][WEC_HL * sub + k] = dw2p[k];
    red[grp][WEC_HID + WEC_HL * sub + k] = dw1p[k];
  }
  if (sub == 0) red[grp][2 * WEC_HID] = db2p;
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * WEC_HID + 1; i += 256) {
    float s = 0.f;
    for (int g = 0; g < NG; ++g) s += red[g][i];
    a.partial[(size_t)blockIdx.x * (2 * WEC_HID + 1) + i] = s;
  }
}

// backward, sender side (CSR groups): dTx[u] = sum_e s_e dout[dst_e] (/deg), dP_a[u] = sum_e dh_e
template <typename T, int OUT>
__global__ __launch_bounds__(256) void wec_bwd_src_kernel(const agn_wec_args a) {
  constexpr int OL = OUT / WEC_G;
  const int sub = threadIdx.x & (WEC_G - 1);
  const int u = blockIdx.x * (256 / WEC_G) + threadIdx.x / WEC_G;
  if (u >= a.n) return;
  const bool compute = a.w_in == nullptr;
  float dtx[OL], dpa[WEC_HL];
#pragma unroll
  for (int i = 0; i < OL; ++i) dtx[i] = 0.f;
#pragma unroll
  for (int k = 0; k < WEC_HL; ++k) dpa[k] = 0.f;
  for (int q = a.rowptr_src[u]; q < a.rowptr_src[u + 1]; ++q) {
    const int j = a.perm_src[q];
    const int v = a.dst[j];
    float s = a.s_csc[j];
    if (a.mean) s /= (float)max(a.rowptr[v + 1] - a.rowptr[v], 1);
    float dv[OL];
    ldv<T, OL>(dv, reinterpret_cast<const T*>(a.dout) + (size_t)v * OUT + OL * sub);
#pragma unroll
    for (int i = 0; i < OL; ++i) dtx[i] += s * dv[i];
    if (compute) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(a.dh + (size_t)j * WEC_HID + WEC_HL * sub);
#pragma unroll
      for (int k = 0; k < WEC_HL; ++k) dpa[k] += d[k];
    }
  }
  stv<T, OL>(reinterpret_cast<T*>(a.dtx) + (size_t)u * OUT + OL * sub, dtx);
  if (compute) stv<T, WEC_HL>(reinterpret_cast<T*>(a.dpa) + (size_t)u * WEC_HID + WEC_HL * sub, dpa);
}

#define WEC_DISPATCH(KERNEL, GRID)                                                                   \
  do {                                                                                               \
    hipStream_t st = (hipStream_t)stream;                                                            \
    if (a->dtype == AGN_F32) {                                                                       \
      if (a->out_dim == 128) hipLaunchKernelGGL((KERNEL<float, 128>), GRID, dim3(256), 0, st, *a);   \
      else if (a->out_dim == 64) hipLaunchKernelGGL((KERNEL<float, 64>), GRID, dim3(256), 0, st, *a); \
      else return AGN_E_SHAPE;                                                                       \
    } else if (a->dtype == AGN_BF16) {                                                               \
      if (a->out_dim == 128) hipLaunchKernelGGL((KERNEL<bf16, 128>), GRID, dim3(256), 0, st, *a);    \
      else if (a->out_dim == 64) hipLaunchKernelGGL((KERNEL<bf16, 64>), GRID, dim3(256), 0, st, *a);  \
      else return AGN_E_SHAPE;                                                                       \
    } else if (a->dtype == AGN_F16) {                                                                \
      if (a->out_dim == 128) hipLaunchKernelGGL((KERNEL<f16, 128>), GRID, dim3(256), 0, st, *a);     \
      else if (a->out_dim == 64) hipLaunchKernelGGL((KERNEL<f16, 64>), GRID, dim3(256), 0, st, *a);   \
      else return AGN_E_SHAPE;                                                                       \
    } else {                                                                                         \
      return AGN_E_DTYPE;                                                                            \
    }                                                                                                \
  } while (0)

int wec_check(const agn_wec_args* a) {
  if (!a || a->n < 0 || a->e < 0 || a->hid != WEC_HID || a->pos_dim < 0 || a->pos_dim > 4) return AGN_E_ARG;
  if (a->w_in == nullptr && (a->pab == nullptr || a->pos == nullptr || a->w1c == nullptr || a->w2 == nullptr))
    return AGN_E_ARG;
  if (a->out != nullptr && a->tx == nullptr) return AGN_E_ARG;
  return 0;
}

}  // namespace

extern "C" {

size_t agn_bfs_work_ints(int n) { return 2 * (size_t)(n > 0 ? n : 1) + 4; }

int agn_bfs_distance(const int32_t* rowptr, const int32_t* nbr, int n, int seed, int32_t* dist, int32_t* work,
                     int* levels_out, void* stream) {
  if (n < 0 || (n > 0 && (seed < 0 || seed >= n))) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return 0;
  int32_t* fa = work;
  int32_t* fb = work + n;
  int32_t* cnt = work + 2 * n;
  hipLaunchKernelGGL(fill_i32_kernel, grid1(n), dim3(256), 0, st, dist, n, -1);
  hipLaunchKernelGGL(bfs_init_kernel, dim3(1), dim3(1), 0, st, dist, fa, cnt, seed);
  const int grid = 2048;
  int level = 0;
  int32_t host_cnt[3];
  for (;;) {
    // a batch of levels without host round trips; empty frontiers make a launch a no-op
    for (int b = 0; b < 32; ++b, ++level) {
      int32_t* fin = (level & 1) ? fb : fa;
      int32_t* fout = (level & 1) ? fa : fb;
      hipLaunchKernelGGL(bfs_expand_kernel, dim3(grid), dim3(256), 0, st, rowptr, nbr, dist, fin, fout, cnt, level);
    }
    hipError_t e = hipMemcpyAsync(host_cnt, cnt, sizeof(host_cnt), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return (int)e;
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    if (host_cnt[level % 3] == 0) break;  // the frontier `level` would expand is empty
    if (level > 4 * n + 64) return AGN_E_ARG;  // cannot happen (depth < n)
  }
  if (levels_out) *levels_out = level;
  return launch_status();
}

int agn_center_seed(const float* pos, int n, int pos_dim, int pos_ld, int32_t* seed, void* stream) {
  if (n < 1 || pos_dim < 1 || pos_dim > 4) return AGN_E_ARG;
  hipLaunchKernelGGL(center_seed_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, pos, n, pos_dim, pos_ld, seed);
  return launch_status();
}

int agn_maxdeg_seed(const int32_t* rowptr, int n, int32_t* seed, void* stream) {
  if (n < 1) return AGN_E_ARG;
  hipLaunchKernelGGL(maxdeg_seed_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rowptr, n, seed);
  return launch_status();
}

size_t agn_compact_work_ints(int n) {
  return 2 * (size_t)(n > 0 ? n : 1) + agn_scan_temp_bytes(n) / sizeof(int32_t) + 4;
}

int agn_bistride_select(const int32_t* dist, int n, int32_t* sel, int* nsel, int32_t* work, void* stream) {
  if (n < 0 || !nsel) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  *nsel = 0;
  if (n == 0) return 0;
  int32_t* flags = work;
  int32_t* pos = work + n;
  int32_t* total = work + 2 * n;
  int32_t* scr = work + 2 * n + 4;
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(select_flags_kernel, grid1(n), dim3(256), 0, st, dist, n, pass == 0 ? 1 : 0, flags);
    int rc = agn_exclusive_scan_i32(flags, pos, n, total, scr, stream);
    if (rc) return rc;
    int32_t cnt = 0;
    hipError_t e = hipMemcpyAsync(&cnt, total, sizeof(cnt), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    // bistride_ops @56: fall back to every reachable node when the even levels keep < 30 %
    if (pass == 0 && (double)cnt < (double)n * 0.3) continue;
    hipLaunchKernelGGL(compact_index_kernel, grid1(n), dim3(256), 0, st, flags, pos, n, sel);
    *nsel = cnt;
    break;
  }
  return launch_status();
}

int agn_index_map(const int32_t* sel, int nsel, int n, int32_t* map, void* stream) {
  if (nsel < 0 || n < 0) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n > 0) hipLaunchKernelGGL(fill_i32_kernel, grid1(n), dim3(256), 0, st, map, n, -1);
  if (nsel > 0) hipLaunchKernelGGL(index_map_kernel, grid1(nsel), dim3(256), 0, st, sel, nsel, map);
  return launch_status();
}

int agn_subgraph_edges(const int64_t* src, const int64_t* dst, int e, const int32_t* map, int64_t* osrc,
                       int64_t* odst, int* ecount, int32_t* work, void* stream) {
  if (e < 0 || !ecount) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  *ecount = 0;
  if (e == 0) return 0;
  int32_t* flags = work;
  int32_t* pos = work + e;
  int32_t* total = work + 2 * e;
  int32_t* scr = work + 2 * e + 4;
  hipLaunchKernelGGL(subgraph_flags_kernel, grid1(e), dim3(256), 0, st, src, dst, e, map, flags);
  int rc = agn_exclusive_scan_i32(flags, pos, e, total, scr, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(subgraph_emit_kernel, grid1(e), dim3(256), 0, st, src, dst, e, map, flags, pos, osrc, odst);
  int32_t cnt = 0;
  hipError_t er = hipMemcpyAsync(&cnt, total, sizeof(cnt), hipMemcpyDeviceToHost, st);
  if (er == hipSuccess) er = hipStreamSynchronize(st);
  if (er != hipSuccess) return (int)er;
  *ecount = cnt;
  return launch_status();
}

int agn_scatter_rows(int rows, int k, int dtype, const int32_t* idx, const void* src, int src_ld, void* out,
                     int out_ld, void* stream) {
  if (rows < 0 || k < 1) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((rows + 15) / 16);
  if (dtype == AGN_F32)
    hipLaunchKernelGGL(scatter_rows_kernel<float>, g, dim3(256), 0, st, rows, k, idx, (const float*)src, src_ld,
                       (float*)out, out_ld);
  else if (dtype == AGN_BF16)
    hipLaunchKernelGGL(scatter_rows_kernel<bf16>, g, dim3(256), 0, st, rows, k, idx, (const bf16*)src, src_ld,
                       (bf16*)out, out_ld);
  else if (dtype == AGN_F16)
    hipLaunchKernelGGL(scatter_rows_kernel<f16>, g, dim3(256), 0, st, rows, k, idx, (const f16*)src, src_ld,
                       (f16*)out, out_ld);
  else if (dtype == AGN_F64)
    hipLaunchKernelGGL(scatter_rows_kernel<double>, g, dim3(256), 0, st, rows, k, idx, (const double*)src, src_ld,
                       (double*)out, out_ld);
  else
    return AGN_E_DTYPE;
  return launch_status();
}

int agn_wec_blocks(int n) { return (n + 256 / WEC_G - 1) / (256 / WEC_G); }

int agn_wec_forward(const agn_wec_args* a, void* stream) {
  if (int rc = wec_check(a)) return rc;
  if (a->n == 0) return 0;
  WEC_DISPATCH(wec_fwd_kernel, dim3(agn_wec_blocks(a->n)));
  return launch_status();
}

int agn_wec_backward(const agn_wec_args* a, void* stream) {
  if (int rc = wec_check(a)) return rc;
  if (!a->dout || !a->s_csc || !a->dtx || !a->rowptr_src || !a->perm_src || !a->dst) return AGN_E_ARG;
  if (a->w_in == nullptr && (!a->dh || !a->dpa || !a->dpb)) return AGN_E_ARG;
  if (a->n == 0) return 0;
  WEC_DISPATCH(wec_bwd_dst_kernel, dim3(agn_wec_blocks(a->n)));
  WEC_DISPATCH(wec_bwd_src_kernel, dim3(agn_wec_blocks(a->n)));
  return launch_status();
}

}  // extern "C"
