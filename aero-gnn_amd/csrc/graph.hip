// Graph-structure kernels for the MeshGraphNet hot path (gfx950): grouped (CSC/CSR) row
// reductions, row gathers, a stable LSD radix sort, scans, and the bi-stride pooling of
// models/bsms_mgn.py:217-306 (_downsample / _unpool_nodes).
//
// Determinism: no float atomics anywhere. Every reduction walks a grouped index in a fixed
// order (for fp32 that order is the torch_scatter / scatter_add_ order of the reference), so
// results are bitwise reproducible run to run.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// ------------------------------------------------------------------ grouped row reductions
// 8 contiguous elements of a row as floats (16 B of bf16, 2 x 16 B of fp32), masked at k.
template <typename T>
AGN_DEV void load8(float (&o)[8], const T* row, int f0, int k, bool vec) {
  if (vec && f0 + 7 < k) {
    if constexpr (sizeof(T) == 2) {
      const u32x4 x = *reinterpret_cast<const u32x4*>(row + f0);
#pragma unroll
      for (int i = 0; i < 4; ++i) { o[2 * i] = lo16<T>(x[i]); o[2 * i + 1] = hi16<T>(x[i]); }
    } else {
      const f32x4 x = load4(row + f0), y = load4(row + f0 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) { o[i] = x[i]; o[4 + i] = y[i]; }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (f0 + i < k) ? to_f(row[f0 + i]) : 0.f;
}
template <typename T>
AGN_DEV void store8(T* row, int f0, int k, bool vec, const float (&v)[8]) {
  if (vec && f0 + 7 < k) {
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<u32x4*>(row + f0) = u32x4{pack2t<T>(v[0], v[1]), pack2t<T>(v[2], v[3]),
                                                  pack2t<T>(v[4], v[5]), pack2t<T>(v[6], v[7])};
    } else {
      store4(row + f0, f32x4{v[0], v[1], v[2], v[3]});
      store4(row + f0 + 4, f32x4{v[4], v[5], v[6], v[7]});
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (f0 + i < k) row[f0 + i] = from_f<T>(v[i]);
}

// float64 (train.py's "double" precision, train.py:20-40): the same kernels with double
// accumulators; 16-, 32-bit storage accumulates in fp32 as above.
template <typename T> struct AccOf { using type = float; };
template <> struct AccOf<double> { using type = double; };
template <typename T> using acc_of = typename AccOf<T>::type;
template <typename T> AGN_DEV acc_of<T> ld1(T v) {
  if constexpr (std::is_same<T, double>::value) return v;
  else return to_f(v);
}
template <typename T> AGN_DEV T st1(acc_of<T> v) {
  if constexpr (std::is_same<T, double>::value) return v;
  else return from_f<T>(v);
}
template <typename T> AGN_DEV acc_of<T> rnd(acc_of<T> v) {
  if constexpr (std::is_same<T, double>::value) return v;
  else return round_t<T>(v);
}
typedef double f64x2 __attribute__((ext_vector_type(2)));
AGN_DEV void load8(double (&o)[8], const double* row, int f0, int k, bool vec) {
  if (vec && f0 + 7 < k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f64x2 x = *reinterpret_cast<const f64x2*>(row + f0 + 2 * i);
      o[2 * i] = x[0];
      o[2 * i + 1] = x[1];
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (f0 + i < k) ? row[f0 + i] : 0.0;
}
AGN_DEV void store8(double* row, int f0, int k, bool vec, const double (&v)[8]) {
  if (vec && f0 + 7 < k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f64x2*>(row + f0 + 2 * i) = f64x2{v[2 * i], v[2 * i + 1]};
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (f0 + i < k) row[f0 + i] = v[i];
}

// out[r] = sum_{j in ptr[r]..ptr[r+1]-1} src[perm ? perm[j] : j]   (/ max(count,1) if mean)
// 16 threads per row, 8 features (16 B of bf16) per thread per pass; fp32 accumulation in
// index order (two rows' loads in flight per step, summed in order).
constexpr int SEG_TPR = 16;
template <typename T>
__global__ __launch_bounds__(256) void segment_sum_kernel(int rows, int k, const int32_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ perm, const T* __restrict__ src,
                                                          int src_ld, T* __restrict__ out, int out_ld, int mean) {
  const int sub = threadIdx.x & (SEG_TPR - 1);
  const int r = blockIdx.x * (256 / SEG_TPR) + threadIdx.x / SEG_TPR;
  if (r >= rows) return;
  const int beg = ptr[r], end = ptr[r + 1];
  constexpr int A = 16 / sizeof(T);
  const bool vec = ((k % A) == 0) && ((src_ld % A) == 0) && ((out_ld % A) == 0) &&
                   ((((uintptr_t)src) | ((uintptr_t)out)) & 15) == 0;
  using A_t = acc_of<T>;
  for (int f0 = 8 * sub; f0 < k; f0 += 8 * SEG_TPR) {
    A_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int j = beg;
    for (; j + 1 < end; j += 2) {
      const int e0 = perm ? perm[j] : j, e1 = perm ? perm[j + 1] : j + 1;
      A_t x[8], y[8];
      load8(x, src + (size_t)e0 * src_ld, f0, k, vec);
      load8(y, src + (size_t)e1 * src_ld, f0, k, vec);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = (s[i] + x[i]) + y[i];
    }
    if (j < end) {
      const int e0 = perm ? perm[j] : j;
      A_t x[8];
      load8(x, src + (size_t)e0 * src_ld, f0, k, vec);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += x[i];
    }
    if (mean) {
      const A_t cnt = (A_t)max(end - beg, 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] /= cnt;
    }
    store8(out + (size_t)r * out_ld, f0, k, vec, s);
  }
}

// The same for 16-bit rows of exactly 8 * SEG_TPR features with 16-B aligned rows (the model's
// H = 128 rows): up to 4 member rows per step, their indices loaded together and then their rows,
// all in flight at once (the loop above waits for an index, then its row, every two rows); the
// sum is the same sequence of fp32 adds in index order, so the result is bitwise the same
constexpr int SEG_NQ = 4;
template <typename T>
__global__ __launch_bounds__(256) void segment_sum4_kernel(int rows, const int32_t* __restrict__ ptr,
                                                           const int32_t* __restrict__ perm, const T* __restrict__ src,
                                                           int src_ld, T* __restrict__ out, int out_ld, int mean) {
  constexpr int K = 8 * SEG_TPR;
  const int f0 = 8 * (threadIdx.x & (SEG_TPR - 1));
  const int r = blockIdx.x * (256 / SEG_TPR) + threadIdx.x / SEG_TPR;
  if (r >= rows) return;
  const int beg = ptr[r], end = ptr[r + 1];
  using A_t = acc_of<T>;
  A_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = beg; j < end; j += SEG_NQ) {
    int e[SEG_NQ];
#pragma unroll
    for (int q = 0; q < SEG_NQ; ++q) e[q] = j + q < end ? (perm ? perm[j + q] : j + q) : -1;
    A_t x[SEG_NQ][8];
#pragma unroll
    for (int q = 0; q < SEG_NQ; ++q)
      if (e[q] >= 0) load8(x[q], src + (size_t)e[q] * src_ld, f0, K, true);
#pragma unroll
    for (int q = 0; q < SEG_NQ; ++q)
      if (e[q] >= 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += x[q][i];
      }
  }
  if (mean) {
    const A_t cnt = (A_t)max(end - beg, 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] /= cnt;
  }
  store8(out + (size_t)r * out_ld, f0, K, true, s);
}

// out[r] = (base[r] + (group a of r)) + (group b of r): the concat edge MLP's node gradient in one
// pass (agn_segment_sum2). Same thread layout and in-order fp32 accumulation as segment_sum_kernel.
template <typename T>
AGN_DEV void seg_accum(acc_of<T> (&s)[8], int beg, int end, const int32_t* __restrict__ perm, const T* __restrict__ src,
                       int ld, int f0, int k, bool vec) {
  int j = beg;
  for (; j + 1 < end; j += 2) {
    const int e0 = perm ? perm[j] : j, e1 = perm ? perm[j + 1] : j + 1;
    acc_of<T> x[8], y[8];
    load8(x, src + (size_t)e0 * ld, f0, k, vec);
    load8(y, src + (size_t)e1 * ld, f0, k, vec);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = (s[i] + x[i]) + y[i];
  }
  if (j < end) {
    const int e0 = perm ? perm[j] : j;
    acc_of<T> x[8];
    load8(x, src + (size_t)e0 * ld, f0, k, vec);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += x[i];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void segment_sum2_kernel(int rows, int k, const T* base, int base_ld,
                                                           const int32_t* __restrict__ ptr_a,
                                                           const int32_t* __restrict__ perm_a,
                                                           const T* __restrict__ src_a, int lda,
                                                           const int32_t* __restrict__ ptr_b,
                                                           const int32_t* __restrict__ perm_b,
                                                           const T* __restrict__ src_b, int ldb, T* out, int out_ld) {
  const int sub = threadIdx.x & (SEG_TPR - 1);
  const int r = blockIdx.x * (256 / SEG_TPR) + threadIdx.x / SEG_TPR;
  if (r >= rows) return;
  constexpr int A = 16 / sizeof(T);
  const bool vec = ((k % A) == 0) && (!base || (base_ld % A) == 0) && ((lda % A) == 0) && ((ldb % A) == 0) &&
                   ((out_ld % A) == 0) &&
                   ((((uintptr_t)base) | ((uintptr_t)src_a) | ((uintptr_t)src_b) | ((uintptr_t)out)) & 15) == 0;
  for (int f0 = 8 * sub; f0 < k; f0 += 8 * SEG_TPR) {
    // each group summed from zero in edge order (segment_sum_kernel's sums), then
    // (base + sum_a) + sum_b: in fp32 bitwise the two-segment-sum composition it replaces
    acc_of<T> sa[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    seg_accum(sa, ptr_a[r], ptr_a[r + 1], perm_a, src_a, lda, f0, k, vec);
    seg_accum(sb, ptr_b[r], ptr_b[r + 1], perm_b, src_b, ldb, f0, k, vec);
    acc_of<T> s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (base) load8(s, base + (size_t)r * base_ld, f0, k, vec);  // read before this thread's own store (out may alias)
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = base ? (s[i] + sa[i]) + sb[i] : sa[i] + sb[i];
    store8(out + (size_t)r * out_ld, f0, k, vec, s);
  }
}

// Global max pooling (torch_geometric global_max_pool = scatter 'max' over graph ids, poolmgn.py:40):
// out[r][f] = max over the members j of group r of src[perm[j]][f] (0 for an empty group, as the
// zero-initialised scatter_reduce(include_self=False) leaves it), argmax[r][f] = the FIRST member
// row attaining it (-1 if empty) for the backward. One thread per (group, feature); members are
// walked in index order. NaN propagates (any NaN member makes the max NaN, first NaN wins).
template <typename T>
__global__ __launch_bounds__(256) void segment_max_kernel(int rows, int k, const int32_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ perm, const T* __restrict__ src,
                                                          int src_ld, T* __restrict__ out, int out_ld,
                                                          int32_t* __restrict__ argmax) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)rows * k) return;
  const int r = (int)(t / k), f = (int)(t - (long)r * k);
  const int beg = ptr[r], end = ptr[r + 1];
  acc_of<T> best = 0;
  int arg = -1;
  for (int j = beg; j < end; ++j) {
    const int e = perm ? perm[j] : j;
    const acc_of<T> v = ld1<T>(src[(size_t)e * src_ld + f]);
    if (arg < 0 || v > best || (v != v && best == best)) { best = v; arg = e; }
  }
  out[(size_t)r * out_ld + f] = st1<T>(best);
  argmax[(size_t)r * k + f] = arg;
}

// backward of segment_max: dx[argmax[r][f]][f] = gout[r][f] (dx zero-filled by the caller; the
// argmax rows of different groups are disjoint, so no two threads write one element)
template <typename T>
__global__ __launch_bounds__(256) void segment_max_bwd_kernel(int rows, int k, const int32_t* __restrict__ argmax,
                                                              const T* __restrict__ gout, int gout_ld,
                                                              T* __restrict__ dx, int dx_ld) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)rows * k) return;
  const int r = (int)(t / k), f = (int)(t - (long)r * k);
  const int a = argmax[t];
  if (a >= 0) dx[(size_t)a * dx_ld + f] = gout[(size_t)r * gout_ld + f];
}

// out[r] = src[idx[r]] / (cnt_ptr ? max(cnt_ptr[idx+1]-cnt_ptr[idx],1) : 1) + (add ? add[r] : 0)
template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(int rows, int k, const int32_t* __restrict__ idx,
                                                          const T* __restrict__ src, int src_ld,
                                                          const int32_t* __restrict__ cnt_ptr,
                                                          const T* __restrict__ add, int add_ld,
                                                          T* __restrict__ out, int out_ld) {
  const int sub = threadIdx.x & (SEG_TPR - 1);
  const int r = blockIdx.x * (256 / SEG_TPR) + threadIdx.x / SEG_TPR;
  if (r >= rows) return;
  const int s = idx ? idx[r] : r;
  constexpr int A = 16 / sizeof(T);
  const bool vec = ((k % A) == 0) && ((src_ld % A) == 0) && ((out_ld % A) == 0) && ((add_ld % A) == 0) &&
                   ((((uintptr_t)src) | ((uintptr_t)out) | ((uintptr_t)add)) & 15) == 0;
  using A_t = acc_of<T>;
  A_t div = 1;
  if (cnt_ptr) div = (A_t)max(cnt_ptr[s + 1] - cnt_ptr[s], 1);
  for (int f0 = 8 * sub; f0 < k; f0 += 8 * SEG_TPR) {
    A_t x[8];
    load8(x, src + (size_t)s * src_ld, f0, k, vec);
    if (cnt_ptr) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] /= div;
    }
    if (add) {
      // the reference rounds the gathered value to T before the add (bsms_mgn.py:199-200)
      A_t y[8];
      load8(y, add + (size_t)r * add_ld, f0, k, vec);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = rnd<T>(x[i]) + y[i];
    }
    store8(out + (size_t)r * out_ld, f0, k, vec, x);
  }
}

// The same for 16-bit rows of exactly 8 * SEG_TPR features with 16-B aligned rows (the model's
// H = 128 rows): each 16-lane group moves 4 rows, all loads issued before the first store, so a
// wave keeps 4 KB in flight instead of 1 (same arithmetic per element: bitwise the kernel above)
constexpr int GR_RPG = 4;  // rows per lane group
template <typename T>
__global__ __launch_bounds__(256) void gather_rows4_kernel(int rows, const int32_t* __restrict__ idx,
                                                           const T* __restrict__ src, int src_ld,
                                                           const int32_t* __restrict__ cnt_ptr,
                                                           const T* __restrict__ add, int add_ld,
                                                           T* __restrict__ out, int out_ld) {
  constexpr int K = 8 * SEG_TPR;
  const int f0 = 8 * (threadIdx.x & (SEG_TPR - 1));
  const int ng = gridDim.x * (256 / SEG_TPR);
  const int g = blockIdx.x * (256 / SEG_TPR) + threadIdx.x / SEG_TPR;
  using A_t = acc_of<T>;
  A_t x[GR_RPG][8], y[GR_RPG][8];
  int s[GR_RPG], cnt[GR_RPG];
#pragma unroll
  for (int i = 0; i < GR_RPG; ++i) {
    const int r = g + i * ng;
    s[i] = r < rows ? (idx ? idx[r] : r) : -1;
  }
  // the rows, the addends and the group counts all issued before the first use
#pragma unroll
  for (int i = 0; i < GR_RPG; ++i) {
    const int r = g + i * ng;
    if (s[i] >= 0) {
      load8(x[i], src + (size_t)s[i] * src_ld, f0, K, true);
      if (add) load8(y[i], add + (size_t)r * add_ld, f0, K, true);
      if (cnt_ptr) cnt[i] = cnt_ptr[s[i] + 1] - cnt_ptr[s[i]];
    }
  }
#pragma unroll
  for (int i = 0; i < GR_RPG; ++i) {
    const int r = g + i * ng;
    if (s[i] < 0) continue;
    if (cnt_ptr) {
      const A_t div = (A_t)max(cnt[i], 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[i][e] /= div;
    }
    if (add) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[i][e] = rnd<T>(x[i][e]) + y[i][e];
    }
    store8(out + (size_t)r * out_ld, f0, K, true, x[i]);
  }
}

// ------------------------------------------------------------------ stable LSD radix sort
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;

__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const uint64_t* __restrict__ keys, int n, int shift,
                                                             int nblocks, int32_t* __restrict__ counts) {
  __shared__ int32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int base = blockIdx.x * RS_TILE;
  for (int i = 0; i < RS_ITEMS; ++i) {
    const int p = base + i * RS_THREADS + threadIdx.x;
    if (p < n) atomicAdd(&h[(keys[p] >> shift) & 255], 1);
  }
  __syncthreads();
  counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of a single array by one block of 1024 threads (chunked per thread)
__global__ __launch_bounds__(1024) void scan_single_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                           int n, int32_t* __restrict__ total) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int b = t * per, e = min(n, b + per);
  int32_t s = 0;
  for (int i = b; i < e; ++i) s += in[i];
  part[t] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan over 1024 partials
  for (int off = 1; off < 1024; off <<= 1) {
    int32_t v = (t >= off) ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int32_t run = (t == 0) ? 0 : part[t - 1];
  for (int i = b; i < e; ++i) {
    const int32_t v = in[i];
    out[i] = run;
    run += v;
  }
  if (t == 1023 && total) *total = part[1023];
}

// ---- 3-phase exclusive scan (int32): block sums -> scan of block sums -> block-local scan + offset
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

__global__ __launch_bounds__(SC_THREADS) void scan_bsum_kernel(const int32_t* __restrict__ in, int n,
                                                              int32_t* __restrict__ bsum) {
  __shared__ int32_t red[SC_THREADS];
  const int base = blockIdx.x * SC_TILE;
  int32_t s = 0;
  for (int i = threadIdx.x; i < SC_TILE; i += SC_THREADS) {
    const int p = base + i;
    if (p < n) s += in[p];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = SC_THREADS / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(SC_THREADS) void scan_tile_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                              int n, const int32_t* __restrict__ boff) {
  __shared__ int32_t buf[SC_TILE];
  __shared__ int32_t part[SC_THREADS];
  const int base = blockIdx.x * SC_TILE;
  for (int i = threadIdx.x; i < SC_TILE; i += SC_THREADS) {
    const int p = base + i;
    buf[i] = p < n ? in[p] : 0;
  }
  __syncthreads();
  int32_t s = 0;
  const int t0 = threadIdx.x * SC_ITEMS;
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) s += buf[t0 + j];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < SC_THREADS; off <<= 1) {
    const int32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t run = (threadIdx.x == 0 ? 0 : part[threadIdx.x - 1]) + (boff ? boff[blockIdx.x] : 0);
#pragma unroll
  for (int j = 0; j < SC_ITEMS; ++j) {
    const int32_t v = buf[t0 + j];
    buf[t0 + j] = run;
    run += v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SC_TILE; i += SC_THREADS) {
    const int p = base + i;
    if (p < n) out[p] = buf[i];
  }
}

// exclusive scan with scratch of (nb + 1) ints, nb = ceil(n / SC_TILE); total (optional) = sum
int scan_launch(const int32_t* in, int32_t* out, int n, int32_t* total, int32_t* scratch, hipStream_t st) {
  const int nb = (n + SC_TILE - 1) / SC_TILE;
  if (nb <= 1) {
    hipLaunchKernelGGL(scan_single_kernel, dim3(1), dim3(1024), 0, st, in, out, n, total);
    return 0;
  }
  int32_t* bsum = scratch;
  int32_t* boff = scratch + nb;
  hipLaunchKernelGGL(scan_bsum_kernel, dim3(nb), dim3(SC_THREADS), 0, st, in, n, bsum);
  hipLaunchKernelGGL(scan_single_kernel, dim3(1), dim3(1024), 0, st, bsum, boff, nb, total);
  hipLaunchKernelGGL(scan_tile_kernel, dim3(nb), dim3(SC_THREADS), 0, st, in, out, n, boff);
  return 0;
}

__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const uint64_t* __restrict__ keys_in,
                                                                const int32_t* __restrict__ vals_in, int n,
                                                                int shift, int nblocks,
                                                                const int32_t* __restrict__ offsets,
                                                                uint64_t* __restrict__ keys_out,
                                                                int32_t* __restrict__ vals_out) {
  __shared__ int32_t base[256];
  __shared__ int32_t wcnt[RS_THREADS / 64][256];
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  base[t] = offsets[(size_t)t * nblocks + blockIdx.x];
  const int tile0 = blockIdx.x * RS_TILE;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // all of the thread's items are loaded up front (their latencies overlap), then ranked round
  // by round in the same order as before
  uint64_t kk[RS_ITEMS];
  int32_t vv[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const int p = tile0 + i * RS_THREADS + t;
    kk[i] = p < n ? keys_in[p] : 0ull;
    vv[i] = p < n ? vals_in[p] : 0;
  }
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    for (int wv = 0; wv < RS_THREADS / 64; ++wv) wcnt[wv][t] = 0;
    __syncthreads();
    const int p = tile0 + i * RS_THREADS + t;
    const bool ok = p < n;
    const uint64_t key = kk[i];
    const int32_t val = vv[i];
    const int d = ok ? (int)((key >> shift) & 255) : 0;
    // peers: lanes of this wave with the same digit (8 ballots)
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint64_t m = __ballot(ok && ((d >> bit) & 1));
      peers &= ((d >> bit) & 1) ? m : ~m;
    }
    const int rank = __popcll(peers & lt);
    if (ok && rank == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (ok) {
      int pos = base[d] + rank;
      for (int wv = 0; wv < w; ++wv) pos += wcnt[wv][d];
      keys_out[pos] = key;
      vals_out[pos] = val;
    }
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int wv = 0; wv < RS_THREADS / 64; ++wv) tot += wcnt[wv][t];
    base[t] += tot;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ misc index kernels
__global__ void row_ptr_kernel(const int32_t* __restrict__ keys, int n, int nrows, int32_t* __restrict__ ptr) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v > nrows) return;
  int lo = 0, hi = n;  // first i with keys[i] >= v
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  ptr[v] = lo;
}

// keys[i] = k32 ? k32[i] : k64[i] as u64 sort keys, vals[i] = i (group_by's stable-sort input)
__global__ void iota_keys_kernel(int n, const int32_t* __restrict__ k32, const int64_t* __restrict__ k64,
                                 int64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = k32 ? (int64_t)k32[i] : k64[i];
  vals[i] = i;
}

// CSC level from edge_index [2][ld] int64 and the receiver-grouping permutation: src / dst int32
// in CSC order, the permutation as int64 and its inverse (caller edge -> CSC position)
__global__ void level_index_kernel(int e, const int64_t* __restrict__ ei, int64_t ld, const int32_t* __restrict__ perm,
                                   int32_t* __restrict__ src, int32_t* __restrict__ dst, int64_t* __restrict__ perm64,
                                   int64_t* __restrict__ inv64, int32_t* __restrict__ inv32) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e) return;
  const int p = perm[i];
  src[i] = (int32_t)ei[p];
  dst[i] = (int32_t)ei[ld + p];
  perm64[i] = p;
  inv64[p] = i;
  if (inv32) inv32[p] = i;
}

__global__ void row_ptr64_kernel(const int64_t* __restrict__ keys, int n, int nrows, int32_t* __restrict__ ptr) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v > nrows) return;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  ptr[v] = lo;
}

// Monotone float -> uint32 key with the comparison torch.argsort uses: -0.0 and +0.0 compare equal
// (both map to +0's key, so the stable index rule decides between them), and every NaN, whatever
// its sign bit, sorts after +inf.
__device__ __forceinline__ uint32_t orderable(float x) {
  if (x != x) return 0xffffffffu;
  if (x == 0.f) x = 0.f;
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void pool_keys_kernel(int n, const int64_t* __restrict__ batch, const float* __restrict__ pos, int ld,
                                 uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = batch ? (uint64_t)batch[i] : 0ull;
  const uint32_t lo = pos ? orderable(pos[(size_t)i * ld]) : (uint32_t)i;
  keys[i] = (g << 32) | lo;
  vals[i] = i;
}

// f2c[sorted[p]] = coff[g] + (p - gstart[g]) / stride,  g = batch[sorted[p]]
__global__ void pool_f2c_kernel(int n, const int64_t* __restrict__ batch, const int32_t* __restrict__ sorted,
                                const int32_t* __restrict__ gstart, const int32_t* __restrict__ coff, int stride,
                                int32_t* __restrict__ f2c) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int node = sorted[p];
  const int g = batch ? (int)batch[node] : 0;
  f2c[node] = coff[g] + (p - gstart[g]) / stride;
}

// coarse node c: members = sorted[beg..end) re-ordered by fine node id (scatter_add order)
__global__ void pool_members_kernel(int nc, int ngraph, const int32_t* __restrict__ sorted,
                                    const int32_t* __restrict__ gstart, const int32_t* __restrict__ coff, int stride,
                                    int32_t* __restrict__ c2f, int32_t* __restrict__ c2f_ptr,
                                    int64_t* __restrict__ cbatch, int n) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > nc) return;
  if (c == nc) { c2f_ptr[nc] = n; return; }
  int lo = 0, hi = ngraph;  // last g with coff[g] <= c
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (coff[mid] <= c) lo = mid;
    else hi = mid;
  }
  const int g = lo;
  const int beg = gstart[g] + stride * (c - coff[g]);
  const int end = min(beg + stride, gstart[g + 1]);
  c2f_ptr[c] = beg;
  cbatch[c] = g;
  for (int i = beg; i < end; ++i) c2f[i] = sorted[i];
  for (int i = beg + 1; i < end; ++i) {  // insertion sort (stride is small)
    const int v = c2f[i];
    int j = i - 1;
    while (j >= beg && c2f[j] > v) { c2f[j + 1] = c2f[j]; --j; }
    c2f[j + 1] = v;
  }
}

// number of fine edges whose receiver pools into coarse node c
__global__ void pool_cand_count_kernel(int nc, const int32_t* __restrict__ c2f, const int32_t* __restrict__ c2f_ptr,
                                       const int32_t* __restrict__ rowptr, int32_t* __restrict__ cnt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int s = 0;
  for (int i = c2f_ptr[c]; i < c2f_ptr[c + 1]; ++i) {
    const int m = c2f[i];
    s += rowptr[m + 1] - rowptr[m];
  }
  cnt[c] = s;
}

// flattened candidate list of coarse node c (member order, then CSC order)
__global__ void pool_cand_list_kernel(int nc, const int32_t* __restrict__ c2f, const int32_t* __restrict__ c2f_ptr,
                                      const int32_t* __restrict__ rowptr, const int32_t* __restrict__ cand_ptr,
                                      int32_t* __restrict__ cand) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int o = cand_ptr[c];
  for (int i = c2f_ptr[c]; i < c2f_ptr[c + 1]; ++i) {
    const int m = c2f[i];
    for (int e = rowptr[m]; e < rowptr[m + 1]; ++e) cand[o++] = e;
  }
}

// One wave per coarse node: rank-sort its candidate fine edges by (f2c[src], refkey)
// (refkey = the fine edge's position in the reference's own edge order at this level).
__global__ __launch_bounds__(256) void pool_cand_sort_kernel(int nc, const int32_t* __restrict__ cand_ptr,
                                                             const int32_t* __restrict__ cand,
                                                             const int32_t* __restrict__ src,
                                                             const int64_t* __restrict__ refkey,
                                                             const int32_t* __restrict__ f2c,
                                                             int32_t* __restrict__ sorted) {
  // the wave's candidate keys are staged in LDS once (the O(d^2) rank loop then reads LDS
  // broadcasts instead of three dependent global loads per comparison); larger lists fall back
  constexpr int CAP = 256;
  __shared__ int sk[4][CAP];
  __shared__ int64_t sr[4][CAP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 4 + w;
  if (c >= nc) return;
  const int b = cand_ptr[c], d = cand_ptr[c + 1] - b;
  if (d <= CAP) {
    for (int i = lane; i < d; i += 64) {
      const int ei = cand[b + i];
      sk[w][i] = f2c[src[ei]];
      sr[w][i] = refkey[ei];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < d; i += 64) {
      const int ki = sk[w][i];
      const int64_t ri = sr[w][i];
      int rank = 0;
      for (int j = 0; j < d; ++j) {
        const int kj = sk[w][j];
        rank += (kj < ki) || (kj == ki && sr[w][j] < ri);
      }
      sorted[b + rank] = cand[b + i];
    }
    return;
  }
  for (int i = lane; i < d; i += 64) {
    const int ei = cand[b + i];
    const int ki = f2c[src[ei]];
    const int64_t ri = refkey[ei];
    int rank = 0;
    for (int j = 0; j < d; ++j) {
      const int ej = cand[b + j];
      const int kj = f2c[src[ej]];
      rank += (kj < ki) || (kj == ki && refkey[ej] < ri);
    }
    sorted[b + rank] = ei;
  }
}

// distinct coarse senders per coarse node (one wave per node, as pool_emit_kernel)
__global__ void pool_uniq_kernel(int nc, const int32_t* __restrict__ cand_ptr, const int32_t* __restrict__ sorted,
                                 const int32_t* __restrict__ src, const int32_t* __restrict__ f2c,
                                 int32_t* __restrict__ uniq) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nc) return;
  const int b = cand_ptr[c], end = cand_ptr[c + 1];
  int u = 0, prev = -1;
  for (int p0 = b; p0 < end; p0 += 64) {
    const int p = p0 + lane;
    const bool in = p < end;
    const int sv = in ? f2c[src[sorted[p]]] : -1;
    int before = __shfl_up(sv, 1, 64);
    if (lane == 0) before = prev;
    u += __popcll(__ballot(in && sv != before));
    prev = __shfl(sv, min(63, end - 1 - p0), 64);
  }
  if (lane == 0) uniq[c] = u;
}

// One wave per coarse node c: its sorted candidates are processed 64 at a time; a candidate
// opens a new coarse edge where its coarse sender differs from its predecessor's, and the coarse
// edge index is crowptr[c] - 1 + the running count of openings (wave ballot + popcount): the same
// output as the sequential walk, without its chain of dependent loads per candidate.
__global__ void pool_emit_kernel(int nc, const int32_t* __restrict__ cand_ptr, const int32_t* __restrict__ sorted,
                                 const int32_t* __restrict__ src, const int32_t* __restrict__ f2c,
                                 const int32_t* __restrict__ crowptr, int32_t* __restrict__ csrc,
                                 int32_t* __restrict__ cdst, int32_t* __restrict__ cmem_ptr,
                                 int32_t* __restrict__ inv, int64_t* __restrict__ crefkey, int e_fine) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) cmem_ptr[crowptr[nc]] = e_fine;
  if (c >= nc) return;
  const int b = cand_ptr[c], end = cand_ptr[c + 1];
  int base = crowptr[c] - 1, prev = -1;  // index of the last opened coarse edge; its sender
  for (int p0 = b; p0 < end; p0 += 64) {
    const int p = p0 + lane;
    const bool in = p < end;
    const int e = in ? sorted[p] : 0;
    const int sv = in ? f2c[src[e]] : -1;
    int before = __shfl_up(sv, 1, 64);
    if (lane == 0) before = prev;
    const bool open = in && sv != before;
    const uint64_t m = __ballot(open);
    const int k = base + __popcll(m & ((2ull << lane) - 1ull));  // lane 63: all bits
    if (open) {
      csrc[k] = sv;
      cdst[k] = c;
      cmem_ptr[k] = p;
      crefkey[k] = (int64_t)sv * nc + c;
    }
    if (in) inv[e] = k;
    base += __popcll(m);
    prev = __shfl(sv, min(63, end - 1 - p0), 64);
  }
}

template <typename T>
int seg_sum_t(int rows, int k, const int32_t* ptr, const int32_t* perm, const void* src, int src_ld, void* out,
              int out_ld, int mean, hipStream_t st) {
  constexpr int A = 16 / sizeof(T);
  if (sizeof(T) == 2 && k == 8 * SEG_TPR && src_ld % A == 0 && out_ld % A == 0 &&
      ((((uintptr_t)src) | ((uintptr_t)out)) & 15) == 0) {
    hipLaunchKernelGGL(segment_sum4_kernel<T>, dim3((rows + 15) / 16), dim3(256), 0, st, rows, ptr, perm,
                       (const T*)src, src_ld, (T*)out, out_ld, mean);
    return launch_status();
  }
  hipLaunchKernelGGL(segment_sum_kernel<T>, dim3((rows + 15) / 16), dim3(256), 0, st, rows, k, ptr, perm,
                     (const T*)src, src_ld, (T*)out, out_ld, mean);
  return launch_status();
}

template <typename T>
int seg_sum2_t(int rows, int k, const void* base, int base_ld, const int32_t* ptr_a, const int32_t* perm_a,
               const void* src_a, int lda, const int32_t* ptr_b, const int32_t* perm_b, const void* src_b, int ldb,
               void* out, int out_ld, hipStream_t st) {
  hipLaunchKernelGGL(segment_sum2_kernel<T>, dim3((rows + 15) / 16), dim3(256), 0, st, rows, k, (const T*)base,
                     base_ld, ptr_a, perm_a, (const T*)src_a, lda, ptr_b, perm_b, (const T*)src_b, ldb, (T*)out,
                     out_ld);
  return launch_status();
}

template <typename T>
int gather_t(int rows, int k, const int32_t* idx, const void* src, int src_ld, const int32_t* cnt_ptr,
             const void* add, int add_ld, void* out, int out_ld, hipStream_t st) {
  constexpr int A = 16 / sizeof(T);
  if (sizeof(T) == 2 && k == 8 * SEG_TPR && src_ld % A == 0 && out_ld % A == 0 && (!add || add_ld % A == 0) &&
      ((((uintptr_t)src) | ((uintptr_t)out) | ((uintptr_t)add)) & 15) == 0) {
    const int groups = (rows + GR_RPG - 1) / GR_RPG;
    hipLaunchKernelGGL(gather_rows4_kernel<T>, dim3((groups + 15) / 16), dim3(256), 0, st, rows, idx, (const T*)src,
                       src_ld, cnt_ptr, (const T*)add, add_ld, (T*)out, out_ld);
    return launch_status();
  }
  hipLaunchKernelGGL(gather_rows_kernel<T>, dim3((rows + 15) / 16), dim3(256), 0, st, rows, k, idx, (const T*)src,
                     src_ld, cnt_ptr, (const T*)add, add_ld, (T*)out, out_ld);
  return launch_status();
}

inline dim3 g1(int n, int b = 256) { return dim3((n + b - 1) / b); }

}  // namespace

extern "C" {

int agn_segment_sum(int rows, int k, int dtype, const int32_t* ptr, const int32_t* perm, const void* src, int src_ld,
                    void* out, int out_ld, int mean, void* stream) {
  if (rows < 0 || k < 1) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == AGN_F32) return seg_sum_t<float>(rows, k, ptr, perm, src, src_ld, out, out_ld, mean, st);
  if (dtype == AGN_BF16) return seg_sum_t<bf16>(rows, k, ptr, perm, src, src_ld, out, out_ld, mean, st);
  if (dtype == AGN_F16) return seg_sum_t<f16>(rows, k, ptr, perm, src, src_ld, out, out_ld, mean, st);
  if (dtype == AGN_F64) return seg_sum_t<double>(rows, k, ptr, perm, src, src_ld, out, out_ld, mean, st);
  return AGN_E_DTYPE;
}

int agn_segment_sum2(int rows, int k, int dtype, const void* base, int base_ld, const int32_t* ptr_a,
                     const int32_t* perm_a, const void* src_a, int lda, const int32_t* ptr_b, const int32_t* perm_b,
                     const void* src_b, int ldb, void* out, int out_ld, void* stream) {
  if (rows < 0 || k < 1) return AGN_E_ARG;
  if (rows == 0) return 0;
  if (!ptr_a || !src_a || !ptr_b || !src_b || !out) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
#define AGN_SS2(T) seg_sum2_t<T>(rows, k, base, base_ld, ptr_a, perm_a, src_a, lda, ptr_b, perm_b, src_b, ldb, out, out_ld, st)
  if (dtype == AGN_F32) return AGN_SS2(float);
  if (dtype == AGN_BF16) return AGN_SS2(bf16);
  if (dtype == AGN_F16) return AGN_SS2(f16);
  if (dtype == AGN_F64) return AGN_SS2(double);
#undef AGN_SS2
  return AGN_E_DTYPE;
}

int agn_segment_max(int rows, int k, int dtype, const int32_t* ptr, const int32_t* perm, const void* src, int src_ld,
                    void* out, int out_ld, int32_t* argmax, void* stream) {
  if (rows < 0 || k < 1 || !argmax) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)rows * k;
  const dim3 g((unsigned)((n + 255) / 256));
  if (dtype == AGN_F32)
    hipLaunchKernelGGL(segment_max_kernel<float>, g, dim3(256), 0, st, rows, k, ptr, perm, (const float*)src, src_ld,
                       (float*)out, out_ld, argmax);
  else if (dtype == AGN_BF16)
    hipLaunchKernelGGL(segment_max_kernel<bf16>, g, dim3(256), 0, st, rows, k, ptr, perm, (const bf16*)src, src_ld,
                       (bf16*)out, out_ld, argmax);
  else if (dtype == AGN_F16)
    hipLaunchKernelGGL(segment_max_kernel<f16>, g, dim3(256), 0, st, rows, k, ptr, perm, (const f16*)src, src_ld,
                       (f16*)out, out_ld, argmax);
  else if (dtype == AGN_F64)
    hipLaunchKernelGGL(segment_max_kernel<double>, g, dim3(256), 0, st, rows, k, ptr, perm, (const double*)src, src_ld,
                       (double*)out, out_ld, argmax);
  else
    return AGN_E_DTYPE;
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int agn_segment_max_backward(int rows, int k, int dtype, const int32_t* argmax, const void* gout, int gout_ld,
                             void* dx, int dx_ld, void* stream) {
  if (rows < 0 || k < 1 || !argmax) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)rows * k;
  const dim3 g((unsigned)((n + 255) / 256));
  if (dtype == AGN_F32)
    hipLaunchKernelGGL(segment_max_bwd_kernel<float>, g, dim3(256), 0, st, rows, k, argmax, (const float*)gout, gout_ld,
                       (float*)dx, dx_ld);
  else if (dtype == AGN_BF16)
    hipLaunchKernelGGL(segment_max_bwd_kernel<bf16>, g, dim3(256), 0, st, rows, k, argmax, (const bf16*)gout, gout_ld,
                       (bf16*)dx, dx_ld);
  else if (dtype == AGN_F16)
    hipLaunchKernelGGL(segment_max_bwd_kernel<f16>, g, dim3(256), 0, st, rows, k, argmax, (const f16*)gout, gout_ld,
                       (f16*)dx, dx_ld);
  else if (dtype == AGN_F64)
    hipLaunchKernelGGL(segment_max_bwd_kernel<double>, g, dim3(256), 0, st, rows, k, argmax, (const double*)gout,
                       gout_ld, (double*)dx, dx_ld);
  else
    return AGN_E_DTYPE;
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int agn_gather_rows(int rows, int k, int dtype, const int32_t* idx, const void* src, int src_ld,
                    const int32_t* cnt_ptr, const void* add, int add_ld, void* out, int out_ld, void* stream) {
  if (rows < 0 || k < 1) return AGN_E_ARG;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == AGN_F32) return gather_t<float>(rows, k, idx, src, src_ld, cnt_ptr, add, add_ld, out, out_ld, st);
  if (dtype == AGN_BF16) return gather_t<bf16>(rows, k, idx, src, src_ld, cnt_ptr, add, add_ld, out, out_ld, st);
  if (dtype == AGN_F16) return gather_t<f16>(rows, k, idx, src, src_ld, cnt_ptr, add, add_ld, out, out_ld, st);
  if (dtype == AGN_F64) return gather_t<double>(rows, k, idx, src, src_ld, cnt_ptr, add, add_ld, out, out_ld, st);
  return AGN_E_DTYPE;
}

size_t agn_radix_sort_temp_bytes(int n) {
  const int nb = (n + RS_TILE - 1) / RS_TILE;
  const int m = 256 * (nb > 0 ? nb : 1);
  return (size_t)(2 * m + 2 * ((m + SC_TILE - 1) / SC_TILE) + 2) * sizeof(int32_t) + 256;
}

int agn_radix_sort_u64(uint64_t* keys, int32_t* vals, int n, int bits, uint64_t* keys_tmp, int32_t* vals_tmp,
                       void* scratch, void* stream) {
  if (n < 0 || bits < 0 || bits > 64) return AGN_E_ARG;
  if (n <= 1 || bits == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (n + RS_TILE - 1) / RS_TILE;
  int32_t* counts = reinterpret_cast<int32_t*>(scratch);
  int32_t* offs = counts + 256 * nb;
  int32_t* sscr = offs + 256 * nb;
  uint64_t *ki = keys, *ko = keys_tmp;
  int32_t *vi = vals, *vo = vals_tmp;
  const int passes = (bits + 7) / 8;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    hipLaunchKernelGGL(rs_hist_kernel, dim3(nb), dim3(RS_THREADS), 0, st, ki, n, shift, nb, counts);
    scan_launch(counts, offs, 256 * nb, (int32_t*)nullptr, sscr, st);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, n, shift, nb, offs, ko, vo);
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
  if (ki != keys) {
    hipError_t e1 = hipMemcpyAsync(keys, ki, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToDevice, st);
    hipError_t e2 = hipMemcpyAsync(vals, vi, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToDevice, st);
    if (e1 != hipSuccess) return (int)e1;
    if (e2 != hipSuccess) return (int)e2;
  }
  return launch_status();
}

size_t agn_scan_temp_bytes(int n) {
  return (size_t)(2 * ((n + SC_TILE - 1) / SC_TILE) + 2) * sizeof(int32_t);
}

int agn_exclusive_scan_i32(const int32_t* in, int32_t* out, int n, int32_t* total, int32_t* scratch, void* stream) {
  if (n < 0) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (total) {
      hipError_t e = hipMemsetAsync(total, 0, sizeof(int32_t), st);
      if (e != hipSuccess) return (int)e;
    }
    return launch_status();
  }
  scan_launch(in, out, n, total, scratch, st);
  return launch_status();
}

int agn_row_ptr(const int32_t* sorted_keys, int n, int nrows, int32_t* ptr, void* stream) {
  if (n < 0 || nrows < 0) return AGN_E_ARG;
  hipLaunchKernelGGL(row_ptr_kernel, g1(nrows + 1), dim3(256), 0, (hipStream_t)stream, sorted_keys, n, nrows, ptr);
  return launch_status();
}

int agn_iota_keys(int n, const int32_t* keys32, const int64_t* keys64, int64_t* keys, int32_t* vals, void* stream) {
  if (n < 0) return AGN_E_ARG;
  if (n == 0) return 0;
  if ((!keys32 && !keys64) || !keys || !vals) return AGN_E_ARG;
  hipLaunchKernelGGL(iota_keys_kernel, g1(n), dim3(256), 0, (hipStream_t)stream, n, keys32, keys64, keys, vals);
  return launch_status();
}

int agn_level_index(int e, const int64_t* edge_index, int64_t ld, const int32_t* perm, int32_t* src, int32_t* dst,
                    int64_t* perm64, int64_t* inv64, int32_t* inv32, void* stream) {
  if (e < 0) return AGN_E_ARG;
  if (e == 0) return 0;
  if (ld < e || !edge_index || !perm || !src || !dst || !perm64 || !inv64) return AGN_E_ARG;
  hipLaunchKernelGGL(level_index_kernel, g1(e), dim3(256), 0, (hipStream_t)stream, e, edge_index, ld, perm, src, dst,
                     perm64, inv64, inv32);
  return launch_status();
}

int agn_row_ptr_i64(const int64_t* sorted_keys, int n, int nrows, int32_t* ptr, void* stream) {
  if (n < 0 || nrows < 0) return AGN_E_ARG;
  hipLaunchKernelGGL(row_ptr64_kernel, g1(nrows + 1), dim3(256), 0, (hipStream_t)stream, sorted_keys, n, nrows, ptr);
  return launch_status();
}

int agn_pool_sort_keys(int n, const int64_t* batch, const float* pos, int pos_ld, uint64_t* keys, int32_t* vals,
                       void* stream) {
  if (n < 0) return AGN_E_ARG;
  if (n == 0) return 0;
  hipLaunchKernelGGL(pool_keys_kernel, g1(n), dim3(256), 0, (hipStream_t)stream, n, batch, pos, pos_ld, keys, vals);
  return launch_status();
}

int agn_pool_assign(int n, int nc, int ngraph, const int64_t* batch, const int32_t* sorted, const int32_t* gstart,
                    const int32_t* coff, int stride, int32_t* f2c, int32_t* c2f, int32_t* c2f_ptr, int64_t* cbatch,
                    void* stream) {
  if (n < 0 || nc < 0 || stride < 1) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n > 0) hipLaunchKernelGGL(pool_f2c_kernel, g1(n), dim3(256), 0, st, n, batch, sorted, gstart, coff, stride, f2c);
  hipLaunchKernelGGL(pool_members_kernel, g1(nc + 1), dim3(256), 0, st, nc, ngraph, sorted, gstart, coff, stride, c2f,
                     c2f_ptr, cbatch, n);
  return launch_status();
}

int agn_pool_edge_candidates(int nc, const int32_t* c2f, const int32_t* c2f_ptr, const int32_t* rowptr,
                             int32_t* cand_cnt, void* stream) {
  if (nc < 0) return AGN_E_ARG;
  if (nc == 0) return 0;
  hipLaunchKernelGGL(pool_cand_count_kernel, g1(nc), dim3(256), 0, (hipStream_t)stream, nc, c2f, c2f_ptr, rowptr,
                     cand_cnt);
  return launch_status();
}

int agn_pool_edge_sort(int nc, const int32_t* c2f, const int32_t* c2f_ptr, const int32_t* rowptr, const int32_t* src,
                       const int64_t* refkey, const int32_t* f2c, const int32_t* cand_ptr, int32_t* cand_tmp,
                       int32_t* cand_sorted, int32_t* uniq, void* stream) {
  if (nc < 0) return AGN_E_ARG;
  if (nc == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(pool_cand_list_kernel, g1(nc), dim3(256), 0, st, nc, c2f, c2f_ptr, rowptr, cand_ptr, cand_tmp);
  hipLaunchKernelGGL(pool_cand_sort_kernel, dim3((nc + 3) / 4), dim3(256), 0, st, nc, cand_ptr, cand_tmp, src, refkey,
                     f2c, cand_sorted);
  hipLaunchKernelGGL(pool_uniq_kernel, dim3((nc + 3) / 4), dim3(256), 0, st, nc, cand_ptr, cand_sorted, src, f2c, uniq);
  return launch_status();
}

int agn_pool_edge_emit(int nc, const int32_t* cand_ptr, const int32_t* cand_sorted, const int32_t* src,
                       const int32_t* f2c, const int32_t* crowptr, int32_t* csrc, int32_t* cdst, int32_t* cmem_ptr,
                       int32_t* inv, int64_t* crefkey, int e_fine, void* stream) {
  if (nc < 0) return AGN_E_ARG;
  hipLaunchKernelGGL(pool_emit_kernel, dim3(nc > 0 ? (nc + 3) / 4 : 1), dim3(256), 0, (hipStream_t)stream, nc,
                     cand_ptr, cand_sorted, src, f2c, crowptr, csrc, cdst, cmem_ptr, inv, crefkey, e_fine);
  return launch_status();
}

}  // extern "C"
