// Weight gradients dW = G^T X (and bias grads db = colsum G) for every Linear of the MLP
// chains: G = dL/d(pre-activation) [rows x M], X = layer input [rows x K], rows = edges or
// nodes (up to tens of millions), M, K <= 256. This is the K-reduction-over-rows half of the
// backward of models/mlp.py / mgnLayer.py Linears (autograd's mm(grad^T, input)).
//
// Split-K over rows: each workgroup owns a contiguous row chunk and one 128x128 output block,
// stages 64-row tiles of G and X in LDS (coalesced 16-B loads), and accumulates on MFMA in
// fp32: bf16 uses v_mfma_f32_32x32x16_bf16 whose A/B operands need 8 consecutive ROWS of one
// column -> ds_read_b64_tr_b16 transposed LDS reads; fp32 uses v_mfma_f32_32x32x2_f32 with
// plain ds_read_b32. Per-chunk partials go to a slab and a second kernel sums the slabs in
// fixed order: deterministic, no atomics.
#include "common.hpp"
#include "aerognn.h"

#include <type_traits>

using namespace agn;

namespace {

#ifndef AGN_DW_ROWS
#define AGN_DW_ROWS 64
#endif
constexpr int DW_ROWS = AGN_DW_ROWS;  // rows per LDS stage
constexpr int DW_BLK = 128;   // output block edge
constexpr int DW_THREADS = 256;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct DwTile;
// LDS row stride in elements: bf16 136 (272 B, breaks the 4-row bank aliasing of tr reads),
// f32 132 (528 B).
template <> struct DwTile<bf16> { static constexpr int LD = 136; };
template <> struct DwTile<f16> { static constexpr int LD = 136; };
template <> struct DwTile<float> { static constexpr int LD = 132; };

// One 64-row x 128-col stage of a row-major [rows][ld] matrix, moved global -> registers ->
// LDS so the next stage's loads are in flight while the current stage is on MFMA. Each thread
// owns NCH 16-B chunks; rows >= rows / cols >= cols read as zero.
template <typename T>
struct StageRegs {
  static constexpr int PER16 = 16 / sizeof(T);                  // elements per 16-B chunk
  static constexpr int CHUNKS = DW_BLK / PER16;                 // chunks per row
  static constexpr int NCH = DW_ROWS * CHUNKS / DW_THREADS;     // chunks per thread
  uint4 v[NCH];

  // AGN_TILED operand (aerognn.h): a 64-row stage of a 128-wide tiled matrix is 64*CHUNKS
  // consecutive 16-B units (r0 is a multiple of 64), so the loads are contiguous.
  static AGN_DEV void tiled_pos(int u, int& row, int& i, int& hh) {
    const int t = u / (CHUNKS * 32), rem = u - t * (CHUNKS * 32);
    i = rem >> 6;
    row = t * 32 + (rem & 31);
    hh = (rem >> 5) & 1;
  }
  // idx (row-major operands only): logical row r is g's row idx[r] (a gathered operand)
  AGN_DEV void load(const T* __restrict__ g, int ld, int rows, int cols, int r0, int c0, int tiled,
                    const int32_t* __restrict__ idx = nullptr) {
    if (tiled) {
      const uint4* gu = reinterpret_cast<const uint4*>(g) + (size_t)(r0 >> 5) * (CHUNKS / 2) * 64;
      if (r0 + DW_ROWS <= rows) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) v[j] = gu[threadIdx.x + j * DW_THREADS];
      } else {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int u = threadIdx.x + j * DW_THREADS;
          int row, i, hh;
          tiled_pos(u, row, i, hh);
          v[j] = (r0 + row < rows) ? gu[u] : uint4{0u, 0u, 0u, 0u};
        }
      }
      return;
    }
    const bool fast = ((ld % PER16) == 0) && ((c0 % PER16) == 0) && (cols - c0 >= DW_BLK) && (r0 + DW_ROWS <= rows);
    if (fast) {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int i = threadIdx.x + j * DW_THREADS;
        const int r = i / CHUNKS, ch = i - r * CHUNKS;
        const size_t gr = idx ? (size_t)idx[r0 + r] : (size_t)(r0 + r);
        v[j] = *reinterpret_cast<const uint4*>(g + gr * ld + c0 + ch * PER16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int i = threadIdx.x + j * DW_THREADS;
        const int r = i / CHUNKS, ch = i - r * CHUNKS;
        const int gr = r0 + r, gc0 = c0 + ch * PER16;
        v[j] = uint4{0u, 0u, 0u, 0u};
        // chunks past the last column stay zero without a load (a narrow X, e.g. K = 4, has one
        // live chunk per row); a live chunk takes the widest aligned loads it can
        if (gr < rows && gc0 < cols) {
          const size_t sr = idx ? (size_t)idx[gr] : (size_t)gr;
          const T* p = g + sr * ld + gc0;
          const int nv = min(PER16, cols - gc0);
          const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
          if (nv == PER16 && (pa & 15) == 0) {
            v[j] = *reinterpret_cast<const uint4*>(p);
          } else if (sizeof(T) == 2 && nv >= 4 && (pa & 7) == 0) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 lo = *reinterpret_cast<const u32x2*>(p);
            T e4[4] = {from_f<T>(0.f), from_f<T>(0.f), from_f<T>(0.f), from_f<T>(0.f)};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (4 + e < nv) e4[e] = p[4 + e];
            const u32x2 hi = *reinterpret_cast<const u32x2*>(e4);
            v[j] = __builtin_bit_cast(uint4, u32x4{lo[0], lo[1], hi[0], hi[1]});
          } else {
            T e8[PER16];
#pragma unroll
            for (int e = 0; e < PER16; ++e) e8[e] = e < nv ? p[e] : from_f<T>(0.f);
            v[j] = *reinterpret_cast<const uint4*>(e8);
          }
        }
      }
    }
  }
  AGN_DEV void store(T* lds, int tiled) const {
    constexpr int LD = DwTile<T>::LD;
    if (tiled) {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        int row, i, hh;
        tiled_pos(threadIdx.x + j * DW_THREADS, row, i, hh);
        if constexpr (sizeof(T) == 2) {  // features 16i+4hh+{0..3} | 16i+8+4hh+{0..3}
          const u32x4 x = __builtin_bit_cast(u32x4, v[j]);
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2*>(lds + row * LD + 16 * i + 4 * hh) = u32x2{x[0], x[1]};
          *reinterpret_cast<u32x2*>(lds + row * LD + 16 * i + 8 + 4 * hh) = u32x2{x[2], x[3]};
        } else {  // features 8i+4hh+{0..3}
          *reinterpret_cast<uint4*>(lds + row * LD + 8 * i + 4 * hh) = v[j];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int i = threadIdx.x + j * DW_THREADS;
      const int r = i / CHUNKS, ch = i - r * CHUNKS;
      *reinterpret_cast<uint4*>(lds + r * LD + ch * PER16) = v[j];
    }
  }
};

// 8 consecutive rows (k) of one column: two ds_read_b64_tr_b16 (rows kb..kb+3, kb+4..kb+7)
AGN_DEV bf16x8 tr_frag(const bf16* lds, int kb, int col_base, int lane) {
  constexpr int LD = DwTile<bf16>::LD;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const bf16* a0 = lds + (kb + q) * LD + col_base + 4 * p;
  const bf16* a1 = a0 + 4 * LD;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  bf16x8 r;
  const bf16x4 l4 = *reinterpret_cast<const bf16x4*>(&lo);
  const bf16x4 h4 = *reinterpret_cast<const bf16x4*>(&hi);
  r[0] = l4[0]; r[1] = l4[1]; r[2] = l4[2]; r[3] = l4[3];
  r[4] = h4[0]; r[5] = h4[1]; r[6] = h4[2]; r[7] = h4[3];
  return r;
}

// grid: x = row chunk (split), y = M block * nKb + K block, z = desc
// XG: some desc has a gathered X (xidx); a separate instantiation keeps the plain path free of it
template <typename T, bool XG>
__global__ __launch_bounds__(DW_THREADS) void wgrad_kernel(const agn_wgrad_batch b, int nsplit) {
  constexpr int LD = DwTile<T>::LD;
  __shared__ __attribute__((aligned(16))) T sg[DW_ROWS * LD];
  __shared__ __attribute__((aligned(16))) T sx[DW_ROWS * LD];
  const agn_wgrad_desc& d = b.d[blockIdx.z];
  const int nKb = (d.k + DW_BLK - 1) / DW_BLK;
  const int nMb = (d.m + DW_BLK - 1) / DW_BLK;
  if ((int)blockIdx.y >= nMb * nKb) return;
  const int mb = blockIdx.y / nKb, kb = blockIdx.y % nKb;
  const int m0 = mb * DW_BLK, k0 = kb * DW_BLK;
  const int split = blockIdx.x;
  const int per = ((d.rows + nsplit - 1) / nsplit + DW_ROWS - 1) / DW_ROWS * DW_ROWS;
  const int rbeg = split * per, rend = min(d.rows, rbeg + per);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wk = (w & 1) * 64;  // this wave's 64x64 sub-block
  const T* G = reinterpret_cast<const T*>(d.g);
  const T* X = reinterpret_cast<const T*>(d.x);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  // bias colsum partial: thread t owns column m0 + (t & 127) over rows 16q..16q+15 of each stage
  // (q = t >> 7 picks the even / odd 16-row groups), so all four waves share the walk; the two
  // halves are added in a fixed order at the end
  float bsum = 0.f;
  __shared__ float bhalf[DW_BLK];
  StageRegs<T> rg, rx;
  if (rbeg < rend) {
    rg.load(G, d.ldg, rend, d.m, rbeg, m0, d.g_tiled);
    rx.load(X, d.ldx, rend, d.k, rbeg, k0, d.x_tiled, XG ? d.xidx : nullptr);
  }
  for (int r0 = rbeg; r0 < rend; r0 += DW_ROWS) {
    __syncthreads();
    rg.store(sg, d.g_tiled);
    rx.store(sx, d.x_tiled);
    __syncthreads();
    if (r0 + DW_ROWS < rend) {  // next stage in flight during this stage's MFMAs
      rg.load(G, d.ldg, rend, d.m, r0 + DW_ROWS, m0, d.g_tiled);
      rx.load(X, d.ldx, rend, d.k, r0 + DW_ROWS, k0, d.x_tiled, XG ? d.xidx : nullptr);
    }
    if (d.db_partial && kb == 0) {
      const int col = threadIdx.x & (DW_BLK - 1), q = threadIdx.x >> 7;
#pragma unroll
      for (int gq = 0; gq < DW_ROWS / 32; ++gq)
#pragma unroll 8
        for (int r = 0; r < 16; ++r) bsum += to_f(sg[(32 * gq + 16 * q + r) * LD + col]);
    }
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int ks = 0; ks < DW_ROWS; ks += 16) {
        const int kbase = ks + 8 * (lane >> 5);
        bf16x8 a[2], bb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = tr_frag(reinterpret_cast<const bf16*>(sg), kbase, wm + 32 * i + 16 * ((lane >> 4) & 1), lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) bb[j] = tr_frag(reinterpret_cast<const bf16*>(sx), kbase, wk + 32 * j + 16 * ((lane >> 4) & 1), lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if constexpr (std::is_same<T, f16>::value)  // same fragments, fp16 products
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a[i]),
                                                                 __builtin_bit_cast(f16x8, bb[j]), acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
          }
      }
    } else {
      const float* fg = reinterpret_cast<const float*>(sg);
      const float* fx = reinterpret_cast<const float*>(sx);
#pragma unroll 4
      for (int ks = 0; ks < DW_ROWS; ks += 2) {
        const int r = ks + (lane >> 5), cidx = lane & 31;
        float a[2], bb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = fg[r * LD + wm + 32 * i + cidx];
#pragma unroll
        for (int j = 0; j < 2; ++j) bb[j] = fx[r * LD + wk + 32 * j + cidx];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // partial slab [split][mpad][kpad] with mpad = nMb*128, kpad = nKb*128
  const int kpad = nKb * DW_BLK;
  float* P = d.dw_partial + (size_t)split * (nMb * DW_BLK) * kpad;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = k0 + wk + 32 * j + (lane & 31);
        P[(size_t)m * kpad + k] = acc[i][j][r];
      }
  if (d.db_partial && kb == 0) {
    __syncthreads();
    if (threadIdx.x >= DW_BLK) bhalf[threadIdx.x - DW_BLK] = bsum;
    __syncthreads();
    if (threadIdx.x < DW_BLK) d.db_partial[(size_t)split * (nMb * DW_BLK) + m0 + threadIdx.x] = bsum + bhalf[threadIdx.x];
  }
}

// out[m][k] = sum_s partial[s][m][k] (m < M, k < K). A block owns RED_Q column quads (4 RED_Q
// floats of the [mpad][kpad] slab); its RED_G thread groups each sum the splits s = g,
// g + RED_G, ... and the group partials are combined in LDS in group order: a fixed
// summation order (deterministic), with RED_G x RED_Q 16-B loads in flight per block. RED_Q = 16
// spreads a 128 x 128 slab over 256 blocks (64 quads per block left 3/4 of the CUs idle: the
// reduce of a 768-split slab ran at ~1.5 TB/s)
constexpr int RED_G = 8;
constexpr int RED_Q = 16;
__global__ __launch_bounds__(RED_Q * RED_G) void wgrad_reduce_kernel(const agn_wgrad_batch b) {
  __shared__ f32x4 part[RED_G][RED_Q];
  __shared__ float bpart[RED_G][RED_Q];
  const agn_wgrad_desc& d = b.d[blockIdx.y];
  const int nsplit = d.nsplit;
  const int nKb = (d.k + DW_BLK - 1) / DW_BLK, nMb = (d.m + DW_BLK - 1) / DW_BLK;
  const int kpad = nKb * DW_BLK, mpad = nMb * DW_BLK;
  const size_t slab = (size_t)mpad * kpad;
  const int kq = kpad / 4;
  const int t = threadIdx.x % RED_Q, g = threadIdx.x / RED_Q;
  const int qidx = blockIdx.x * RED_Q + t;  // column quad over [mpad][kpad / 4]
  const bool in_slab = qidx < mpad * kq;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (in_slab) {
    const float* p = d.dw_partial + (size_t)qidx * 4;
    // 4 splits' loads in flight per step, added in split order (the same sums)
    int sp = g;
    for (; sp + 3 * RED_G < nsplit; sp += 4 * RED_G) {
      f32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const f32x4*>(p + (size_t)(sp + j * RED_G) * slab);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[0] += v[j][0]; s[1] += v[j][1]; s[2] += v[j][2]; s[3] += v[j][3];
      }
    }
    for (; sp < nsplit; sp += RED_G) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(p + (size_t)sp * slab);
      s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
    }
  }
  part[g][t] = s;
  // bias: block b covers bias entries RED_Q b .. RED_Q b + RED_Q - 1
  const int bi = blockIdx.x * RED_Q + t;
  float bs = 0.f;
  if (d.db && bi < d.m)
    for (int sp = g; sp < nsplit; sp += RED_G) bs += d.db_partial[(size_t)sp * mpad + bi];
  bpart[g][t] = bs;
  __syncthreads();
  if (g == 0) {
    f32x4 r = part[0][t];
    float rb = bpart[0][t];
#pragma unroll
    for (int j = 1; j < RED_G; ++j) {
      const f32x4 v = part[j][t];
      r[0] += v[0]; r[1] += v[1]; r[2] += v[2]; r[3] += v[3];
      rb += bpart[j][t];
    }
    if (in_slab) {
      const int m = qidx / kq, k0 = 4 * (qidx - m * kq);
      if (m < d.m) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k0 + e < d.k) d.dw[(size_t)m * d.ldw + k0 + e] = r[e];
      }
    }
    if (d.db && bi < d.m) d.db[bi] = rb;
  }
}

// deterministic 2-level column reduction of a [nw][n] fp32 matrix
__global__ void colsum_stage1(const float* __restrict__ p, int nw, int n, int chunk, float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int r0 = blockIdx.y * chunk, r1 = min(nw, r0 + chunk);
  if (c >= n) return;
  float s = 0.f;
  int r = r0;
  for (; r + 3 < r1; r += 4) {  // 4 loads in flight, added in row order
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = p[(size_t)(r + j) * n + c];
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[j];
  }
  for (; r < r1; ++r) s += p[(size_t)r * n + c];
  part[(size_t)blockIdx.y * n + c] = s;
}

// stage 2: RED_G groups per 64 columns, group g sums chunks g, g + RED_G, ..., then the group
// partials are added in group order (fixed order: deterministic)
__global__ __launch_bounds__(64 * RED_G) void colsum_stage2(const float* __restrict__ part, int nc, int n,
                                                           float* __restrict__ out) {
  __shared__ float red[RED_G][64];
  const int t = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + t;
  float s = 0.f;
  if (c < n) {
    int r = g;
    for (; r + 3 * RED_G < nc; r += 4 * RED_G) {  // 4 loads in flight, added in chunk order
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = part[(size_t)(r + j * RED_G) * n + c];
#pragma unroll
      for (int j = 0; j < 4; ++j) s += v[j];
    }
    for (; r < nc; r += RED_G) s += part[(size_t)r * n + c];
  }
  red[g][t] = s;
  __syncthreads();
  if (g == 0 && c < n) {
    float r = red[0][t];
#pragma unroll
    for (int j = 1; j < RED_G; ++j) r += red[j][t];
    out[c] = r;
  }
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

namespace {
int wgrad_resident() {
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, ncu = 256, per = 3;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ncu = p.multiProcessorCount;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, wgrad_kernel<bf16, false>, DW_THREADS, 0) != hipSuccess || per < 1)
      per = 3;
    resident = ncu * per;
  }
  return resident;
}
int out_blocks(const agn_wgrad_desc& d) { return ((d.m + DW_BLK - 1) / DW_BLK) * ((d.k + DW_BLK - 1) / DW_BLK); }
}  // namespace

int agn_wgrad_nsplit(int rows, int ndesc_blocks) {
  // exactly one full wave of resident workgroups over all descriptors/blocks (no tail wave),
  // >= 2 LDS stages per split
  int ns = wgrad_resident() / (ndesc_blocks > 0 ? ndesc_blocks : 1);
  const int maxs = (rows + 2 * DW_ROWS - 1) / (2 * DW_ROWS);
  if (ns > maxs) ns = maxs;
  return ns < 1 ? 1 : ns;
}

size_t agn_wgrad_partial_floats(int m, int k, int nsplit) {
  const int mp = (m + DW_BLK - 1) / DW_BLK * DW_BLK, kp = (k + DW_BLK - 1) / DW_BLK * DW_BLK;
  return (size_t)nsplit * mp * kp;
}

int agn_wgrad_plan(agn_wgrad_batch* b) {
  // One wave of resident workgroups. Splits are uniform across the descs of a batch: the kernel is
  // HBM-bound, so a desc whose splits finish early leaves bandwidth to the others; splitting in
  // proportion to rows measured 6 % slower at C3 (more, shorter splits) and is not used.
  if (!b || b->n < 1 || b->n > AGN_MAX_WGRAD) return AGN_E_ARG;
  int nblk = 0, rows = 0;
  for (int i = 0; i < b->n; ++i) {
    nblk += out_blocks(b->d[i]);
    rows = b->d[i].rows > rows ? b->d[i].rows : rows;
  }
  const int ns = agn_wgrad_nsplit(rows, nblk);
  for (int i = 0; i < b->n; ++i) b->d[i].nsplit = ns;
  return 0;
}

int agn_wgrad(const agn_wgrad_batch* b, int dtype, int nsplit, void* stream) {
  if (!b || b->n < 1 || b->n > AGN_MAX_WGRAD) return AGN_E_ARG;
  agn_wgrad_batch bb = *b;
  int total = 0, maxq = 1;
  for (int i = 0; i < bb.n; ++i) {
    agn_wgrad_desc& d = bb.d[i];
    if (d.m < 1 || d.k < 1 || d.rows < 0) return AGN_E_ARG;
    if ((d.g_tiled && d.m != DW_BLK) || (d.x_tiled && d.k != DW_BLK)) return AGN_E_SHAPE;
    if (d.xidx && d.x_tiled) return AGN_E_ARG;
    if (nsplit > 0) d.nsplit = nsplit;
    if (d.nsplit < 1) return AGN_E_ARG;
    total += out_blocks(d) * d.nsplit;
    const int kpad = ((d.k + DW_BLK - 1) / DW_BLK) * DW_BLK, mpad = ((d.m + DW_BLK - 1) / DW_BLK) * DW_BLK;
    maxq = mpad * kpad / 4 > maxq ? mpad * kpad / 4 : maxq;
  }
  hipStream_t st = (hipStream_t)stream;
  // one split count for the whole batch (agn_wgrad_plan is uniform): grid (split, block, desc)
  const int ns = bb.d[0].nsplit;
  int maxblk = 1;
  for (int i = 0; i < bb.n; ++i) {
    if (bb.d[i].nsplit != ns) return AGN_E_ARG;
    maxblk = out_blocks(bb.d[i]) > maxblk ? out_blocks(bb.d[i]) : maxblk;
  }
  (void)total;
  dim3 grid(ns, maxblk, bb.n);
  bool xg = false;
  for (int i = 0; i < bb.n; ++i) xg = xg || bb.d[i].xidx != nullptr;
#define AGN_WG(T)                                                                             \
  do {                                                                                        \
    if (xg) hipLaunchKernelGGL((wgrad_kernel<T, true>), grid, dim3(DW_THREADS), 0, st, bb, ns); \
    else hipLaunchKernelGGL((wgrad_kernel<T, false>), grid, dim3(DW_THREADS), 0, st, bb, ns);   \
  } while (0)
  if (dtype == AGN_BF16) AGN_WG(bf16);
  else if (dtype == AGN_F16) AGN_WG(f16);
  else if (dtype == AGN_F32) AGN_WG(float);
  else return AGN_E_DTYPE;
#undef AGN_WG
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((maxq + RED_Q - 1) / RED_Q, bb.n), dim3(RED_Q * RED_G), 0, st, bb);
  return launch_status();
}

int agn_wgrad_reduce(const agn_wgrad_batch* b, int nsplit, void* stream) {
  if (!b || b->n < 1 || b->n > AGN_MAX_WGRAD || nsplit < 1) return AGN_E_ARG;
  agn_wgrad_batch bb = *b;
  int maxq = 1;
  for (int i = 0; i < bb.n; ++i) {
    bb.d[i].nsplit = nsplit;
    const int kpad = ((bb.d[i].k + DW_BLK - 1) / DW_BLK) * DW_BLK;
    const int mpad = ((bb.d[i].m + DW_BLK - 1) / DW_BLK) * DW_BLK;
    maxq = mpad * kpad / 4 > maxq ? mpad * kpad / 4 : maxq;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((maxq + RED_Q - 1) / RED_Q, bb.n), dim3(RED_Q * RED_G), 0, (hipStream_t)stream, bb);
  return launch_status();
}

int agn_colsum(const float* p, int nw, int n, float* scratch, int scratch_rows, float* out, void* stream) {
  if (nw < 0 || n < 1 || scratch_rows < 1) return AGN_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (nw == 0) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * n, st);
    return e == hipSuccess ? 0 : (int)e;
  }
  const int chunk = (nw + scratch_rows - 1) / scratch_rows;
  const int nc = (nw + chunk - 1) / chunk;
  hipLaunchKernelGGL(colsum_stage1, dim3((n + 255) / 256, nc), dim3(256), 0, st, p, nw, n, chunk, scratch);
  hipLaunchKernelGGL(colsum_stage2, dim3((n + 63) / 64), dim3(64 * RED_G), 0, st, scratch, nc, n, out);
  return launch_status();
}

}  // extern "C"
