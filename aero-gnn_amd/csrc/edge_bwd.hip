// Fused backward of the sum-trick edge MLP with in-kernel weight gradients (gfx950, bf16, H=128).
//
// Reference chain (mgnLayer.py:72-105, residual :205):
//   h0 = e W_e^T + P_s[src] + P_d[dst];  a1 = relu(h0); h1 = a1 W1^T + b1; a2 = relu(h1);
//   h2 = a2 W2^T + b2; a3 = relu(h2); h3 = a3 W3^T + b3; e' = e + LN(h3).
// Backward for one edge tile (S = dL/de' = g + g2[dst]):
//   G3 = LN'(S)  -> dW3 += G3^T a3, db3 += sum G3
//   G2 = (G3 W3) . [a3 > 0] -> dW2 += G2^T a2 ...  G1 -> dW1 += G1^T a1;  G0 = (G1 W1) . [a1 > 0]
//   de = G0 W_e + S;  G0 is written (its sender / receiver sums are dP_s / dP_d; dW_e = G0^T e).
//
// The split path (agn_mlp_backward + agn_wgrad) writes G0..G3 (1 KB/edge) and agn_wgrad reads them
// back together with the saved activations (2 KB/edge). Here one persistent launch keeps dW1..dW3
// in registers for its whole lifetime, so G1..G3 never reach HBM:
//
//  * one 256-thread block per CU (4 waves, one per SIMD: 512 registers each); the block walks
//    ROUNDS of 128 edges (four 32-row tiles, tile p on wave p) in CSC order, XCD-grouped like
//    the resident kernels;
//  * per layer step L = 3, 2, 1 the round's G_L and X_L (= a_L) sit in LDS as [128 rows][128]
//    bf16 images (XOR-swizzled 8-byte units, see swz): the dW MFMAs read 8-row columns of both
//    with ds_read_b64_tr_b16 (k = rows), the chain MFMA (rows on lanes, common.hpp) reads its B
//    operand rows straight from the G image and W_L^T from a double-buffered LDS copy that the
//    previous step prefetched with global_load_lds;
//  * wave w owns dW_L[0..127][32w..32w+31] for L = 1..3: 4 accumulator tiles per L, 192
//    registers for the whole launch; its 32 dW MFMAs per step match its 32 chain MFMAs;
//  * the LayerNorm backward runs before this kernel (an LN-only agn_mlp_backward writes G3);
//    db_L are column sums of the G_L images.
// Measured: exact, but latency-bound at one wave per SIMD, so it is opt-in.
// Partials per block go to slabs summed in fixed order by agn_wgrad_reduce / agn_colsum: no atomics.
#include "common.hpp"
#include "aerognn.h"

#include <type_traits>

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int EB_WAVES = 4;                 // one wave per SIMD: 512 registers each
constexpr int EB_THREADS = 64 * EB_WAVES;
constexpr int EB_ROUND = 32 * EB_WAVES;     // rows per round: one 32-row tile per wave
constexpr int LDI = 128;                    // LDS image row stride (bf16), unpadded: bank spread by swizzle
constexpr int WUNITS = 4 * 8 * 64;          // packed 128x128 operand: [ot 4][ku 8][lane 64] x 16 B = 32 KB

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// LDS images [rows][128] bf16 are stored with an XOR swizzle of their 8-byte units:
// unit u of row r sits at u ^ f(r & 31), f(x) = (x & 3) << 3 | x >> 2. Both read patterns are then
// conflict-free: a row per lane (32 rows, one unit: f injective over 0..31) and the transposed
// reads (rows kb..kb+3 x 8 units per 32-lane half: q << 3 picks 4 distinct 8-unit blocks).
AGN_DEV int swz(int r, int col) {  // element offset of (row, col), col a multiple of 4
  const int x = r & 31;
  return r * LDI + (col ^ ((((x & 3) << 3) | (x >> 2)) << 2));
}

// 8 consecutive rows (kb..kb+7) of one column of an LDS image: the MFMA A/B fragment with k = rows
AGN_DEV bf16x8 tr8(const bf16* img, int kb, int col_base, int lane) {
  const int q = (lane & 15) >> 2, pp = lane & 3;
  const bf16* a0 = img + swz(kb + q, col_base + 4 * pp);
  const bf16* a1 = img + swz(kb + 4 + q, col_base + 4 * pp);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo);
  const bf16x4 h4 = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{l4[0], l4[1], l4[2], l4[3], h4[0], h4[1], h4[2], h4[3]};
}

// B operand of the rows-on-lanes chain MFMA for k-step u (features 16u+4h..+3 | 16u+8+4h..+3 of
// the lane's row, common.hpp acc-register order) from a row of an LDS image
AGN_DEV bf16x8 brow(const bf16* img, int r, int u, int h) {
  const u32x2 lo = *reinterpret_cast<const u32x2*>(img + swz(r, 16 * u + 4 * h));
  const u32x2 hi = *reinterpret_cast<const u32x2*>(img + swz(r, 16 * u + 8 + 4 * h));
  return __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
}
// 8-byte unit store / load of an LDS image
AGN_DEV void put4(bf16* img, int r, int col, uint32_t a, uint32_t b) {
  *reinterpret_cast<u32x2*>(img + swz(r, col)) = u32x2{a, b};
}
AGN_DEV u32x2 get4(const bf16* img, int r, int col) { return *reinterpret_cast<const u32x2*>(img + swz(r, col)); }

// dW accumulation with the accumulator pinned to AGPRs ("+a"): the dW tiles live for the whole
// launch (192 AGPRs per lane), so the VALU working set keeps all 256 arch VGPRs.
AGN_DEV void mfma_acc(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// Wait for every outstanding vector-memory operation of this wave, global_load_lds included
// (the LDS copy is only visible to the other waves after this wait and the next barrier).
AGN_DEV void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Async copy of one packed 32 KB operand into an LDS buffer: 8 x 1 KB per wave (lane-linear).
AGN_DEV void glds_weights(uint4* dst, const void* src, int wave, int lane) {
  const char* g = reinterpret_cast<const char*>(src);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int piece = wave * 8 + j;  // 32 pieces of 1 KB
    __builtin_amdgcn_global_load_lds(g + piece * 1024 + lane * 16,
                                     (__attribute__((address_space(3))) void*)(dst + piece * 64), 16, 0, 0);
  }
}

// One 32-row tile of an AGN_TILED [rows][128] bf16 matrix (8 KB: 8 units per lane, 1 KB per
// instruction), moved to rows 32p.. of an LDS image in natural feature order.
struct TiledTile {
  uint4 v[8];
  AGN_DEV void load(const void* base, int tile, int ntiles, int rows, int lane) {
    const uint4* b = reinterpret_cast<const uint4*>(base) + (size_t)tile * 8 * 64;
    const bool ok = tile < ntiles && tile * 32 + (lane & 31) < rows;  // padded rows are never written
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ok ? b[i * 64 + lane] : uint4{0u, 0u, 0u, 0u};
  }
  // unit (i, lane = c + 32 hh) holds features 16i+4hh..+3 | 16i+8+4hh..+3 of row c
  AGN_DEV void store(bf16* img, int p, int lane) const {
    const int r = 32 * p + (lane & 31), h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, v[i]);
      put4(img, r, 16 * i + 4 * h, x[0], x[1]);
      put4(img, r, 16 * i + 8 + 4 * h, x[2], x[3]);
    }
  }
};

// A row-major [rows][128] bf16 tile row pair (16 B per lane at features 16i + 8h): the incoming
// gradient rows of the residual (common.hpp load8_w without the exchange, done at use)
struct RowTile {
  uint4 v[8];
  AGN_DEV void load(const bf16* rowp, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const uint4*>(rowp + 16 * i + 8 * (lane >> 5));
  }
  AGN_DEV void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = uint4{0u, 0u, 0u, 0u};
  }
};

__global__ __launch_bounds__(EB_THREADS, 1) void edge_bwd_fused_kernel(const agn_edge_bwd_args a) {
  __shared__ uint4 wbuf[2][WUNITS];
  __shared__ __attribute__((aligned(16))) bf16 gs[EB_ROUND * LDI];
  __shared__ __attribute__((aligned(16))) bf16 xs[EB_ROUND * LDI];

  const int lane0 = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntiles = (a.rows + 31) / 32;
  const int nrounds = (ntiles + EB_WAVES - 1) / EB_WAVES;
  // XCD-grouped round walk (blocks b and b + 8 share an XCD and its L2)
  int first, end, step;
  if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
    const int grp = blockIdx.x & 7, per = (nrounds + 7) / 8;
    first = grp * per + (blockIdx.x >> 3);
    end = min(nrounds, (grp + 1) * per);
    step = gridDim.x >> 3;
  } else {
    first = blockIdx.x;
    end = nrounds;
    step = gridDim.x;
  }

  // wave w owns dW_L[0..127][32w..32w+31] (4 output tiles) for L = 1..3, in AGPRs (mfma_acc)
  f32x16 dw[3][4];
#pragma unroll
  for (int l = 0; l < 3; ++l)
#pragma unroll
    for (int t = 0; t < 4; ++t) dw[l][t] = f32x16{};
  float db[3][4];
#pragma unroll
  for (int l = 0; l < 3; ++l) db[l][0] = db[l][1] = db[l][2] = db[l][3] = 0.f;

  // prologue: W3^T -> buffer 1 (buffers: W3, W1 in 1; W2, W_e in 0); the first round's G3 and a3
  glds_weights(wbuf[1], a.wtpk[3], w, lane0);
  if (first < end) {
    TiledTile t3;
    t3.load(a.g3, first * EB_WAVES + w, ntiles, a.rows, lane0);
    t3.store(gs, w, lane0);
    t3.load(a.act[2], first * EB_WAVES + w, ntiles, a.rows, lane0);
    t3.store(xs, w, lane0);
  }
  vm_drain();
  __syncthreads();

  // diagnostic timing (a.stamps != NULL, a separate measurement run): s_memtime per phase for
  // blocks 0 and 128, every wave, the first 8 rounds -> stamps[((sel * 4 + w) * 8 + round) * 32 + point]
  unsigned long long* stp = nullptr;
  if (a.stamps && (blockIdx.x == 0 || blockIdx.x == 128))
    stp = a.stamps + ((size_t)((blockIdx.x == 0 ? 0 : 1) * EB_WAVES + w) * 8) * 32;
  int rcount = 0;
#define EB_STAMP(k)                                                                      \
  do {                                                                                  \
    if (stp && rcount < 8 && lane0 == 0) stp[rcount * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

  for (int rd = first; rd < end; rd += step, ++rcount) {
    EB_STAMP(0);
    const int tile = rd * EB_WAVES + w;
    const int mtile = tile < ntiles ? tile : ntiles - 1;
    const int nrd = rd + step;
    TiledTile xr, gn;  // next step's X image share; next round's G3 share

    // ---------------------------------------------------------------- steps L = 3, 2, 1
    auto layer_step = [&](auto Lc) {
      constexpr int L = decltype(Lc)::value;
      int lane = lane0;
      asm volatile("" : "+v"(lane));  // per-step addresses: recompute, do not hoist
      const int c = lane & 31, hl = lane >> 5;
      const int lr = 32 * w + c;
      const uint4* wcur = wbuf[L & 1];
      glds_weights(wbuf[(L - 1) & 1], a.wtpk[L - 1], w, lane);  // W_{L-1}^T for the next step
      if constexpr (L >= 2) {
        xr.load(a.act[L - 2], tile, ntiles, a.rows, lane);  // X_{L-1} = a_{L-1}
      } else if (nrd < end) {
        xr.load(a.act[2], nrd * EB_WAVES + w, ntiles, a.rows, lane);  // next round: a3, G3
        gn.load(a.g3, nrd * EB_WAVES + w, ntiles, a.rows, lane);
      }
      const uint32_t* mp = reinterpret_cast<const uint32_t*>(a.mask[L - 1]) + (size_t)mtile * 2 * 64 + lane;
      const uint32_t mk0 = mp[0], mk1 = mp[64];
      // dW_L[:, 32w..] += G_L^T X_L over the round's rows
#pragma unroll 4
      for (int ks = 0; ks < EB_ROUND / 16; ++ks) {
        const int kb = 16 * ks + 8 * hl;
        const int sub = 16 * ((lane >> 4) & 1);
        const bf16x8 xb = tr8(xs, kb, 32 * w + sub, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 ga = tr8(gs, kb, 32 * t + sub, lane);
          dw[L - 1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, xb, dw[L - 1][t], 0, 0, 0);
        }
      }
      EB_STAMP(1 + 5 * (3 - L));
      // db_L partial: thread (rg, cq) sums rows 16rg..16rg+15 of features 4cq..4cq+3
      {
        const int cq = threadIdx.x & 31, rg = threadIdx.x >> 5;
#pragma unroll 4
        for (int r = 0; r < EB_ROUND / 8; ++r) {
          const u32x2 x = get4(gs, 16 * rg + r, 4 * cq);
          db[L - 1][0] += lo_bf16(x[0]);
          db[L - 1][1] += hi_bf16(x[0]);
          db[L - 1][2] += lo_bf16(x[1]);
          db[L - 1][3] += hi_bf16(x[1]);
        }
      }
      // chain: G_{L-1} = (G_L W_L) . [a_L > 0], rows on lanes (the k-step / tile order of
      // common.hpp gemm(): bitwise the split path's pre-activation gradients)
      f32x16 acc[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
#pragma unroll 4
      for (int u = 0; u < 8; ++u) {
        const bf16x8 b = brow(gs, lr, u, hl);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 wa = __builtin_bit_cast(bf16x8, wcur[(t * 8 + u) * 64 + lane]);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, b, acc[t], 0, 0, 0);
        }
      }
      EB_STAMP(2 + 5 * (3 - L));
      __syncthreads();  // every read of the G / X images and of W_L is done
      EB_STAMP(3 + 5 * (3 - L));
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t mk = (t < 2) ? mk0 : mk1;  // register 16t + r -> dword t >> 1, bit 16 (t & 1) + r
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int bit = 16 * (t & 1) + 4 * q + e;
            v[e] = __uint_as_float(__float_as_uint(acc[t][4 * q + e]) & (uint32_t)__builtin_amdgcn_sbfe((int32_t)mk, bit, 1));
          }
          put4(gs, lr, 32 * t + 8 * q + 4 * hl, pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
      if constexpr (L >= 2) xr.store(xs, w, lane);
      vm_drain();  // W_{L-1}^T has landed
      EB_STAMP(4 + 5 * (3 - L));
      __syncthreads();
      EB_STAMP(5 + 5 * (3 - L));
    };
    layer_step(std::integral_constant<int, 3>{});
    layer_step(std::integral_constant<int, 2>{});
    layer_step(std::integral_constant<int, 1>{});

    // ---------------------------------------------------------------- step 0: de, G0
    {
      int lane = lane0;
      asm volatile("" : "+v"(lane));
      const int c = lane & 31, hl = lane >> 5;
      const int lr = 32 * w + c;
      const int row = tile * 32 + c;
      const bool valid = tile < ntiles && row < a.rows;
      const int rr = valid ? row : a.rows - 1;
      if (nrd < end) {
        glds_weights(wbuf[1], a.wtpk[3], w, lane);  // next round's W3^T
        xr.store(xs, w, lane);                      // X image is free in step 0 (dW_e is not fused)
      }
      RowTile g1, g2;  // residual: dL/de' = g + g2[dst]
      if (a.g) g1.load(reinterpret_cast<const bf16*>(a.g) + (size_t)rr * H, lane);
      else g1.zero();
      g2.load(reinterpret_cast<const bf16*>(a.g2) + (size_t)a.gidx[rr] * H, lane);
      f32x16 acc[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
      const uint4* wcur = wbuf[0];
#pragma unroll 4
      for (int u = 0; u < 8; ++u) {
        const bf16x8 b = brow(gs, lr, u, hl);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 wa = __builtin_bit_cast(bf16x8, wcur[(t * 8 + u) * 64 + lane]);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, b, acc[t], 0, 0, 0);
        }
      }
      EB_STAMP(16);
      // de = G0 W_e + (g + g2): acc registers 8i..8i+7 = acc[i >> 1][8 (i & 1) + e]
      bf16* dep = reinterpret_cast<bf16*>(a.de) + (size_t)rr * H;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v[8], x[8], y[8];
        unpack8_w(x, g1.v[i]);
        unpack8_w(y, g2.v[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = acc[i >> 1][8 * (i & 1) + e] + (x[e] + y[e]);
        store8_w(dep, i, hl, v, valid);
      }
      // G0 tile -> HBM (16-B chunks of the own rows of the G image), then the next round's G3
      bf16* g0 = reinterpret_cast<bf16*>(a.g0) + (size_t)tile * 32 * H;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = lane + 64 * k, r = q >> 4, ch = q & 15;
        const u32x2 lo = get4(gs, 32 * w + r, 8 * ch), hi = get4(gs, 32 * w + r, 8 * ch + 4);
        if (tile < ntiles && tile * 32 + r < a.rows)
          *reinterpret_cast<uint4*>(g0 + (size_t)r * H + 8 * ch) = __builtin_bit_cast(uint4, u32x4{lo[0], lo[1], hi[0], hi[1]});
      }
      if (nrd < end) gn.store(gs, w, lane);  // only this wave ever reads its rows in step 0
      EB_STAMP(17);
    }
    vm_drain();       // next round's W3^T has landed
    EB_STAMP(18);
    __syncthreads();
    EB_STAMP(19);
  }
#undef EB_STAMP

  // ---------------------------------------------------------------- per-block partials
  const int lane = lane0, c = lane0 & 31, hl = lane0 >> 5;
  const size_t slab = (size_t)H * H;
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    float* P = a.dw_partial + ((size_t)l * a.nblk + blockIdx.x) * slab;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 32 * t + 8 * (r >> 2) + 4 * hl + (r & 3);
        P[(size_t)m * H + 32 * w + c] = dw[l][t][r];
      }
  }
  // db: 8 row groups per column quad, summed in group order through the (now free) X image
  float* red = reinterpret_cast<float*>(xs);  // [3][8][128] floats = 12 KB
  {
    const int cq = threadIdx.x & 31, rg = threadIdx.x >> 5;
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(l * 8 + rg) * H + 4 * cq + e] = db[l][e];
  }
  __syncthreads();
  (void)lane;
  for (int i = threadIdx.x; i < 3 * H; i += EB_THREADS) {
    const int l = i / H, f = i - l * H;
    float s = 0.f;
    for (int rg = 0; rg < 8; ++rg) s += red[(l * 8 + rg) * H + f];
    a.db_partial[((size_t)l * a.nblk + blockIdx.x) * H + f] = s;
  }
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int g_cus = 0;

}  // namespace

extern "C" {

int agn_edge_bwd_blocks(int rows) {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) g_cus = pr.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  const int rounds = ((rows + 31) / 32 + 3) / 4;
  if (rounds >= g_cus) return g_cus;
  const int n = (rounds + 7) / 8 * 8;
  return n < 8 ? 8 : n;
}

int agn_edge_bwd_fused(const agn_edge_bwd_args* a, void* stream) {
  if (!a || a->rows < 1 || a->nblk < 1 || !a->g2 || !a->gidx || !a->g3 || !a->de || !a->g0 || !a->dw_partial ||
      !a->db_partial)
    return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wtpk[l]) return AGN_E_ARG;
  for (int l = 0; l < 3; ++l)
    if (!a->act[l] || !a->mask[l]) return AGN_E_ARG;
  hipLaunchKernelGGL(edge_bwd_fused_kernel, dim3(a->nblk), dim3(EB_THREADS), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
