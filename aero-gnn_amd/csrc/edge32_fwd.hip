// Forward of the sum-trick edge MLP on 32-row tiles with 32x32x16 MFMAs (gfx950, bf16, H = 128):
//   e' = e + LN(W3 relu(W2 relu(W1 relu(e W_e^T + P_s[src] + P_d[dst]) + b1) + b2) + b3)
// (models/mgnLayer.py:72-105 EdgeBlockSum, residual :205), bitwise agn_mlp_forward's resident
// kernel on the same operands (mlp.hip mlp_fwd_res_kernel: the same MFMA sequence per accumulator,
// the same exact MFMA row sum P_s + P_d, the same LayerNorm and residual steps), so the 32-row
// fused backward (edge_bwd.hip), which recomputes that kernel's chain, pairs with it unchanged.
//
// The residual add round(LN(h3)) + e runs on the matrix cores like the row sum (round 6: 160 VALU
// fewer per tile, -1 % per launch).
//
// Why a second kernel: the chain is vector-issue-bound on the SIMD, not HBM- or MFMA-bound
// (DESIGN.md §9 round 5). A v_mfma_f32_32x32x16_bf16 holds the SIMD's vector issue for 8 of its
// 32 cycles; the exact MFMA row sum replaces ~190 VALU unpack/add instructions per tile. Against the
// resident kernel (two waves per SIMD at <= 256 registers, the previous tile's stores deferred in
// registers) this one runs three waves per SIMD at <= 168 registers, keeping the residual
// operand; the weight fragments stream two deep instead of a whole k-step ahead. (16 waves at
// <= 128 registers, re-reading the residual, spilled and ran 0.94 -> 1.64 ms per C3 launch;
// static per-SIMD wave priorities changed nothing: both removed in round 6.)
//
// Training saves (SAVE): the first ReLU output a1 in AGN_TILED (the packed operand as it stands, one
// 1-KB store per unit) and the LayerNorm (mean, rstd). The fused backward (edge_bwd.hip) starts its
// recompute at Lin1 from them: 264 B per edge written here against e, P_s[src], P_d[dst], W_e and the
// statistics recomputed there.
//
// Persistent: one workgroup per CU, the four packed weight images resident in LDS (128 KB), each
// wave streaming 32-row tiles in CSC order over an XCD-grouped walk; a tile's node ids are loaded
// one tile ahead through the wave's LDS slot (a loop-carried load result would make the compiler
// wait vmcnt(0) at the loop head, i.e. for the previous tile's stores too).
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4;                   // 32-feature output tiles
constexpr int NR = 64;                  // acc registers per lane (features of the lane's row half)
constexpr int NU = 8;                   // k-steps of 16 per layer
constexpr int LAYER = NT * NU * 64;     // packed units (16 B) per weight image
#ifndef AGN_E32_PF
#define AGN_E32_PF 2
#endif
constexpr int PF = AGN_E32_PF;          // weight fragments in flight
#ifndef AGN_E32_DIAG
#define AGN_E32_DIAG 0  // timing diagnostics only (outputs wrong): 1 no LayerNorm statistics, 3 no row sum
#endif

constexpr int NW = 12;  // waves per CU (three per SIMD)

struct Smem {
  uint4 w[4 * LAYER];   // packed A units [layer][ot][ku][lane] (agn_pack trans = 0 layout, as is)
  float pv[5][H];       // b1, b2, b3, LN gamma, LN beta
  int ids[NW][64];      // per wave: next tile's src (lanes 0-31) / dst (32-63)
};
static_assert(sizeof(Smem) <= 160 * 1024, "LDS budget");

// acc[ot] += W[ot tile] . b over k-steps u = 0..7 in order (the resident kernel's per-accumulator
// sequence: common.hpp gemm); fragments (u, ot) stream PF deep, ot inner
AGN_DEV void gemm4(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int lane) {
  uint4 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = w[((i % NT) * NU + i / NT) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < NT * NU; ++idx) {
    const uint4 cur = f[idx % PF];
    const int nx = idx + PF;
    if (nx < NT * NU) f[idx % PF] = w[((nx % NT) * NU + nx / NT) * 64 + lane];
    b.mfma(acc[idx % NT], cur, idx / NT);
  }
}

// XCD-aware walk (mlp.hip ResTiles): blocks b and b + 8 share an XCD and its L2, so each group of
// blocks {g, g + 8, ...} walks one contiguous eighth of the tiles
struct Walk {
  int first, end, step;
  AGN_DEV Walk(int ntiles, int w, int nw) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int g = blockIdx.x & 7, bi = blockIdx.x >> 3, nb = gridDim.x >> 3;
      const int per = (ntiles + 7) / 8;
      first = g * per + bi * nw + w;
      end = min(ntiles, (g + 1) * per);
      step = nb * nw;
    } else {
      first = blockIdx.x * nw + w;
      end = ntiles;
      step = gridDim.x * nw;
    }
  }
};

// Diagnostic phase clocks (built with -DAGN_E32_STAMPS into a separate library only,
// tools/e32_stamps.py): the waves of block 0 record s_memtime at 8 points of their first 16 tiles
// into agn_e32_stamps[(wave * 16 + tile) * 16 + point], s_memrealtime (100 MHz) at point 15.
#ifdef AGN_E32_STAMPS
__device__ unsigned long long* agn_e32_stamps;
#define E32_STAMP(k)                                                                                   \
  do {                                                                                                 \
    if (agn_e32_stamps && blockIdx.x == 0 && lane0 == 0 && ntile < 16)                                 \
      agn_e32_stamps[((threadIdx.x >> 6) * 16 + ntile) * 16 + (k)] =                                    \
          (k) == 15 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();                   \
  } while (0)
#else
#define E32_STAMP(k) \
  do {               \
  } while (0)
#endif

template <bool SAVE>
__global__ __launch_bounds__(64 * NW) void edge32_fwd_kernel(const agn_edge_fwd_args a) {
  constexpr int NTHR = 64 * NW;
  __shared__ Smem sm;
  {
    const uint4* const* wp = reinterpret_cast<const uint4* const*>(a.wpk);
    for (int i = threadIdx.x; i < 4 * LAYER; i += NTHR) sm.w[i] = wp[i / LAYER][i % LAYER];
    for (int i = threadIdx.x; i < 5 * H; i += NTHR) {
      const int l = i / H, f = i - l * H;
      sm.pv[l][f] = l < 3 ? (a.bias[l + 1] ? a.bias[l + 1][f] : 0.f) : (l == 3 ? a.ln_g[f] : a.ln_b[f]);
    }
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 31) / 32;
  const Walk walk(ntiles, w, NW);
  int* wids = sm.ids[w];
  const int32_t* const idp = lane0 < 32 ? a.src : a.dst;
  auto tile_id = [&](int t) { return idp[min(t * 32 + (lane0 & 31), a.rows - 1)]; };
  if (walk.first < walk.end) wids[lane0] = tile_id(walk.first);
  const bf16* P = reinterpret_cast<const bf16*>(a.proj);
  const bf16* E = reinterpret_cast<const bf16*>(a.e);
#ifdef AGN_E32_STAMPS
  int ntile = 0;
#endif
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    E32_STAMP(0);
    E32_STAMP(15);
    // lane-derived offsets recomputed per tile, not hoisted and kept live (common.hpp opaque_v)
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const bool more = tile + walk.step < walk.end;
    const int nid = tile_id(more ? tile + walk.step : tile);
    f32x16 acc[NT];
    BOp<bf16, NR> b;
    {
      const int cs = wids[c], cd = wids[32 + c];
      if (more) wids[lane] = nid;  // (this tile's reads of the slot are done: LDS is in order per wave)
      // acc = P_s[src] + P_d[dst] on the matrix cores (exact fp32 add, common.hpp acc_add2_mfma)
      uint4 rs[NR / 8], rd[NR / 8];
      const bf16* ps = P + (size_t)cs * (2 * H) + 8 * h;
      const bf16* pd = P + (size_t)cd * (2 * H) + H + 8 * h;
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        rs[i] = *reinterpret_cast<const uint4*>(ps + 16 * i);
        rd[i] = *reinterpret_cast<const uint4*>(pd + 16 * i);
      }
      b.load_w(E + (size_t)rr * H, h);
      // all 24 row loads in flight before the first use: without this fence the scheduler of the
      // SAVE instantiation (a1 / statistics stores, 152 registers) issued the P_d rows two at a time
      // behind vmcnt(0) waits (1.01 -> 1.46 ms per C3 launch)
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 f0, f1;
      ident_frags_rows(f0, f1, lane);
      if (AGN_E32_DIAG == 3) {
#pragma unroll
        for (int ot = 0; ot < NT; ++ot) acc[ot] = f32x16{};
      } else {
        acc_add2_mfma_rows<NT, NR / 8>(acc, rs, rd, f0, f1);  // rows as loaded: no lane-half exchange
      }
    }
    E32_STAMP(1);
    const BOp<bf16, NR> e0 = b;  // the residual operand
    gemm4(acc, b, sm.w, lane);
    E32_STAMP(2);
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      cbarrier();
      b.template set_relu<NT>(acc);
      if constexpr (SAVE) {  // a1 (AGN_TILED); behind Lin1's MFMAs or non-temporal: no faster (round 6)
        if (l == 1) b.store_tiled(reinterpret_cast<bf16*>(a.act[0]), row, h, valid);
      }
#pragma unroll
      for (int q = 0; q < 4 * NT; ++q) {  // acc = bias of Linear l (mlp.hip acc_bias_lds)
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sm.pv[l - 1][8 * q + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
      }
      gemm4(acc, b, sm.w + l * LAYER, lane);
      E32_STAMP(2 + l);
    }
    cbarrier();
    // LayerNorm statistics over the row's 128 features (two lanes per row), resident kernel order
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < (AGN_E32_DIAG == 1 ? 1 : NR); ++i) s += acc[i / 16][i % 16];
    s = sum32(s);
    const float mean = s / (float)H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < (AGN_E32_DIAG == 1 ? 2 : NR); i += 2) q = ln_sq_acc2(q, acc[i / 16][i % 16], acc[(i + 1) / 16][(i + 1) % 16], mean);
    q = sum32(q);
    const float rstd = 1.0f / sqrtf(q / (float)H + 1e-5f);
    if constexpr (SAVE) {
      if (h == 0 && valid) *reinterpret_cast<f32x2*>(a.stats + 2 * (size_t)row) = f32x2{mean, rstd};
    }
    E32_STAMP(6);
    bf16* op = reinterpret_cast<bf16*>(a.out) + (size_t)row * H;
    {
      // LN(h3) rounded to bf16 (the operand's packing), then round(LN) + e on the matrix cores: the
      // identity-fragment sum of two bf16 rows is the VALU path's fp32 add bit for bit (a -0 sum
      // comes out +0), and it replaces 160 unpack / add VALU per tile
      float v[NR];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int f0 = 16 * i + 8 * j + 4 * h;
          const f32x4 g4 = *reinterpret_cast<const f32x4*>(&sm.pv[3][f0]);
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sm.pv[4][f0]);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const int r = 8 * i + 4 * j + e;
            const f32x2 o = ln_out2(f2(acc[r / 16][r % 16], acc[(r + 1) / 16][(r + 1) % 16]), mean, rstd,
                                    f2(g4[e], g4[e + 1]), f2(b4[e], b4[e + 1]));
            v[r] = o[0];
            v[r + 1] = o[1];
          }
        }
      }
      BOp<bf16, NR> lnb;
      lnb.set(v);
      bf16x8 f0, f1;
      ident_frags(f0, f1, lane);
      acc_add2_mfma<NT, NR>(acc, lnb, e0, f0, f1);
    }
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
      store8_w(op, i, h, v, valid);
    }

    E32_STAMP(7);
#ifdef AGN_E32_STAMPS
    ++ntile;
#endif
  }
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int g_cus = 0;
int cu_count() {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) g_cus = pr.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  return g_cus;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

#ifdef AGN_E32_STAMPS
int agn_debug_e32_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(agn_e32_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

int agn_edge_fwd32_blocks(int rows) {
  const int cus = cu_count();
  const int tiles = (rows + 31) / 32;
  const int need = (tiles + NW - 1) / NW;
  if (need >= cus) return cus;
  const int n = (need + 7) / 8 * 8;
  return n < 8 ? 8 : n;
}

int agn_edge_forward32(const agn_edge_fwd_args* a, void* stream) {
  if (!a || a->rows < 0 || a->nblk < 1) return AGN_E_ARG;
  if (a->rows == 0) return 0;
  if (!a->e || !a->proj || !a->src || !a->dst || !a->out || !a->ln_g || !a->ln_b) return AGN_E_ARG;
  if (a->act[1] || a->act[2] || a->hpre) return AGN_E_ARG;  // a1 and the statistics are the only saves
  const bool save = a->act[0] != nullptr;
  if (save != (a->stats != nullptr) || (save && (!al16(a->act[0]) || (reinterpret_cast<uintptr_t>(a->stats) & 7))))
    return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wpk[l] || !al16(a->wpk[l])) return AGN_E_ARG;
  if (!al16(a->e) || !al16(a->proj) || !al16(a->out)) return AGN_E_ARG;
  if (save) hipLaunchKernelGGL(edge32_fwd_kernel<true>, dim3(a->nblk), dim3(64 * NW), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL(edge32_fwd_kernel<false>, dim3(a->nblk), dim3(64 * NW), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
