// Node-row projections of the sum-trick edge block (mgnLayer.py:72-105), as one persistent
// resident-weight kernel (gfx950, bf16, H = 128):
//   forward   P[r, 0:256]  = x[r] [W_s; W_d]^T + [0; b]            (agn_proj_forward, 1 segment)
//   backward  dx[r]       += dP_s[r] W_s + dP_d[r] W_d             (agn_proj_backward, 2 segments)
// The general MLP kernel runs these as 4-wave blocks that restage the packed weights (64 KB) from
// L2 for every 128 rows and synchronise per segment; at these shapes (1 Linear, short rows) that
// staging, not HBM, set their time (≈2 TB/s). Here each block stages the whole packed matrix
// once and its waves stream 32-row tiles, with every row load / store going through an 8-row LDS
// staging area (1-KB contiguous instructions, common.hpp tile_load_chunks / tile_store_chunks).
// Arithmetic, MFMA k-order and rounding are those of mlp_fwd_kernel (nlin = 1, M_VEC): outputs
// are bitwise identical (tests/test_gpu_fullsize.py::test_proj_kernels_bitwise_equal_general).
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4, NR = 64;
constexpr int PJ_WPB = 4;  // 4-wave blocks, two per CU (64 KB weights + 9 KB staging each)
constexpr int PJ_BLOCK = 64 * PJ_WPB;
constexpr int PJ_UNITS = 8 * 8 * 64;  // packed [8 out tiles][8 k-units] or [4][16] x 16 B: 64 KB

// XCD-grouped tile walk (blocks b and b + 8 share an XCD and its L2), as the resident kernels
struct Tiles {
  int first, end, step;
  AGN_DEV Tiles(int ntiles, int wid) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int g = blockIdx.x & 7, bi = blockIdx.x >> 3, nb = gridDim.x >> 3;
      const int per = (ntiles + 7) / 8;
      first = g * per + bi * PJ_WPB + wid;
      end = min(ntiles, (g + 1) * per);
      step = nb * PJ_WPB;
    } else {
      first = blockIdx.x * PJ_WPB + wid;
      end = ntiles;
      step = gridDim.x * PJ_WPB;
    }
  }
};


// NSEG input segments of 128 features; NGRP output groups of 128 (packed matrix: NGRP * 4 out
// tiles x NSEG * 8 k-units, unit = (ot * KU + ku) * 64 + lane)
template <int NSEG, int NGRP>
__global__ __launch_bounds__(PJ_BLOCK, 2) void proj_kernel(int rows, const bf16* __restrict__ x0,
                                                         const bf16* __restrict__ x1, int x_ld,
                                                         const uint4* __restrict__ wpk, const float* __restrict__ bias,
                                                         const bf16* resid, bf16* out,  // may alias (dx +=)
                                                         int out_ld) {
  static_assert(NSEG * NGRP == 2, "64 KB of packed weights");
  constexpr int KU = 8 * NSEG;
  __shared__ uint4 w[PJ_UNITS];
  __shared__ uint4 stg[PJ_WPB][8][H / 8 + STG_PAD];  // per-wave 8-row staging: 1-KB row I/O
  for (int i = threadIdx.x; i < PJ_UNITS; i += PJ_BLOCK) w[i] = wpk[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int c = lane & 31, h = lane >> 5;
  const int ntiles = (rows + 31) / 32;
  const int wid = threadIdx.x >> 6;
  const Tiles tw(ntiles, wid);
  for (int tile = tw.first; tile < tw.end; tile += tw.step) {
    cbarrier();  // keep the LDS weight reads inside the loop
    // one input segment (the forward's x): its tile is loaded once for both output groups, so
    // group 1 does not reload it behind group 0's stores (a load wait also waits for every
    // older store: DESIGN.md §9, round 4)
    BOp<bf16, NR> b1;
    if constexpr (NSEG == 1) {
      uint4 mine[NR / 8];
      tile_load_chunks<H / 8>(mine, x0 + (size_t)tile * 32 * x_ld, rows - tile * 32, stg[wid], lane, x_ld / 8);
      b1.set_w(mine);
    }
#pragma unroll
    for (int grp = 0; grp < NGRP; ++grp) {
      f32x16 acc[NT];
      {
        float v[NR];
        if (bias) load_param<NR, true>(v, bias + grp * H, H, h);
        else load_param<NR, false>(v, nullptr, H, h);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t][r] = v[16 * t + r];
      }
#pragma unroll
      for (int s = 0; s < NSEG; ++s) {
        BOp<bf16, NR> b;
        if constexpr (NSEG == 1) {
          b = b1;
        } else {
          uint4 mine[NR / 8];
          tile_load_chunks<H / 8>(mine, (s == 0 ? x0 : x1) + (size_t)tile * 32 * x_ld, rows - tile * 32, stg[wid],
                                  lane, x_ld / 8);
          b.set_w(mine);
        }
        gemm<bf16, NT, NR, true>(acc, b, 8, w + ((size_t)grp * NT * KU + 8 * s) * 64, KU, NT, lane);
      }
      uint4 res[NR / 8];
      if (resid)
        tile_load_chunks<H / 8>(res, resid + (size_t)tile * 32 * out_ld + grp * H, rows - tile * 32, stg[wid], lane,
                                out_ld / 8);
      uint4 ob[NR / 8];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
        if (resid) {
          float r8[8];
          unpack8_w(r8, res[i]);
#pragma unroll
          for (int e = 0; e < 8; ++e) v8[e] = round_t<bf16>(v8[e]) + r8[e];
        }
        ob[i] = pack8_w(v8, h);
      }
      // output rows through the LDS staging rows: 1-KB store instructions (direct 16-B stores
      // measured slower, 94 -> 120 us per C3 launch: DESIGN.md §9, round 3)
      tile_store_chunks<H / 8>(ob, out + (size_t)tile * 32 * out_ld + grp * H, rows - tile * 32, stg[wid], lane,
                                 out_ld / 8);
    }
  }
}

int g_cus = 0;
int blocks(int rows) {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) g_cus = p.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  const int need = ((rows + 31) / 32 + PJ_WPB - 1) / PJ_WPB;
  const int cap = 2 * g_cus;  // 64 KB of LDS and 128 VGPRs: two blocks per CU
  return need < cap ? (need > 0 ? need : 1) : cap;
}
inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }
inline int status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

int agn_proj_forward(int rows, const void* x, int x_ld, const void* wpk, const float* bias, void* out, int out_ld,
                     void* stream) {
  if (rows < 0 || !x || !wpk || !out || x_ld % 8 || out_ld % 8 || out_ld < 2 * H || !al16(x) || !al16(out) ||
      !al16(wpk) || (bias && !al16(bias)))
    return AGN_E_ARG;
  if (rows == 0) return 0;
  hipLaunchKernelGGL((proj_kernel<1, 2>), dim3(blocks(rows)), dim3(PJ_BLOCK), 0, (hipStream_t)stream, rows,
                     (const bf16*)x, (const bf16*)nullptr, x_ld, (const uint4*)wpk, bias, (const bf16*)nullptr,
                     (bf16*)out, out_ld);
  return status();
}

int agn_proj_backward(int rows, const void* dps, const void* dpd, int dp_ld, const void* wtpk, void* dx, int dx_ld,
                      void* stream) {
  if (rows < 0 || !dps || !dpd || !wtpk || !dx || dp_ld % 8 || dx_ld % 8 || dx_ld < H || !al16(dps) || !al16(dpd) ||
      !al16(dx) || !al16(wtpk))
    return AGN_E_ARG;
  if (rows == 0) return 0;
  hipLaunchKernelGGL((proj_kernel<2, 1>), dim3(blocks(rows)), dim3(PJ_BLOCK), 0, (hipStream_t)stream, rows,
                     (const bf16*)dps, (const bf16*)dpd, dp_ld, (const uint4*)wtpk, (const float*)nullptr,
                     (const bf16*)dx, (bf16*)dx, dx_ld);
  return status();
}

}  // extern "C"
