// Forward of the sum-trick edge MLP on 16-row tiles (gfx950, bf16, H = 128):
//   e' = e + LN(W3 relu(W2 relu(W1 relu(e W_e^T + P_s[src] + P_d[dst]) + b1) + b2) + b3)
// (models/mgnLayer.py:72-105 EdgeBlockSum, residual :205). The chain's operands and the MFMA
// k-order are those of edge16.hpp, shared with the fused backward (edge16_bwd.hip), which
// recomputes this kernel's h0..h3 bitwise.
//
// Persistent: one 1024-thread workgroup per CU, 16 waves (four per SIMD, <= 128 registers each),
// all four weight images resident in LDS (128 KB). Each wave streams 16-edge tiles in CSC order
// over an XCD-grouped walk; a tile's node ids are loaded one tile ahead and handed over through
// the wave's LDS slot (a loop-carried load result would make the compiler wait vmcnt(0) at the
// loop head, i.e. for the previous tile's stores too).
#include "edge16.hpp"
#include "aerognn.h"

using namespace agn;
using namespace agn::e16;

namespace {

constexpr int NW = 16;
constexpr int NTHR = 64 * NW;
constexpr int OFF_PV = 4 * IMG_B;                 // fp32 [5][H]: b1, b2, b3, LN gamma, LN beta
constexpr int OFF_IDS = OFF_PV + 5 * H * 4;       // int [NW][32]: next tile's src (0-15) / dst (16-31)
constexpr int LDS_B = OFF_IDS + NW * 32 * 4;
static_assert(LDS_B <= 160 * 1024, "LDS budget");

__global__ __launch_bounds__(NTHR) void edge16_fwd_kernel(const agn_edge_fwd_args a) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_B];
  load_images(lds, a.wpk, threadIdx.x, NTHR);
  float* pv = reinterpret_cast<float*>(lds + OFF_PV);
  for (int i = threadIdx.x; i < 5 * H; i += NTHR) {
    const int l = i / H, f = i - l * H;
    pv[i] = l < 3 ? (a.bias[l + 1] ? a.bias[l + 1][f] : 0.f) : (l == 3 ? a.ln_g[f] : a.ln_b[f]);
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 15) / 16;
  const Walk walk(ntiles, w, NW);
  int* ids = reinterpret_cast<int*>(lds + OFF_IDS) + w * 32;
  const int32_t* const srcp = a.src;
  const int32_t* const dstp = a.dst;
  // lane l < 32 loads the src (l < 16) or dst (16 <= l < 32) of row l & 15; lanes 32-63 repeat it
  auto tile_id = [&](int t) {
    const int rr = min(t * 16 + (lane0 & 15), a.rows - 1);
    return ((lane0 & 16) ? dstp : srcp)[rr];
  };
  if (walk.first < walk.end && lane0 < 32) ids[lane0] = tile_id(walk.first);
  const bf16* P = reinterpret_cast<const bf16*>(a.proj);
  const bf16* E = reinterpret_cast<const bf16*>(a.e);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = fresh(lane0);
    const int r = lane & 15, g = lane >> 4;
    const int row = tile * 16 + r;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const bool more = tile + walk.step < walk.end;
    const int nid = tile_id(more ? tile + walk.step : tile);
    const int sid = ids[r], did = ids[16 + r];
    f32x4 acc[8];
    Op x, e0;
    {
      uint4 xs[4], xd[4];
      load_raw(xs, P + (size_t)sid * (2 * H), lane);
      load_raw(xd, P + (size_t)did * (2 * H) + H, lane);
      load_op(e0, E + (size_t)rr * H, lane);
      acc_sum2(acc, xs, xd);
    }
    if (lane < 32 && more) ids[lane] = nid;  // (this tile's reads of the slot are done: LDS is in order per wave)
    gemm_fwd(acc, e0, lds, 0 * IMG_B, fresh(lane));
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      cbarrier();
      relu_op(x, acc);
      if (a.act[l - 1]) store_op(reinterpret_cast<bf16*>(a.act[l - 1]) + (size_t)row * H, x, lane, valid);
      bias_init(acc, pv + (l - 1) * H, lane);
      gemm_fwd(acc, x, lds, l * IMG_B, fresh(lane));
    }
    cbarrier();
    float mean, rstd;
    ln_stats(acc, mean, rstd);
    if (a.hpre) {
      Op hp;
      pack_op(hp, acc);
      store_op(reinterpret_cast<bf16*>(a.hpre) + (size_t)row * H, hp, lane, valid);
    }
    if (a.stats && valid && g == 0) {
      a.stats[2 * (size_t)row] = mean;
      a.stats[2 * (size_t)row + 1] = rstd;
    }
    // e' = e + round(gamma * xhat + beta), rounded again (the bf16 module's two roundings)
    const float* gm = pv + 3 * H;
    const float* bt = pv + 4 * H;
    uint4 o[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint32_t wv[4];
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        const int ob = 2 * s + hb;
        const int f0 = 32 * s + 8 * g + 4 * hb;
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(gm + f0);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bt + f0);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 v = ln_out2(f2(acc[ob][e], acc[ob][e + 1]), mean, rstd, f2(g4[e], g4[e + 1]), f2(b4[e], b4[e + 1]));
          const uint32_t p = pack2(v[0], v[1]);
          const f32x2 y = f2(lo_bf16(p), hi_bf16(p)) + f2(op_el(e0, ob, e), op_el(e0, ob, e + 1));
          wv[2 * hb + e / 2] = pack2(y[0], y[1]);
        }
      }
      o[s] = __builtin_bit_cast(uint4, u32x4{wv[0], wv[1], wv[2], wv[3]});
    }
    store_raw(reinterpret_cast<bf16*>(a.out) + (size_t)row * H, o, lane, valid);
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

int agn_edge_fwd_blocks(int rows) {
  const int cus = cu_count();
  const int waves = (rows + 15) / 16;
  const int need = (waves + NW - 1) / NW;
  if (need >= cus) return cus;
  const int n = (need + 7) / 8 * 8;
  return n < 8 ? 8 : n;
}

int agn_edge_forward(const agn_edge_fwd_args* a, void* stream) {
  if (!a || a->rows < 0 || a->nblk < 1) return AGN_E_ARG;
  if (a->rows == 0) return 0;
  if (!a->e || !a->proj || !a->src || !a->dst || !a->out || !a->ln_g || !a->ln_b) return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wpk[l] || !al16(a->wpk[l])) return AGN_E_ARG;
  if (!al16(a->e) || !al16(a->proj) || !al16(a->out)) return AGN_E_ARG;
  for (int l = 0; l < 3; ++l)
    if (!al16(a->act[l])) return AGN_E_ARG;
  if (!al16(a->hpre)) return AGN_E_ARG;
  hipLaunchKernelGGL(edge16_fwd_kernel, dim3(a->nblk), dim3(NTHR), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
