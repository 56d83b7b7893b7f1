// Forward of the sum-trick edge MLP on 16-row tiles (gfx950, bf16, H = 128):
//   e' = e + LN(W3 relu(W2 relu(W1 relu(e W_e^T + P_s[src] + P_d[dst]) + b1) + b2) + b3)
// (models/mgnLayer.py:72-105 EdgeBlockSum, residual :205). The chain's operands and the MFMA
// k-order are those of edge16.hpp, shared with the fused backward (edge16_bwd.hip), which
// recomputes this kernel's h0..h3 bitwise.
//
// Persistent: one workgroup per CU, all four weight images resident in LDS (128 KB). Each wave
// streams tiles of 16 NH edges (NH 16-row halves: every weight fragment read from LDS feeds NH
// MFMAs) in CSC order over an XCD-grouped walk; a tile's node ids are loaded one tile ahead and handed over through
// the wave's LDS slot (a loop-carried load result would make the compiler wait vmcnt(0) at the
// loop head, i.e. for the previous tile's stores too).
#include "edge16.hpp"
#include "aerognn.h"

using namespace agn;
using namespace agn::e16;

namespace {

// Variants: NH 16-row halves per wave (a 16 NH-row tile; gemm_fwd_n shares each weight fragment
// read among the halves), NW waves per CU. NH = 1, NW = 16: four waves per SIMD at <= 128
// registers; NH = 2: half the LDS reads per row, at NW = 12 (three per SIMD, <= 168 registers,
// the residual operand kept) or NW = 16 (<= 128, the residual re-read from L2 in the epilogue).
// agn_set_option(AGN_OPT_EDGE_FWD_HALVES / _WAVES) selects one.
int g_fwd_nh = 2;
int g_fwd_nw = 12;  // waves per CU for NH = 2

constexpr int OFF_PV = 4 * IMG_B;                 // fp32 [5][H]: b1, b2, b3, LN gamma, LN beta
constexpr int OFF_IDS = OFF_PV + 5 * H * 4;       // int [NW][2 * 16 NH]: next tile's src / dst
template <int NH, int NW> constexpr int lds_bytes() { return OFF_IDS + NW * 2 * 16 * NH * 4; }
static_assert(lds_bytes<1, 16>() <= 160 * 1024 && lds_bytes<2, 16>() <= 160 * 1024, "LDS budget");

template <int NH, int NW>
__global__ __launch_bounds__(64 * NW) void edge16_fwd_kernel(const agn_edge_fwd_args a) {
  constexpr int NTHR = 64 * NW;
  constexpr bool KEEP_E = NH == 1 || NW < 16;  // the residual operand kept from the first GEMM
  constexpr int TR = 16 * NH;  // rows per tile
  __shared__ __attribute__((aligned(16))) char lds[lds_bytes<NH, NW>()];
  load_images(lds, a.wpk, threadIdx.x, NTHR);
  float* pv = reinterpret_cast<float*>(lds + OFF_PV);
  for (int i = threadIdx.x; i < 5 * H; i += NTHR) {
    const int l = i / H, f = i - l * H;
    pv[i] = l < 3 ? (a.bias[l + 1] ? a.bias[l + 1][f] : 0.f) : (l == 3 ? a.ln_g[f] : a.ln_b[f]);
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + TR - 1) / TR;
  const Walk walk(ntiles, w, NW);
  int* ids = reinterpret_cast<int*>(lds + OFF_IDS) + w * 2 * TR;
  const int32_t* const srcp = a.src;
  const int32_t* const dstp = a.dst;
  // lane l < 2 TR loads the src (l < TR) or dst of tile row l % TR; other lanes repeat a row
  auto tile_id = [&](int t) {
    const int rr = min(t * TR + lane0 % TR, a.rows - 1);
    return ((lane0 / TR) & 1 ? dstp : srcp)[rr];
  };
  if (walk.first < walk.end && lane0 < 2 * TR) ids[lane0] = tile_id(walk.first);
  const bf16* P = reinterpret_cast<const bf16*>(a.proj);
  const bf16* E = reinterpret_cast<const bf16*>(a.e);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = fresh(lane0);
    const int r = lane & 15, g = lane >> 4;
    const bool more = tile + walk.step < walk.end;
    const int nid = tile_id(more ? tile + walk.step : tile);
    int row[NH];
    bool valid[NH];
    f32x4 acc[NH][8];
    Op x[NH], e0[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      row[h] = tile * TR + 16 * h + r;
      valid[h] = row[h] < a.rows;
      const int rr = valid[h] ? row[h] : a.rows - 1;
      const int sid = ids[16 * h + r], did = ids[TR + 16 * h + r];
      uint4 xs[4], xd[4];
      load_raw(xs, P + (size_t)sid * (2 * H), lane);
      load_raw(xd, P + (size_t)did * (2 * H) + H, lane);
      load_op(e0[h], E + (size_t)rr * H, lane);
      acc_sum2(acc[h], xs, xd);
    }
    if (lane < 2 * TR && more) ids[lane] = nid;  // (this tile's reads of the slot are done: LDS is in order per wave)
    gemm_fwd_n<NH>(acc, e0, lds, 0 * IMG_B, fresh(lane));
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      cbarrier();
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        relu_op(x[h], acc[h]);
        if (a.act[l - 1]) store_op(reinterpret_cast<bf16*>(a.act[l - 1]) + (size_t)row[h] * H, x[h], lane, valid[h]);
        bias_init(acc[h], pv + (l - 1) * H, lane);
      }
      gemm_fwd_n<NH>(acc, x, lds, l * IMG_B, fresh(lane));
    }
    cbarrier();
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float mean, rstd;
      ln_stats(acc[h], mean, rstd);
      if (a.hpre) {
        Op hp;
        pack_op(hp, acc[h]);
        store_op(reinterpret_cast<bf16*>(a.hpre) + (size_t)row[h] * H, hp, lane, valid[h]);
      }
      if (a.stats && valid[h] && g == 0) {
        a.stats[2 * (size_t)row[h]] = mean;
        a.stats[2 * (size_t)row[h] + 1] = rstd;
      }
      // e' = e + round(gamma * xhat + beta), rounded again (the bf16 module's two roundings); the
      // residual is the kept operand, or (KEEP_E false: registers for a fourth wave per SIMD) e's
      // row read again here (an L2 hit: the tile's first GEMM read it)
      uint4 er[4];
      if (!KEEP_E) load_raw(er, E + (size_t)(valid[h] ? row[h] : a.rows - 1) * H, lane);
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
            const f32x2 v = ln_out2(f2(acc[h][ob][e], acc[h][ob][e + 1]), mean, rstd, f2(g4[e], g4[e + 1]),
                                    f2(b4[e], b4[e + 1]));
            const uint32_t p = pack2(v[0], v[1]);
            const f32x2 y = f2(lo_bf16(p), hi_bf16(p)) + (KEEP_E ? f2(op_el(e0[h], ob, e), op_el(e0[h], ob, e + 1))
                                                                 : f2(raw_el(er, ob, e), raw_el(er, ob, e + 1)));
            wv[2 * hb + e / 2] = pack2(y[0], y[1]);
          }
        }
        o[s] = __builtin_bit_cast(uint4, u32x4{wv[0], wv[1], wv[2], wv[3]});
      }
      store_raw(reinterpret_cast<bf16*>(a.out) + (size_t)row[h] * H, o, lane, valid[h]);
    }
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

namespace agn {
// agn_set_option(AGN_OPT_EDGE_FWD_HALVES) (mlp.hip)
int edge16_fwd_set_halves(int nh) {
  const int old = g_fwd_nh;
  if (nh != 1 && nh != 2) return AGN_E_ARG;
  g_fwd_nh = nh;
  return old;
}
// agn_set_option(AGN_OPT_EDGE_FWD_WAVES): waves per CU of the two-halves variant
int edge16_fwd_set_waves(int nw) {
  const int old = g_fwd_nw;
  if (nw != 12 && nw != 16) return AGN_E_ARG;
  g_fwd_nw = nw;
  return old;
}
}  // namespace agn

extern "C" {

int agn_edge_fwd_blocks(int rows) {
  const int cus = cu_count();
  const int nw = g_fwd_nh == 1 ? 16 : g_fwd_nw;
  const int waves = (rows + 16 * g_fwd_nh - 1) / (16 * g_fwd_nh);
  const int need = (waves + nw - 1) / nw;
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
  if (g_fwd_nh == 1)
    hipLaunchKernelGGL((edge16_fwd_kernel<1, 16>), dim3(a->nblk), dim3(64 * 16), 0, (hipStream_t)stream, *a);
  else if (g_fwd_nw == 16)
    hipLaunchKernelGGL((edge16_fwd_kernel<2, 16>), dim3(a->nblk), dim3(64 * 16), 0, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL((edge16_fwd_kernel<2, 12>), dim3(a->nblk), dim3(64 * 12), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
