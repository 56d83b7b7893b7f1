// Forward of an encoder MLP on narrow input rows (gfx950, bf16, H = 128): the node and edge
// encoders of the model (mlp.py MLP on d_n = 6 / d_e = 4 features, models/bsms_mgn.py encoders),
//   y = LN(W_{L-1} relu( ... relu(W0 x + b0) ... ) + b_{L-1}),   x: k <= 16 features, PLAIN or GATHER,
// bitwise agn_mlp_forward's general kernel in its narrow-input mode (mlp.hip mlp_fwd_kernel, M_NIN:
// the same single k-step for layer 0, the same MFMA sequence per accumulator after it, the same
// LayerNorm), training saves included. agn_mlp_forward routes such calls here (enc32_fwd_try)
// unless AGN_OPT_RESIDENT is 0.
//
// Why: the general kernel restages the three weight images into LDS for every 128-row block,
// which on a 6M-row edge encoder costs more than the rows' own traffic (8 B in, 256 B out). Here
// they stay resident (4 + 32 (L - 1) KB) and 16 waves per CU stream 32-row tiles.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4;
constexpr int NR = 64;
constexpr int NU = 8;
constexpr int LW0 = NT * 64;          // W0: one k-step unit per output tile (K <= 16)
constexpr int LW = NT * NU * 64;      // W1 .. W_{L-1}
constexpr int NW = 16;
constexpr int PF = 2;

template <int NLIN> struct Smem {
  uint4 w0[LW0];
  uint4 w[NLIN - 1][LW];
  float pv[NLIN + 2][H];  // b0 .. b_{NLIN-1}, LN gamma, LN beta
};
static_assert(sizeof(Smem<4>) <= 160 * 1024, "LDS budget");

AGN_DEV void gemm_k8(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int lane) {
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

struct Walk {
  int first, end, step;
  AGN_DEV Walk(int ntiles, int w, int nw = NW) {
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

// SAVES: relu outputs act[l] (+ AGN_RELU_MASK bits), hpre, stats, as the general kernel writes them
template <int NLIN, bool SAVES>
__global__ __launch_bounds__(64 * NW) void enc32_fwd_kernel(const agn_mlp_fwd_args a) {
  constexpr int NTHR = 64 * NW;
  __shared__ Smem<NLIN> sm;
  {
    const uint4* w0 = reinterpret_cast<const uint4*>(a.wpk[0]);
    for (int i = threadIdx.x; i < LW0; i += NTHR) sm.w0[i] = w0[i];
    for (int l = 1; l < NLIN; ++l) {
      const uint4* wl = reinterpret_cast<const uint4*>(a.wpk[l]);
      for (int i = threadIdx.x; i < LW; i += NTHR) sm.w[l - 1][i] = wl[i];
    }
    for (int i = threadIdx.x; i < (NLIN + 2) * H; i += NTHR) {
      const int l = i / H, f = i - l * H;
      const float* p = l < NLIN ? a.bias[l] : (l == NLIN ? a.ln_g : a.ln_b);
      sm.pv[l][f] = p ? p[f] : 0.f;
    }
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 31) / 32;
  const Walk walk(ntiles, w);
  const agn_seg& sx = a.seg[0];
  const bf16* X = reinterpret_cast<const bf16*>(sx.ptr);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const int src = sx.kind == AGN_SEG_GATHER ? sx.index[rr] : rr;
    BOp<bf16, NR> b;
    {
      // the row's k <= 16 features (mlp.hip load_row_narrow: registers 4q..4q+3 = features
      // 8q + 4h .. +3, q < 2; the rest zero)
      float v[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) v[i] = 0.f;
      const bf16* rowp = X + (size_t)src * sx.ld;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 x = load4_masked(rowp, 8 * q + 4 * h, sx.k, false);
        v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
      }
      b.set(v);
    }
    f32x16 acc[NT];
#pragma unroll
    for (int q = 0; q < 4 * NT; ++q) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(&sm.pv[0][8 * q + 4 * h]);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
    }
#pragma unroll
    for (int ot = 0; ot < NT; ++ot) b.mfma(acc[ot], sm.w0[ot * 64 + lane], 0);
#pragma unroll
    for (int l = 1; l < NLIN; ++l) {
      cbarrier();
      b.template set_relu<NT>(acc);
      if constexpr (SAVES) {
        if (a.act[l - 1]) {
          if (a.tiled) b.store_tiled(reinterpret_cast<bf16*>(a.act[l - 1]), row, h, valid);
          else b.store(reinterpret_cast<bf16*>(a.act[l - 1]) + (size_t)row * H, h, valid);
        }
        if (a.mask[l - 1]) store_relu_mask<bf16, NR>(a.mask[l - 1], b, tile, lane);
      }
#pragma unroll
      for (int q = 0; q < 4 * NT; ++q) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sm.pv[l][8 * q + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
      }
      gemm_k8(acc, b, sm.w[l - 1], lane);
    }
    cbarrier();
    if constexpr (SAVES) {
      if (a.hpre) {
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
          if (a.tiled) store8_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.hpre), i, row, h, v, valid);
          else store8_w(reinterpret_cast<bf16*>(a.hpre) + (size_t)row * H, i, h, v, valid);
        }
      }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) s += acc[i / 16][i % 16];
    s = sum32(s);
    const float mean = s / (float)H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NR; i += 2) q = ln_sq_acc2(q, acc[i / 16][i % 16], acc[(i + 1) / 16][(i + 1) % 16], mean);
    q = sum32(q);
    const float rstd = 1.0f / sqrtf(q / (float)H + 1e-5f);
    if constexpr (SAVES) {
      if (a.stats && valid && h == 0) {
        a.stats[2 * (size_t)row] = mean;
        a.stats[2 * (size_t)row + 1] = rstd;
      }
    }
    bf16* op = reinterpret_cast<bf16*>(a.out) + (size_t)row * a.out_ld;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int f0 = 16 * i + 8 * jj + 4 * h;
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(&sm.pv[NLIN][f0]);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sm.pv[NLIN + 1][f0]);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 o = ln_out2(f2(v[4 * jj + e], v[4 * jj + e + 1]), mean, rstd, f2(g4[e], g4[e + 1]),
                                  f2(b4[e], b4[e + 1]));
          v[4 * jj + e] = o[0];
          v[4 * jj + e + 1] = o[1];
        }
      }
      store8_w(op, i, h, v, valid);
    }
  }
}

// The decoder (mlp.py MLP on H-wide rows to <= 32 outputs, no LayerNorm; models/bsms_mgn.py
// decoder), bitwise the general kernel's narrow-output mode (mlp.hip M_NOUT: the last Linear
// computes output tile 0 only, its bias masked to out_dim), training saves included: weights
// resident, 16 waves per CU (12 with the saves, which spill at 128 registers).
template <int NLIN> struct DecSmem {
  uint4 w[NLIN][LW];      // the last image holds output tile 0 only (its first NU * 64 units)
  float pv[NLIN][H];
};
static_assert(sizeof(DecSmem<4>) <= 160 * 1024, "LDS budget");

// DNW waves per CU: 16 (<= 128 registers) at inference, 12 (<= 168) with the training saves
template <int NLIN, bool SAVES, int DNW>
__global__ __launch_bounds__(64 * DNW) void dec32_fwd_kernel(const agn_mlp_fwd_args a) {
  constexpr int NTHR = 64 * DNW;
  __shared__ DecSmem<NLIN> sm;
  for (int l = 0; l < NLIN; ++l) {
    const uint4* wl = reinterpret_cast<const uint4*>(a.wpk[l]);
    const int n = l < NLIN - 1 ? LW : NU * 64;
    for (int i = threadIdx.x; i < n; i += NTHR) sm.w[l][i] = wl[i];
  }
  for (int i = threadIdx.x; i < NLIN * H; i += NTHR) {
    const int l = i / H, f = i - l * H;
    sm.pv[l][f] = (a.bias[l] && (l < NLIN - 1 || f < a.out_dim)) ? a.bias[l][f] : 0.f;
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 31) / 32;
  const Walk walk(ntiles, w, DNW);
  const agn_seg& sx = a.seg[0];
  const bf16* X = reinterpret_cast<const bf16*>(sx.ptr);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    BOp<bf16, NR> b;
    b.load_w(X + (size_t)rr * sx.ld, h);
    f32x16 acc[NT];
#pragma unroll
    for (int q = 0; q < 4 * NT; ++q) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(&sm.pv[0][8 * q + 4 * h]);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
    }
    gemm_k8(acc, b, sm.w[0], lane);
#pragma unroll
    for (int l = 1; l < NLIN; ++l) {
      cbarrier();
      b.template set_relu<NT>(acc);
      if constexpr (SAVES) {
        if (a.act[l - 1]) {
          if (a.tiled) b.store_tiled(reinterpret_cast<bf16*>(a.act[l - 1]), row, h, valid);
          else b.store(reinterpret_cast<bf16*>(a.act[l - 1]) + (size_t)row * H, h, valid);
        }
        if (a.mask[l - 1]) store_relu_mask<bf16, NR>(a.mask[l - 1], b, tile, lane);
      }
#pragma unroll
      for (int q = 0; q < 4 * NT; ++q) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&sm.pv[l][8 * q + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
      }
      if (l < NLIN - 1) {
        gemm_k8(acc, b, sm.w[l], lane);
      } else {  // output tile 0 only, k-steps in order
#pragma unroll
        for (int u = 0; u < NU; ++u) b.mfma(acc[0], sm.w[l][u * 64 + lane], u);
      }
    }
    bf16* op = reinterpret_cast<bf16*>(a.out) + (size_t)row * a.out_ld;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = {acc[0][4 * q], acc[0][4 * q + 1], acc[0][4 * q + 2], acc[0][4 * q + 3]};
      if (valid) store4_masked(op, 8 * q + 4 * h, a.out_dim, false, v);
    }
  }
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

long g_launches = 0;
long g_dec_launches = 0;

}  // namespace

extern "C" long agn_debug_enc32_launches(void) { return g_launches; }
extern "C" long agn_debug_dec32_launches(void) { return g_dec_launches; }

namespace agn {
// agn_mlp_forward (mlp.hip) hands over the narrow-input encoder MLPs this kernel covers: returns
// false (nothing launched) otherwise; *rc = the launch status
bool enc32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc) {
  if (a->dtype != AGN_BF16 || a->hidden != H || (a->nlin != 3 && a->nlin != 4) || a->nseg != 1 || a->out_dim != H ||
      !a->use_ln || a->act_fn != AGN_ACT_RELU || a->proj || a->resid || a->rows < 64 * 1024)
    return false;
  const agn_seg& sx = a->seg[0];
  if ((sx.kind != AGN_SEG_PLAIN && sx.kind != AGN_SEG_GATHER) || sx.k < 1 || sx.k > 16 || !sx.ptr) return false;
  if (sx.kind == AGN_SEG_GATHER && !sx.index) return false;
  if (a->out_ld % 8 || !al16(a->out)) return false;
  bool saves = a->hpre || a->stats;
  for (int l = 0; l < AGN_MAX_LIN; ++l) {
    if (a->pre[l] || (l >= a->nlin - 1 && (a->act[l] || a->mask[l]))) return false;
    saves = saves || a->act[l] || a->mask[l];
    if (!al16(a->act[l])) return false;
  }
  if (!al16(a->hpre)) return false;
  for (int l = 0; l < a->nlin; ++l)
    if (!a->wpk[l] || !al16(a->wpk[l])) return false;
  const int tiles = (a->rows + 31) / 32;
  const int need = (tiles + NW - 1) / NW;
  const int cus = cu_count();
  const int nblk = need >= cus ? cus : ((need + 7) / 8 * 8 < 8 ? 8 : (need + 7) / 8 * 8);
  const dim3 g(nblk), blk(64 * NW);
  hipStream_t st = (hipStream_t)stream;
  if (a->nlin == 4) {
    if (saves) hipLaunchKernelGGL((enc32_fwd_kernel<4, true>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((enc32_fwd_kernel<4, false>), g, blk, 0, st, *a);
  } else {
    if (saves) hipLaunchKernelGGL((enc32_fwd_kernel<3, true>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((enc32_fwd_kernel<3, false>), g, blk, 0, st, *a);
  }
  ++g_launches;
  const hipError_t e = hipGetLastError();
  *rc = e == hipSuccess ? 0 : (int)e;
  return true;
}
// the decoder: agn_mlp_forward's narrow-output calls (M_NOUT) this kernel covers
bool dec32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc) {
  if (a->dtype != AGN_BF16 || a->hidden != H || (a->nlin != 3 && a->nlin != 4) || a->nseg != 1 || a->out_dim > 32 ||
      a->out_dim < 1 || a->use_ln || a->act_fn != AGN_ACT_RELU || a->proj || a->resid || a->rows < 64 * 1024)
    return false;
  const agn_seg& sx = a->seg[0];
  if (sx.kind != AGN_SEG_PLAIN || sx.k != H || sx.ld % 8 || !sx.ptr || !al16(sx.ptr)) return false;
  // training saves: relu outputs and their mask bits (no LayerNorm here, so no hpre / stats)
  bool saves = false;
  for (int l = 0; l < AGN_MAX_LIN; ++l) {
    if (a->pre[l] || (l >= a->nlin - 1 && (a->act[l] || a->mask[l]))) return false;
    saves = saves || a->act[l] || a->mask[l];
    if (!al16(a->act[l])) return false;
  }
  if (a->hpre || a->stats) return false;
  for (int l = 0; l < a->nlin; ++l)
    if (!a->wpk[l] || !al16(a->wpk[l])) return false;
  const int dnw = saves ? 12 : 16;
  const int tiles = (a->rows + 31) / 32;
  const int need = (tiles + dnw - 1) / dnw;
  const int cus = cu_count();
  const int nblk = need >= cus ? cus : ((need + 7) / 8 * 8 < 8 ? 8 : (need + 7) / 8 * 8);
  const dim3 g(nblk);
  hipStream_t st = (hipStream_t)stream;
  if (saves) {
    if (a->nlin == 4) hipLaunchKernelGGL((dec32_fwd_kernel<4, true, 12>), g, dim3(64 * 12), 0, st, *a);
    else hipLaunchKernelGGL((dec32_fwd_kernel<3, true, 12>), g, dim3(64 * 12), 0, st, *a);
  } else {
    if (a->nlin == 4) hipLaunchKernelGGL((dec32_fwd_kernel<4, false, 16>), g, dim3(64 * 16), 0, st, *a);
    else hipLaunchKernelGGL((dec32_fwd_kernel<3, false, 16>), g, dim3(64 * 16), 0, st, *a);
  }
  ++g_dec_launches;
  const hipError_t e = hipGetLastError();
  *rc = e == hipSuccess ? 0 : (int)e;
  return true;
}
}  // namespace agn
