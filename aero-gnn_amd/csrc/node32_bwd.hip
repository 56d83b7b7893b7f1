// Backward of a processor layer's node MLP (gfx950, bf16, H = 128, four Linears, LayerNorm,
// residual; mgnLayer.py NodeBlock and :205 under autograd): given g = dL/dx' and the forward's
// saves (pre-LN rows, LN statistics, ReLU mask bits), writes the pre-activation gradients G_3..G_0
// (for agn_wgrad), the LayerNorm parameter partials, dx = W0x^T G_0 + g and dagg = W0a^T G_0.
// Bitwise agn_mlp_backward's general kernel on the same operands (mlp.hip mlp_bwd_kernel, M_VEC:
// the same LayerNorm backward steps and butterflies, the same MFMA sequence per accumulator, the
// same per-128-row-block LayerNorm partial sums); agn_mlp_backward routes such calls here
// (node32_bwd_try) unless AGN_OPT_RESIDENT is 0.
//
// Why: the general kernel restages every layer's weights (160 KB per chain) into LDS for each
// 128-row block. Here W0^T (256 x 128), W3^T and W2^T stay resident (128 KB; W1^T streams from
// L2) and 8 waves per CU stream 32-row tiles. The LayerNorm partials of a tile go to a workspace
// and a second launch sums each 128-row block's four tiles in the general kernel's order.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4;
constexpr int NR = 64;
constexpr int NP = NR / 32;
constexpr int NU = 8;
constexpr int LW = NT * NU * 64;       // a 128 x 128 image (units)
constexpr int NW = 8;
constexpr int PF = 2;
constexpr int PFG = 4;
constexpr int ROWS_PER_BLOCK = 128;    // the general kernel's block (its LayerNorm partial rows)

struct Smem {
  uint4 w0t[2 * LW];   // W0^T: 256 outputs (dx | dagg) x 128
  uint4 w3t[LW];
  uint4 w2t[LW];
  float gam[H];
};
static_assert(sizeof(Smem) <= 160 * 1024, "LDS budget");

// acc[ot] += A[ot0 + ot, k-steps 0..7] . b (ot0 in output tiles of the image), k-steps in order
AGN_DEV void gemm_l(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int ot0, int lane) {
  uint4 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = w[((ot0 + i % NT) * NU + i / NT) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < NT * NU; ++idx) {
    const uint4 cur = f[idx % PF];
    const int nx = idx + PF;
    if (nx < NT * NU) f[idx % PF] = w[((ot0 + nx % NT) * NU + nx / NT) * 64 + lane];
    b.mfma(acc[idx % NT], cur, idx / NT);
  }
}
AGN_DEV void gemm_g(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int lane) {
  uint4 f[PFG];
#pragma unroll
  for (int i = 0; i < PFG; ++i) f[i] = w[((i % NT) * NU + i / NT) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < NT * NU; ++idx) {
    const uint4 cur = f[idx % PFG];
    const int nx = idx + PFG;
    if (nx < NT * NU) f[idx % PFG] = w[((nx % NT) * NU + nx / NT) * 64 + lane];
    b.mfma(acc[idx % NT], cur, idx / NT);
  }
}

struct Walk {
  int first, end, step;
  AGN_DEV Walk(int ntiles, int w) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int g = blockIdx.x & 7, bi = blockIdx.x >> 3, nb = gridDim.x >> 3;
      const int per = (ntiles + 7) / 8;
      first = g * per + bi * NW + w;
      end = min(ntiles, (g + 1) * per);
      step = nb * NW;
    } else {
      first = blockIdx.x * NW + w;
      end = ntiles;
      step = gridDim.x * NW;
    }
  }
};

// the general kernel's load_grad (M_VEC, no g2): the row of g, zero for rows past the end
AGN_DEV void load_g(float (&A)[NR], const bf16* g, int rr, bool valid, int h) {
  load_row_w<bf16, NR>(A, g + (size_t)rr * H, h);
  if (!valid) {
#pragma unroll
    for (int i = 0; i < NR; ++i) A[i] = 0.f;
  }
}

__global__ __launch_bounds__(64 * NW) void node32_bwd_kernel(const agn_mlp_bwd_args a, float* lnt) {
  constexpr int NTHR = 64 * NW;
  __shared__ Smem sm;
  {
    const uint4* w0 = reinterpret_cast<const uint4*>(a.wtpk[0]);
    const uint4* w3 = reinterpret_cast<const uint4*>(a.wtpk[3]);
    const uint4* w2 = reinterpret_cast<const uint4*>(a.wtpk[2]);
    for (int i = threadIdx.x; i < 2 * LW; i += NTHR) sm.w0t[i] = w0[i];
    for (int i = threadIdx.x; i < LW; i += NTHR) {
      sm.w3t[i] = w3[i];
      sm.w2t[i] = w2[i];
    }
    for (int i = threadIdx.x; i < H; i += NTHR) sm.gam[i] = a.ln_g[i];
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 31) / 32;
  const Walk walk(ntiles, w);
  const bf16* G = reinterpret_cast<const bf16*>(a.g);
  const bf16* HP = reinterpret_cast<const bf16*>(a.hpre);
  const uint4* w1g = reinterpret_cast<const uint4*>(a.wtpk[1]);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    float A[NR];
    load_g(A, G, rr, valid, h);
    // every layer's ReLU mask bits, loaded before the tile's first store (vmcnt retires in order:
    // a load issued after the gpre stores would wait for them)
    uint32_t mks[3][mask_dwords<NR>()];
#pragma unroll
    for (int l = 0; l < 3; ++l) load_relu_mask<NR>(mks[l], a.mask[l], tile, lane);
    {
      // ---- LayerNorm backward (mlp_bwd_kernel: hpre and gamma read per 4-feature chunk, twice)
      const float mean = a.stats[2 * (size_t)rr], rstd = a.stats[2 * (size_t)rr + 1];
      float B[NR];
      float c1 = 0.f, c2 = 0.f;
#pragma unroll
      for (int q = 0; q < NR / 4; ++q) {
        const int f0 = 8 * q + 4 * h;
        const f32x4 hv = a.tiled ? load4_tiled<bf16, NR>(HP, q, rr, h) : load4(HP + (size_t)rr * H + f0);
        const f32x4 gm = *reinterpret_cast<const f32x4*>(&sm.gam[f0]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (hv[e] - mean) * rstd;
          ln_bwd_acc(c1, c2, A[4 * q + e], gm[e], xh);
          B[4 * q + e] = A[4 * q + e] * xh;
        }
      }
      c1 = sum32(c1);
      c2 = sum32(c2);
      c1 /= (float)H;
      c2 /= (float)H;
      if (a.ln_partial) {  // this tile's LayerNorm parameter partials (butterflies over its 32 rows)
        butterfly_reduce<NR>(B, lane);
        float pg[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) pg[i] = B[i];
#pragma unroll
        for (int i = 0; i < NR; ++i) B[i] = A[i];
        butterfly_reduce<NR>(B, lane);
        float* lp = lnt + (size_t)tile * 2 * H;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int f = feat_of((c * NR) / 32 + i, h);
          lp[f] = pg[i];
          lp[H + f] = B[i];
        }
      }
#pragma unroll
      for (int q = 0; q < NR / 4; ++q) {
        const int f0 = 8 * q + 4 * h;
        const f32x4 hv = a.tiled ? load4_tiled<bf16, NR>(HP, q, rr, h) : load4(HP + (size_t)rr * H + f0);
        const f32x4 gm = *reinterpret_cast<const f32x4*>(&sm.gam[f0]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (hv[e] - mean) * rstd;
          A[4 * q + e] = ln_bwd_out(A[4 * q + e], gm[e], c1, c2, xh, rstd);
        }
      }
    }
    // ---- chain rule through the Linear / ReLU stack
    f32x16 acc[NT];
    BOp<bf16, NR> b;
#pragma unroll
    for (int l = 3; l >= 1; --l) {
      cbarrier();
      if (a.gpre[l]) {
        if ((a.gpre_tiled >> l) & 1) store_row_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[l]), A, row, h, valid);
        else store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[l]) + (size_t)row * H, A, h, valid);
      }
      b.set(A);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
      if (l == 1) gemm_g(acc, b, w1g, lane);
      else gemm_l(acc, b, l == 3 ? sm.w3t : sm.w2t, 0, lane);
      cbarrier();
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) A[16 * t + r] = acc[t][r];
#pragma unroll
      for (int i = 0; i < NR; ++i) A[i] = mask_sel(mks[l - 1], i, A[i]);
    }
    if (a.gpre[0]) {
      if (a.gpre_tiled & 1) store_row_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[0]), A, row, h, valid);
      else store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[0]) + (size_t)row * H, A, h, valid);
    }
    b.set(A);
    // ---- dX: the x rows (+ the residual's g) and the aggregate's rows of W0^T
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!a.din[s]) continue;
      cbarrier();
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
      gemm_l(acc, b, sm.w0t, NT * s, lane);
      float v[NR];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[16 * t + r] = acc[t][r];
      if (a.din_resid[s]) {
        float gg[NR];
        load_g(gg, G, rr, valid, h);
#pragma unroll
        for (int i = 0; i < NR; ++i) v[i] += gg[i];
      }
      store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.din[s]) + (size_t)row * H, v, h, valid);
    }
  }
}

// ln_partial[b] = sum over the block's 4 tiles in order of their partials (the general kernel's
// per-block sum over its waves; tiles past the last one add 0)
__global__ __launch_bounds__(256) void node32_lnp_kernel(const float* __restrict__ lnt, int ntiles, int nblk,
                                                         float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nblk * 2 * H) return;
  const int b = i / (2 * H), f = i - b * (2 * H);
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < ROWS_PER_BLOCK / 32; ++w) {
    const int t = b * (ROWS_PER_BLOCK / 32) + w;
    s += t < ntiles ? lnt[(size_t)t * 2 * H + f] : 0.f;
  }
  out[i] = s;
}

// ------------------------------------------------------------------------- decoder backward
// The decoder MLP (H-wide rows -> out_dim <= 32 outputs, no LayerNorm, NLIN = 3 or 4 Linears;
// models/bsms_mgn.py decoder): bitwise mlp_bwd_kernel<bf16, 4, M_NOUT> on the same operands (the
// narrow g row loaded as its load_grad, the same MFMA sequence per accumulator, the same masked
// stores). Every W^T image stays resident (104 KB at most); 8 waves per CU stream 32-row tiles.
constexpr int LWL = NT * 2 * 64;  // the last layer's W^T: 4 output tiles x <= 2 k-units
struct DSmem {
  uint4 w0t[LW];
  uint4 wh[2][LW];
  uint4 wl[LWL];
};
static_assert(sizeof(DSmem) <= 160 * 1024, "LDS budget");

AGN_DEV void store_narrow(bf16* rowp, int k, const float (&v)[NR], int h, bool valid) {
  if (!valid) return;
#pragma unroll
  for (int q = 0; q < NR / 4; ++q)
    store4_masked(rowp, 8 * q + 4 * h, k, false, f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]});
}

template <int NLIN>
__global__ __launch_bounds__(64 * NW) void dec32_bwd_kernel(const agn_mlp_bwd_args a) {
  constexpr int NTHR = 64 * NW;
  __shared__ DSmem sm;
  const int M = a.out_dim;
  const int kul = (M + 15) / 16;
  {
    const uint4* w0 = reinterpret_cast<const uint4*>(a.wtpk[0]);
    for (int i = threadIdx.x; i < LW; i += NTHR) sm.w0t[i] = w0[i];
#pragma unroll
    for (int l = 1; l + 1 < NLIN; ++l) {
      const uint4* wg = reinterpret_cast<const uint4*>(a.wtpk[l]);
      for (int i = threadIdx.x; i < LW; i += NTHR) sm.wh[l - 1][i] = wg[i];
    }
    const uint4* wg = reinterpret_cast<const uint4*>(a.wtpk[NLIN - 1]);
    for (int i = threadIdx.x; i < NT * kul * 64; i += NTHR) sm.wl[i] = wg[i];
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = (a.rows + 31) / 32;
  const Walk walk(ntiles, w);
  const bf16* G = reinterpret_cast<const bf16*>(a.g);
  // a tile's loads (the narrow g row, every layer's ReLU mask bits) are issued one tile ahead,
  // before the current tile's stores: vmcnt retires in order, so a load issued after a tile's
  // gpre / dx stores would wait for those stores to complete
  constexpr int ND = mask_dwords<NR>();
  f32x4 pg[4];
  uint32_t pm[NLIN - 1][ND];
  auto prefetch = [&](int t) {
    const int c = lane0 & 31, h = lane0 >> 5;
    const int r = min(t * 32 + c, a.rows - 1);
    const bf16* g1 = G + (size_t)r * M;
#pragma unroll
    for (int q = 0; q < 4; ++q) pg[q] = load4_masked(g1, 8 * q + 4 * h, M, false);
#pragma unroll
    for (int l = 0; l + 1 < NLIN; ++l) load_relu_mask<NR>(pm[l], a.mask[l], t, lane0);
  };
  if (walk.first < walk.end) prefetch(walk.first);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    float A[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) A[i] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) A[4 * q + e] = valid ? pg[q][e] : 0.f;
    uint32_t mks[NLIN - 1][ND];
#pragma unroll
    for (int l = 0; l + 1 < NLIN; ++l)
#pragma unroll
      for (int d = 0; d < ND; ++d) mks[l][d] = pm[l][d];
    if (tile + walk.step < walk.end) prefetch(tile + walk.step);
    f32x16 acc[NT];
    BOp<bf16, NR> b;
    // ---- the last Linear (out_dim outputs): its G rows, then W^T over kul k-units
    if (a.gpre[NLIN - 1]) store_narrow(reinterpret_cast<bf16*>(a.gpre[NLIN - 1]) + (size_t)row * M, M, A, h, valid);
    b.set(A);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    for (int u = 0; u < kul; ++u)
#pragma unroll
      for (int ot = 0; ot < NT; ++ot) b.mfma(acc[ot], sm.wl[(ot * kul + u) * 64 + lane], u);
#pragma unroll
    for (int l = NLIN - 1; l >= 1; --l) {
      cbarrier();
      if (l < NLIN - 1) {  // a hidden Linear: H -> H
        if (a.gpre[l]) {
          if ((a.gpre_tiled >> l) & 1) store_row_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[l]), A, row, h, valid);
          else store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[l]) + (size_t)row * H, A, h, valid);
        }
        b.set(A);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
        gemm_l(acc, b, sm.wh[l - 1], 0, lane);
        cbarrier();
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) A[16 * t + r] = acc[t][r];
#pragma unroll
      for (int i = 0; i < NR; ++i) A[i] = mask_sel(mks[l - 1], i, A[i]);
    }
    if (a.gpre[0]) {
      if (a.gpre_tiled & 1) store_row_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[0]), A, row, h, valid);
      else store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.gpre[0]) + (size_t)row * H, A, h, valid);
    }
    if (a.din[0]) {
      b.set(A);
      cbarrier();
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
      gemm_l(acc, b, sm.w0t, 0, lane);
      float v[NR];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[16 * t + r] = acc[t][r];
      store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.din[0]) + (size_t)row * H, v, h, valid);
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

// per-tile LayerNorm partial workspace, grown on demand (device memory kept for the process)
// LayerNorm partial-row workspace, one per device (a process driving two devices must not
// share it); a call on another stream than the last user first waits for that stream, which may still
// be reading it
struct LnScratch {
  float* p = nullptr;
  size_t cap = 0;
  hipStream_t last = nullptr;
};
LnScratch g_lnt[64];
long g_launches = 0;
long g_dec_launches = 0;

int grid_for(int ntiles) {
  const int need_blocks = (ntiles + NW - 1) / NW;
  const int cus = cu_count();
  return need_blocks >= cus ? cus : ((need_blocks + 7) / 8 * 8 < 8 ? 8 : (need_blocks + 7) / 8 * 8);
}

}  // namespace

extern "C" long agn_debug_node32_bwd_launches(void) { return g_launches; }
extern "C" long agn_debug_dec32_bwd_launches(void) { return g_dec_launches; }

namespace agn {
// agn_mlp_backward (mlp.hip) hands over the processor-layer node MLP backward this kernel covers:
// returns false (nothing launched) otherwise; *rc = the launch status; *ln_rows = the rows of
// ln_partial written (the general kernel's block count)
bool node32_bwd_try(const agn_mlp_bwd_args* a, void* stream, int* rc, int* ln_rows) {
  if (a->dtype != AGN_BF16 || a->hidden != H || a->nlin != 4 || a->out_dim != H || a->in_dim != 2 * H ||
      !a->use_ln || a->act_fn != AGN_ACT_RELU || a->din_nseg != 2 || a->din_k[0] != H || a->din_k[1] != H ||
      a->rows < 64 * 1024 || a->rows >= (1 << 26))
    return false;
  if (!a->g || a->g2 || a->gidx || !a->hpre || !a->stats || !a->ln_g) return false;
  for (int l = 0; l < 3; ++l)
    if (!a->mask[l]) return false;
  for (int l = 0; l < 4; ++l)
    if (!a->wtpk[l] || !al16(a->wtpk[l]) || !al16(a->gpre[l])) return false;
  if (!al16(a->g) || !al16(a->hpre) || !al16(a->din[0]) || !al16(a->din[1])) return false;
  // the general kernel's LN partial rows: one per 128-row block
  const int ntiles = (a->rows + 31) / 32;
  const int nblk = (ntiles + ROWS_PER_BLOCK / 32 - 1) / (ROWS_PER_BLOCK / 32);
  hipStream_t st = (hipStream_t)stream;
  float* lnt = nullptr;
  if (a->ln_partial) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    LnScratch& w = g_lnt[dev & 63];
    if (w.last && w.last != st && hipStreamSynchronize(w.last) != hipSuccess) return false;
    const size_t need = (size_t)ntiles * 2 * H;
    if (need > w.cap) {
      if (w.p) {
        if (hipStreamSynchronize(st) != hipSuccess) return false;
        (void)hipFree(w.p);
        w.p = nullptr;
        w.cap = 0;
      }
      if (hipMalloc(&w.p, need * sizeof(float)) != hipSuccess) {
        w.p = nullptr;
        return false;
      }
      w.cap = need;
    }
    w.last = st;
    lnt = w.p;
  }
  const int grid = grid_for(ntiles);
  hipLaunchKernelGGL(node32_bwd_kernel, dim3(grid), dim3(64 * NW), 0, st, *a, lnt);
  if (a->ln_partial)
    hipLaunchKernelGGL(node32_lnp_kernel, dim3((nblk * 2 * H + 255) / 256), dim3(256), 0, st, lnt, ntiles, nblk,
                       a->ln_partial);
  ++g_launches;
  *ln_rows = nblk;
  const hipError_t e = hipGetLastError();
  *rc = e == hipSuccess ? 0 : (int)e;
  return true;
}

// the decoder's backward (dec32_bwd_kernel); false (nothing launched) for any other call
bool dec32_bwd_try(const agn_mlp_bwd_args* a, void* stream, int* rc) {
  if (a->dtype != AGN_BF16 || a->hidden != H || (a->nlin != 3 && a->nlin != 4) || a->out_dim < 1 ||
      a->out_dim > 32 || a->in_dim != H || a->use_ln || a->act_fn != AGN_ACT_RELU || a->din_nseg != 1 ||
      a->din_k[0] != H || a->din_resid[0] || a->rows < 64 * 1024 || a->rows >= (1 << 26))
    return false;
  if (!a->g || a->g2 || a->gidx || ((a->gpre_tiled >> (a->nlin - 1)) & 1)) return false;
  for (int l = 0; l + 1 < a->nlin; ++l)
    if (!a->mask[l]) return false;
  for (int l = 0; l < a->nlin; ++l)
    if (!a->wtpk[l] || !al16(a->wtpk[l]) || !al16(a->gpre[l])) return false;
  if (!al16(a->din[0])) return false;
  const int ntiles = (a->rows + 31) / 32;
  hipStream_t st = (hipStream_t)stream;
  if (a->nlin == 4) hipLaunchKernelGGL(dec32_bwd_kernel<4>, dim3(grid_for(ntiles)), dim3(64 * NW), 0, st, *a);
  else hipLaunchKernelGGL(dec32_bwd_kernel<3>, dim3(grid_for(ntiles)), dim3(64 * NW), 0, st, *a);
  ++g_dec_launches;
  const hipError_t e = hipGetLastError();
  *rc = e == hipSuccess ? 0 : (int)e;
  return true;
}
}  // namespace agn
