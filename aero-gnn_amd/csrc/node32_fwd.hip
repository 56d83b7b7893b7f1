// Forward of the node MLP of a processor layer with the receiver aggregation walked in (gfx950,
// bf16, H = 128, three or four Linears):
//   agg = sum (mean) of e' rows rowptr[r] .. rowptr[r+1]-1        (mgnLayer.py:144-146 scatter)
//   x'  = x + LN(W3 relu(W2 relu(W1 relu(W0 [x | agg] + b0) + b1) + b2) + b3)  (mgnLayer.py NodeBlock)
// bitwise agn_mlp_forward's general kernel on the same operands (mlp.hip mlp_fwd_kernel, M_VEC:
// the same fp32 walk in edge order with one rounding, the same MFMA sequence per accumulator over
// the x units then the agg units, the same LayerNorm and residual steps). agn_mlp_forward routes
// such calls here (node32_fwd_try) unless AGN_OPT_RESIDENT is 0.
//
// Why: the general kernel restages every layer's weights into LDS for each 128-row block, and its
// walk has each lane pair read its own node's rows, so one load instruction touches 32 rows (32-64
// cache lines, 32 B of each). Here W0..W2 stay resident in LDS (128 KB: W0 is 128 x 256; a fourth
// Linear's 32 KB stream from L2) and each of 8 waves per CU streams 32-node tiles: the receivers'
// CSC offsets are prefetched a tile ahead through the wave's LDS slot, the e' rows are walked
// coalesced (16 lanes per row, 4 rows per load instruction, 4 rows in flight per node), the rounded
// sums reach the operand layout through a 2-KB LDS buffer, then the chain runs on the MFMA as
// edge32_fwd.hip's does. C3 level-0 node MLP: 378 against 453 us per launch for the per-lane walk at
// 12 waves (profiles/r5_node32_walk_ab.txt), 490 us for the general kernel.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4;
constexpr int NR = 64;
constexpr int NU = 8;                     // k-steps of 16 per 128 input features
constexpr int L0 = NT * 2 * NU * 64;      // W0 units (K = 256)
constexpr int L1 = NT * NU * 64;          // W1 / W2 units
#ifndef AGN_N32_NW
#define AGN_N32_NW 8
#endif
#ifndef AGN_N32_NQ
#define AGN_N32_NQ 4
#endif
constexpr int NW = AGN_N32_NW;            // waves per CU (8: 256 registers for the walk's loads in flight)
constexpr int NQ = AGN_N32_NQ;            // rows in flight per walked node
constexpr int PF = 2;

constexpr int PFG = 4;  // fragments in flight from L2 (the fourth Linear's weights)

template <int NLIN> struct Smem {
  uint4 w0[L0];
  uint4 w1[L1];
  uint4 w2[L1];          // (W3 of a four-Linear chain streams from L2: 160 KB do not fit beside the rest)
  float pv[NLIN + 2][H]; // b0 .. b_{NLIN-1}, LN gamma, LN beta
  int rp[NW][64];        // per wave: next tile's row pointers (33 used)
  char agg[NW][2048];    // per wave: 8 nodes' rounded sums on their way to the owning lanes
};
static_assert(sizeof(Smem<4>) <= 160 * 1024, "LDS budget");

// acc[ot] += W[ot tile, units u0 .. u0+7] . b, k-steps in order (common.hpp gemm's per-accumulator
// sequence); fragments stream PF deep, ot inner
AGN_DEV void gemm_k8(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int ku_total, int u0, int lane) {
  uint4 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = w[((i % NT) * ku_total + u0 + i / NT) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < NT * NU; ++idx) {
    const uint4 cur = f[idx % PF];
    const int nx = idx + PF;
    if (nx < NT * NU) f[idx % PF] = w[((nx % NT) * ku_total + u0 + nx / NT) * 64 + lane];
    b.mfma(acc[idx % NT], cur, idx / NT);
  }
}

// the same from global memory (an L2-resident 32 KB image), PFG fragments in flight
AGN_DEV void gemm_k8_g(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int lane) {
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

// SAVES: the training saves of agn_mlp_fwd_args (relu outputs act[0..1] with their AGN_RELU_MASK
// bits, hpre, stats; row-major or AGN_TILED as a.tiled says), as the general kernel writes them
template <int NLIN, bool SAVES>
__global__ __launch_bounds__(64 * NW) void node32_fwd_kernel(const agn_mlp_fwd_args a) {
  constexpr int NTHR = 64 * NW;
  __shared__ Smem<NLIN> sm;
  {
    const uint4* w0 = reinterpret_cast<const uint4*>(a.wpk[0]);
    const uint4* w1 = reinterpret_cast<const uint4*>(a.wpk[1]);
    const uint4* w2 = reinterpret_cast<const uint4*>(a.wpk[2]);
    for (int i = threadIdx.x; i < L0; i += NTHR) sm.w0[i] = w0[i];
    for (int i = threadIdx.x; i < L1; i += NTHR) {
      sm.w1[i] = w1[i];
      sm.w2[i] = w2[i];
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
  int* wrp = sm.rp[w];
  const agn_seg& sx = a.seg[0];
  const agn_seg& sg = a.seg[1];
  const int32_t* const rowptr = sg.index;
  // lane l <= 32 loads rowptr[32 t + l] (clamped: a partial last tile's rows past the end are empty)
  auto tile_rp = [&](int t) { return rowptr[min(t * 32 + min(lane0, 32), a.rows)]; };
  if (walk.first < walk.end) wrp[lane0] = tile_rp(walk.first);
  const bf16* X = reinterpret_cast<const bf16*>(sx.ptr);
  const bf16* EP = reinterpret_cast<const bf16*>(sg.ptr);
  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    cbarrier();
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const bool more = tile + walk.step < walk.end;
    const int nrp = tile_rp(more ? tile + walk.step : tile);
    // ---- agg: each node's e' rows in edge order, fp32, one rounding (mlp.hip walk2_segment's
    // values). The rows are read coalesced: lane group g = lane / 16 walks one node of a round,
    // lane k = lane % 16 loads chunk k (16 B) of each of its rows, so one load instruction covers 4
    // whole rows; two nodes per lane group (A, B) with up to 4 rows each in flight. The rounded sums
    // reach the owning lanes (node c: lanes c and c + 32, the operand layout) through the wave's
    // 2-KB LDS buffer, 8 nodes per batch.
    BOp<bf16, NR> bagg;
    {
      const int g = lane >> 4, k = lane & 15;
      char* buf = sm.agg[w];
      uint4 mine[NR / 8];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) mine[i] = uint4{0u, 0u, 0u, 0u};
      const bf16* ek = EP + 8 * k;
#pragma unroll 1
      for (int bt = 0; bt < 4; ++bt) {
        int beg[2], end[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int nl = 8 * bt + 4 * n + g;  // tile-local node
          // a partial last tile's rows past the end walk the last row's edges, as the general
          // kernel does (its padding rows then carry the same values, mask bits included)
          const int cc = tile * 32 + nl < a.rows ? nl : a.rows - 1 - tile * 32;
          beg[n] = wrp[cc];
          end[n] = wrp[cc + 1];
        }
        float sum[2][8];
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int e = 0; e < 8; ++e) sum[n][e] = 0.f;
        const int steps = max(end[0] - beg[0], end[1] - beg[1]);
#pragma unroll 1
        for (int j = 0; j < steps; j += NQ) {
          uint4 r[2][NQ];
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int q = 0; q < NQ; ++q)
              if (beg[n] + j + q < end[n]) r[n][q] = *reinterpret_cast<const uint4*>(ek + (size_t)(beg[n] + j + q) * sg.ld);
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int q = 0; q < NQ; ++q)
              if (beg[n] + j + q < end[n]) {
                const u32x4 x = __builtin_bit_cast(u32x4, r[n][q]);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                  sum[n][2 * d] += lo_bf16(x[d]);
                  sum[n][2 * d + 1] += hi_bf16(x[d]);
                }
              }
        }
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if (sg.kind == AGN_SEG_MEAN) {
            const float cnt = (float)max(end[n] - beg[n], 1);
#pragma unroll
            for (int e = 0; e < 8; ++e) sum[n][e] = sum[n][e] / cnt;
          }
          const u32x4 pk = {pack2(sum[n][0], sum[n][1]), pack2(sum[n][2], sum[n][3]), pack2(sum[n][4], sum[n][5]),
                            pack2(sum[n][6], sum[n][7])};
          const int nl = 8 * bt + 4 * n + g;
          if (sg.store && tile * 32 + nl < a.rows)
            *reinterpret_cast<u32x4*>(reinterpret_cast<bf16*>(sg.store) + (size_t)(tile * 32 + nl) * H + 8 * k) = pk;
          *reinterpret_cast<u32x4*>(buf + (4 * n + g) * 256 + 16 * k) = pk;
        }
        // owners of this batch's nodes take their chunks (2i + h of their row) from the buffer
        // (LDS is in order per wave: the reads see the writes above)
        // (every lane reads, the owners keep: mine starts at 0 and each lane owns one batch's node)
        const int nb = c - 8 * bt;
        const uint32_t keep = (unsigned)nb < 8u ? ~0u : 0u;
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) {
          const uint4 v = *reinterpret_cast<const uint4*>(buf + (nb & 7) * 256 + 16 * (2 * i + h));
          mine[i].x |= v.x & keep;
          mine[i].y |= v.y & keep;
          mine[i].z |= v.z & keep;
          mine[i].w |= v.w & keep;
        }
      }
      if (more) wrp[lane] = nrp;  // (this tile's reads of the slot are done)
      bagg.set_w(mine);
      // the operand materialised here, before the x loads (else the two overlap and spill)
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        u32x4 t = __builtin_bit_cast(u32x4, bagg.u[i]);
        asm volatile("" : "+v"(t));
        bagg.u[i] = __builtin_bit_cast(bf16x8, t);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- layer 0: bias, then the x units, then the agg units. Row offsets are recomputed from an
    // opaque lane id here, not carried across the walk (where they would spill)
    cbarrier();
    const int lane_b = opaque_v(lane0);
    const int hb = lane_b >> 5;
    const int row_b = tile * 32 + (lane_b & 31);
    const bool valid_b = row_b < a.rows;
    BOp<bf16, NR> bx;
    bx.load_w(X + (size_t)(valid_b ? row_b : a.rows - 1) * sx.ld, hb);
    f32x16 acc[NT];
#pragma unroll
    for (int q = 0; q < 4 * NT; ++q) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&sm.pv[0][8 * q + 4 * hb]);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = v[e];
    }
    gemm_k8(acc, bx, sm.w0, 2 * NU, 0, lane_b);
    gemm_k8(acc, bagg, sm.w0, 2 * NU, NU, lane_b);
    BOp<bf16, NR> b;
#pragma unroll
    for (int l = 1; l < NLIN; ++l) {
      cbarrier();
      b.template set_relu<NT>(acc);
      auto save = [&]() {
        if (a.act[l - 1]) {
          if (a.tiled) b.store_tiled(reinterpret_cast<bf16*>(a.act[l - 1]), row_b, hb, valid_b);
          else b.store(reinterpret_cast<bf16*>(a.act[l - 1]) + (size_t)row_b * H, hb, valid_b);
        }
        if (a.mask[l - 1]) store_relu_mask<bf16, NR>(a.mask[l - 1], b, tile, lane_b);
      };
      // the layer whose weights stream from L2 (W3) saves its input after the product: vmcnt retires
      // loads and stores in issue order, so W3 fragments loaded after the saves would wait for them
      if constexpr (SAVES) {
        if (l != 3) save();
      }
#pragma unroll
      for (int q = 0; q < 4 * NT; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(&sm.pv[l][8 * q + 4 * hb]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = v[e];
      }
      if (l == 3) gemm_k8_g(acc, b, reinterpret_cast<const uint4*>(a.wpk[3]), lane_b);
      else gemm_k8(acc, b, l == 1 ? sm.w1 : sm.w2, NU, 0, lane_b);
      if constexpr (SAVES) {
        if (l == 3) save();
      }
    }
    cbarrier();
    if constexpr (SAVES) {  // the pre-LayerNorm row (the backward's LayerNorm input)
      if (a.hpre) {
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
          if (a.tiled) store8_tiled<bf16, NR>(reinterpret_cast<bf16*>(a.hpre), i, row_b, hb, v, valid_b);
          else store8_w(reinterpret_cast<bf16*>(a.hpre) + (size_t)row_b * H, i, hb, v, valid_b);
        }
      }
    }
    // ---- LayerNorm (general kernel order), residual x, store
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
      if (a.stats && valid_b && hb == 0) {
        a.stats[2 * (size_t)row_b] = mean;
        a.stats[2 * (size_t)row_b + 1] = rstd;
      }
    }
    bf16* op = reinterpret_cast<bf16*>(a.out) + (size_t)row_b * a.out_ld;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int f0 = 16 * i + 8 * jj + 4 * hb;
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
      float r[8];
      bx.get8(r, i);
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t p = pack2(v[e], v[e + 1]);
        const f32x2 o = f2(lo_bf16(p), hi_bf16(p)) + f2(r[e], r[e + 1]);
        v[e] = o[0];
        v[e + 1] = o[1];
      }
      store8_w(op, i, hb, v, valid_b);
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

long g_launches = 0;  // launches so far (agn_debug_node32_launches: tests check the dispatch)

}  // namespace

extern "C" long agn_debug_node32_launches(void) { return g_launches; }

namespace agn {
// agn_mlp_forward (mlp.hip) hands over the node MLPs this kernel covers: returns false (nothing
// launched) otherwise; *rc = the launch status
bool node32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc) {
  if (a->dtype != AGN_BF16 || a->hidden != H || (a->nlin != 3 && a->nlin != 4) || a->nseg != 2 || a->out_dim != H || !a->use_ln ||
      a->act_fn != AGN_ACT_RELU || a->proj || a->rows < 64 * 1024 || a->rows >= (1 << 26))
    return false;
  const agn_seg& sx = a->seg[0];
  const agn_seg& sg = a->seg[1];
  if (sx.kind != AGN_SEG_PLAIN || sx.k != H || sx.ld % 8 || !sx.ptr) return false;
  if ((sg.kind != AGN_SEG_SUM && sg.kind != AGN_SEG_MEAN) || sg.k != H || sg.ld % 8 || !sg.ptr || !sg.index) return false;
  if (a->resid != sx.ptr || a->out_ld != sx.ld || a->out_ld % 8) return false;
  // training saves: ReLU outputs (+ mask bits), hpre, stats (no pre-activations: ReLU only)
  bool saves = a->hpre || a->stats;
  for (int l = 0; l < AGN_MAX_LIN; ++l) {
    if (a->pre[l] || (l >= a->nlin - 1 && (a->act[l] || a->mask[l]))) return false;
    saves = saves || a->act[l] || a->mask[l];
    if (!al16(a->act[l])) return false;
  }
  if (!al16(a->hpre)) return false;
  for (int l = 0; l < a->nlin; ++l)
    if (!a->wpk[l] || !al16(a->wpk[l])) return false;
  if (!al16(sx.ptr) || !al16(sg.ptr) || !al16(a->out) || !al16(sg.store)) return false;
  const int tiles = (a->rows + 31) / 32;
  const int need = (tiles + NW - 1) / NW;
  const int cus = cu_count();
  const int nblk = need >= cus ? cus : ((need + 7) / 8 * 8 < 8 ? 8 : (need + 7) / 8 * 8);
  const dim3 g(nblk), blk(64 * NW);
  hipStream_t st = (hipStream_t)stream;
  if (a->nlin == 4) {
    if (saves) hipLaunchKernelGGL((node32_fwd_kernel<4, true>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((node32_fwd_kernel<4, false>), g, blk, 0, st, *a);
  } else {
    if (saves) hipLaunchKernelGGL((node32_fwd_kernel<3, true>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((node32_fwd_kernel<3, false>), g, blk, 0, st, *a);
  }
  ++g_launches;
  const hipError_t e = hipGetLastError();
  *rc = e == hipSuccess ? 0 : (int)e;
  return true;
}
}  // namespace agn
