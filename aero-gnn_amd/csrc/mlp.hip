// Fused MLP chains on MFMA for the MeshGraphNet hot path (gfx950).
//
// One kernel evaluates a whole reference MLP — models/mlp.py:40-51 (Linear -> ReLU -> ... ->
// Linear -> LayerNorm) — for 32 rows per wave, with the layer-0 input assembled on the fly:
//   * EdgeBlockSum (models/mgnLayer.py:93-105): acc0 = P_s[src] + P_d[dst], input e, K = H,
//     then ReLU/Linear chain, LN, and the residual e' = e + LN(..) of mgnLayer.py:205;
//   * EdgeBlock    (mgnLayer.py:32-49): input cat[e, x[row], x[col]] via GATHER segments;
//   * NodeBlock    (mgnLayer.py:134-153): input cat[x, scatter_add(e', col)] where the SUM
//     segment reduces the receiver-grouped (CSC) rows of e' in edge order (bitwise the
//     torch_scatter summation order for fp32), residual x' = x + .. (mgnLayer.py:211);
//   * encoders / decoder / node projections: plain inputs.
// Activations never leave registers between layers (see common.hpp for the layout); only
// the block output (and, when training, the per-layer activations) are written to HBM.
// Each layer's packed weights are staged in LDS once per 128-row block.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int WPB = 4;           // waves per block
constexpr int BLOCK = 64 * WPB;  // 128 data rows per block

template <typename T, int NT>
constexpr int lds_units() { return NT * (nrk(32 * NT) / BOp<T, 16>::RPU) * 64; }

// Stage the packed A fragments of out tiles [ot0, ot0+otn) x K units [unit0, unit0+nu) of a
// packed matrix with `ku_total` units per tile into LDS as [otn][nu][64] (16 B each).
AGN_DEV void stage_block(uint4* lds, const void* gw, int ku_total, int ot0, int otn, int unit0, int nu) {
  const uint4* g = reinterpret_cast<const uint4*>(gw);
  const int per = nu * 64;
  const int n = otn * per;
  for (int i = threadIdx.x; i < n; i += BLOCK) {
    const int ot = i / per, rem = i - ot * per;
    lds[i] = g[((size_t)(ot0 + ot) * ku_total + unit0) * 64 + rem];
  }
}

// Row I/O in acc layout. VEC: k == 32*NT features, 16-B aligned rows -> 16-B per-lane
// accesses through lane-half exchanges (common.hpp load8_w/store8_w; all lanes of a row pair
// must be active together). !VEC: masked 4-feature chunks.
template <typename T, int NR, bool VEC>
AGN_DEV void load_row(float (&v)[NR], const T* rowp, int k, int h) {
  if constexpr (VEC) {
    load_row_w<T, NR>(v, rowp, h);
  } else {
#pragma unroll
    for (int q = 0; q < NR / 4; ++q) {
      const f32x4 x = load4_masked(rowp, 8 * q + 4 * h, k, false);
      v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
    }
  }
}
template <typename T, int NR, bool VEC>
AGN_DEV void add_row(float (&v)[NR], const T* rowp, int k, int h) {
  if constexpr (VEC) {
    add_row_w<T, NR>(v, rowp, h);
  } else {
#pragma unroll
    for (int q = 0; q < NR / 4; ++q) {
      const f32x4 x = load4_masked(rowp, 8 * q + 4 * h, k, false);
      v[4 * q] += x[0]; v[4 * q + 1] += x[1]; v[4 * q + 2] += x[2]; v[4 * q + 3] += x[3];
    }
  }
}
template <typename T, int NR, bool VEC>
AGN_DEV void store_row(T* rowp, int k, const float (&v)[NR], int h, bool valid) {
  if constexpr (VEC) {
    store_row_w<T, NR>(rowp, v, h, valid);
  } else if (valid) {
#pragma unroll
    for (int q = 0; q < NR / 4; ++q) {
      const f32x4 x = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      store4_masked(rowp, 8 * q + 4 * h, k, false, x);
    }
  }
}

template <int NT, int NR>
AGN_DEV void acc_to_regs(float (&v)[NR], const f32x16 (&acc)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[16 * t + r] = acc[t][r];
}

template <int NT, bool FULL>
AGN_DEV void acc_bias(f32x16 (&acc)[NT], const float* b, int nvalid, int h) {
  float v[16 * NT];
  if (FULL && b) load_param<16 * NT, true>(v, b, nvalid, h);
  else load_param<16 * NT, false>(v, b, nvalid, h);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = v[16 * t + r];
}

// bias from an LDS copy of the parameter vector (H floats)
template <int NT>
AGN_DEV void acc_bias_lds(f32x16 (&acc)[NT], const float* pv, int h) {
#pragma unroll
  for (int q = 0; q < 4 * NT; ++q) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(pv + 8 * q + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
  }
}

// Stage the per-feature fp32 parameter vectors of a resident chain into LDS:
// pv[l] = bias of Linear l (0 if absent), pv[RES_MAXL] = LN gamma, pv[RES_MAXL + 1] = LN beta.
template <int H, int NV>
AGN_DEV void stage_params(float (*pv)[H], const float* const* bias, int nlin, const float* g, const float* b,
                          int nthreads) {
  for (int i = threadIdx.x; i < NV * H; i += nthreads) {
    const int l = i / H, f = i - l * H;
    const float* src = l < NV - 2 ? (l < nlin ? bias[l] : nullptr) : (l == NV - 2 ? g : b);
    pv[l][f] = src ? src[f] : 0.f;
  }
}

// Load one input segment for data row `rr` into acc-layout registers.
template <typename T, int NR, bool VEC>
AGN_DEV void load_segment(float (&in)[NR], const agn_seg& s, int rr, bool valid, int h) {
  const T* base = reinterpret_cast<const T*>(s.ptr);
  if (s.kind == AGN_SEG_PLAIN || s.kind == AGN_SEG_GATHER) {
    const int r = (s.kind == AGN_SEG_GATHER) ? s.index[rr] : rr;
    load_row<T, NR, VEC>(in, base + (size_t)r * s.ld, s.k, h);
  } else {  // SUM / MEAN over rows index[rr] .. index[rr+1]-1 (receiver-grouped edges)
#pragma unroll
    for (int i = 0; i < NR; ++i) in[i] = 0.f;
    const int beg = s.index[rr], end = s.index[rr + 1];
    for (int j = beg; j < end; ++j) add_row<T, NR, VEC>(in, base + (size_t)j * s.ld, s.k, h);
    if (s.kind == AGN_SEG_MEAN) {
      const float cnt = (float)max(end - beg, 1);
#pragma unroll
      for (int i = 0; i < NR; ++i) in[i] = in[i] / cnt;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) in[i] = round_t<T>(in[i]);
    if (s.store) store_row<T, NR, VEC>(reinterpret_cast<T*>(s.store) + (size_t)rr * s.k, s.k, in, h, valid);
  }
}

// ------------------------------------------------------------------------- forward
// I/O modes of the general kernels (compile-time, chosen on the host per call):
//   M_VEC : every input segment and the output are H wide (16-B row I/O everywhere)
//   M_NIN : one PLAIN or GATHER input of k <= 16 features (encoders: d_n = 6, d_e = 4), output H wide
//   M_NOUT: H-wide inputs, nlin > 1, output of <= 32 features, no LayerNorm (decoder: d_out = 4)
//   M_GEN : anything else (masked 4-feature chunks)
enum { M_VEC = 0, M_GEN = 1, M_NIN = 2, M_NOUT = 3 };

// k <= 16 features of one row into acc-layout registers (features >= k and >= 16 are zero)
template <typename T, int NR>
AGN_DEV void load_row_narrow(float (&v)[NR], const T* rowp, int k, int h) {
#pragma unroll
  for (int i = 0; i < NR; ++i) v[i] = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const f32x4 x = load4_masked(rowp, 8 * q + 4 * h, k, false);
    v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
  }
}

// load_segment's SUM / MEAN walk with two member rows' loads in flight per step (adds in edge
// order, one rounding: the same values). Run before anything else of the wave is live.
#ifndef AGN_WALK2
#define AGN_WALK2 1
#endif
template <int NR>
AGN_DEV void walk2_segment(float (&in)[NR], const agn_seg& s, int rr, bool valid, int h) {
  const bf16* base = reinterpret_cast<const bf16*>(s.ptr);
#pragma unroll
  for (int i = 0; i < NR; ++i) in[i] = 0.f;
  const int beg = s.index[rr], end = s.index[rr + 1];
  int j = beg;
  for (; j + 1 < end; j += 2) {
    uint4 r0[NR / 8], r1[NR / 8];
    const bf16* p0 = base + (size_t)j * s.ld;
    const bf16* p1 = p0 + s.ld;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) r0[i] = *reinterpret_cast<const uint4*>(p0 + 16 * i + 8 * h);
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) r1[i] = *reinterpret_cast<const uint4*>(p1 + 16 * i + 8 * h);
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float o[8];
      unpack8_w(o, r0[i]);  // load8_w's exchange + conversion
#pragma unroll
      for (int e = 0; e < 8; ++e) in[8 * i + e] += o[e];
    }
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float o[8];
      unpack8_w(o, r1[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) in[8 * i + e] += o[e];
    }
  }
  if (j < end) add_row_w<bf16, NR>(in, base + (size_t)j * s.ld, h);
  if (s.kind == AGN_SEG_MEAN) {
    const float cnt = (float)max(end - beg, 1);
#pragma unroll
    for (int i = 0; i < NR; ++i) in[i] = in[i] / cnt;
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) in[i] = round_t<bf16>(in[i]);
  if (s.store) store_row<bf16, NR, true>(reinterpret_cast<bf16*>(s.store) + (size_t)rr * s.k, s.k, in, h, valid);
}

// A hidden activation other than ReLU (AGN_ACT_*): the Linear output rounded to T, saved to pre
// (the backward's x) when given, the activation applied in fp32 and packed (rounded) into b
template <typename T, int NT, int NR>
AGN_DEV void set_act(BOp<T, NR>& b, const f32x16 (&acc)[NT], int k, T* pre, int tiled, int row, int h, bool valid) {
  constexpr int H = 32 * NT;
  float v[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) v[i] = round_t<T>(acc[i / 16][i % 16]);
  if (pre) {
    BOp<T, NR> pb;
    pb.set(v);
    if (tiled) pb.store_tiled(pre, row, h, valid);
    else pb.store(pre + (size_t)row * H, h, valid);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) v[i] = act_fwd(k, v[i]);
  b.set(v);
}

// GACT: a hidden activation other than ReLU (agn_mlp_*_args.act_fn); the ReLU instantiations
// carry none of its registers
template <typename T, int NT, int MODE, bool GACT>
__global__ __launch_bounds__(BLOCK, 2) void mlp_fwd_kernel(const agn_mlp_fwd_args a) {
  constexpr int H = 32 * NT;
  constexpr int NR = 16 * NT;
  constexpr int NUH = nrk(H) / BOp<T, NR>::RPU;  // K units of an H-wide input
  constexpr bool IN_FULL = (MODE == M_VEC || MODE == M_NOUT);
  constexpr bool OUT_FULL = (MODE == M_VEC || MODE == M_NIN);
  __shared__ uint4 wl[lds_units<T, NT>()];
  // 8-row LDS staging of full-width PLAIN inputs / outputs (bf16, H >= 64): measured slower in this
  // non-persistent kernel (node MLP 0.60 -> 0.73 ms: extra LDS passes + spills), so it is off
  constexpr bool STAGE = false;
  __shared__ uint4 stg[STAGE ? WPB : 1][8][STAGE ? 4 * NT + STG_PAD : 1];
  const int lane = threadIdx.x & 63;
  const int c = lane & 31, h = lane >> 5;
  const int wave = blockIdx.x * WPB + (threadIdx.x >> 6);
  const int row = wave * 32 + c;
  const bool valid = row < a.rows;
  const int rr = valid ? row : a.rows - 1;

  f32x16 acc[NT];
  float v[NR];
  BOp<T, NR> b;

  int k0 = 0;
  for (int s = 0; s < a.nseg; ++s) k0 += a.seg[s].k;
  const int ku0 = units_k<T>(k0);
  // a node MLP's SUM / MEAN input is walked first, while nothing else of the wave is live, and
  // kept packed until its GEMM (the layer-0 GEMM order, hence every sum, is unchanged)
  constexpr bool W2 = AGN_WALK2 && MODE == M_VEC && std::is_same<T, bf16>::value && NT == 4;
  const bool walk2 = W2 && a.nseg == 2 && (a.seg[1].kind == AGN_SEG_SUM || a.seg[1].kind == AGN_SEG_MEAN) &&
                     a.seg[1].k == H;
  BOp<T, NR> bagg;
  if constexpr (W2) {
    if (walk2) {
      walk2_segment<NR>(v, a.seg[1], rr, valid, h);
      bagg.set(v);
    }
  }
  const int ngrp = (a.nlin == 1) ? (a.out_dim + H - 1) / H : 1;

  for (int grp = 0; grp < ngrp; ++grp) {
    const int out0 = (a.nlin == 1) ? a.out_dim : H;
    const int gofs = grp * H;
    const int nv0 = min(H, out0 - gofs);
    const int otn0 = (nv0 + 31) / 32;
    // ---- layer-0 accumulator init: bias, or the EdgeBlockSum projections gathered by src/dst
    if (a.proj) {
      const T* P = reinterpret_cast<const T*>(a.proj);
      const T* ps = P + (size_t)a.src[rr] * (2 * H);
      const T* pd = P + (size_t)a.dst[rr] * (2 * H) + H;
      // one 16-feature pair per round: keeps the gathered rows from all being live at once
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        cbarrier();
        float x[8], y[8];
        load8_w(x, ps, i, h);
        load8_w(y, pd, i, h);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[(8 * i + e) / 16][(8 * i + e) % 16] = x[e] + y[e];
      }
    } else {
      acc_bias<NT, OUT_FULL || MODE == M_NOUT>(acc, a.bias[0] ? a.bias[0] + gofs : nullptr, nv0, h);
    }
    // ---- layer 0: sum over input segments
    int unit = 0;
    for (int s = 0; s < a.nseg; ++s) {
      const int nu = units_k<T>(a.seg[s].k);
      __syncthreads();
      stage_block(wl, a.wpk[0], ku0, grp * NT, otn0, unit, nu);
      if constexpr (MODE == M_NIN) {  // PLAIN, or GATHER (the caller's row order permuted in the load)
        const int src_row = a.seg[s].kind == AGN_SEG_GATHER ? a.seg[s].index[rr] : rr;
        load_row_narrow<T, NR>(v, reinterpret_cast<const T*>(a.seg[s].ptr) + (size_t)src_row * a.seg[s].ld, a.seg[s].k, h);
      } else {
        bool staged = false;
        if constexpr (STAGE && IN_FULL) {
          if (a.seg[s].kind == AGN_SEG_PLAIN) {
            uint4 mine[NR / 8];
            tile_load_chunks<4 * NT>(mine, reinterpret_cast<const bf16*>(a.seg[s].ptr) + (size_t)wave * 32 * a.seg[s].ld,
                                     a.rows - wave * 32, stg[threadIdx.x >> 6], lane, a.seg[s].ld / 8);
            b.set_w(mine);  // the operand from the chunks directly (no fp32 round trip)
            staged = true;
          }
        }
        if (!staged) {
          if (W2 && walk2 && s == 1) staged = true;
          else load_segment<T, NR, IN_FULL>(v, a.seg[s], rr, valid, h);
        }
      }
      bool staged_b = false;
      if constexpr (STAGE && IN_FULL && MODE != M_NIN) staged_b = a.seg[s].kind == AGN_SEG_PLAIN;
      if (W2 && walk2 && s == 1) b = bagg;
      else if (!staged_b) b.set(v);
      __syncthreads();
      if constexpr (IN_FULL) gemm<T, NT, NR, true>(acc, b, NUH, wl, NUH, NT, lane);
      else if constexpr (MODE == M_NIN) gemm<T, NT, NR, true>(acc, b, nu, wl, nu, NT, lane);
      else gemm<T, NT, NR>(acc, b, nu, wl, nu, otn0, lane);
      unit += nu;
    }
    // ---- hidden layers: relu(acc) -> packed operand -> next Linear (registers only)
    for (int l = 1; l < a.nlin; ++l) {
      const bool last = (l == a.nlin - 1);
      const int outl = last ? a.out_dim : H;
      const int otn = (outl + 31) / 32;
      __syncthreads();
      stage_block(wl, a.wpk[l], NUH, 0, otn, 0, NUH);
      if constexpr (GACT) set_act<T, NT, NR>(b, acc, a.act_fn, reinterpret_cast<T*>(a.pre[l - 1]), a.tiled, row, h, valid);
      else b.template set_relu<NT>(acc);
      if (a.act[l - 1]) {
        if (a.tiled) b.store_tiled(reinterpret_cast<T*>(a.act[l - 1]), row, h, valid);
        else b.store(reinterpret_cast<T*>(a.act[l - 1]) + (size_t)row * H, h, valid);
      }
      // waves past the last 32-row tile (the grid rounds up to WPB waves) own no mask tile
      if (!GACT && a.mask[l - 1] && wave * 32 < a.rows)
        store_relu_mask<T, NR>(a.mask[l - 1], b, wave, lane);
      if (OUT_FULL || !last) acc_bias<NT, true>(acc, a.bias[l], H, h);
      else acc_bias<NT, false>(acc, a.bias[l], outl, h);
      __syncthreads();
      if (OUT_FULL || !last) gemm<T, NT, NR, true>(acc, b, NUH, wl, NUH, NT, lane);
      else gemm<T, NT, NR>(acc, b, NUH, wl, NUH, otn, lane);
    }
    // ---- epilogue: LayerNorm, residual, store
    const int outd = (a.nlin == 1) ? nv0 : a.out_dim;
    float mean = 0.f, rstd = 1.f;
    if (MODE != M_NOUT && a.use_ln) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NR; ++i) s += (OUT_FULL || feat_of(i, h) < outd) ? acc[i / 16][i % 16] : 0.f;
      s = sum32(s);
      mean = s / (float)outd;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const float d = acc[i / 16][i % 16] - mean;
        if (OUT_FULL || feat_of(i, h) < outd) q = ln_sq_acc(q, d);
      }
      q = sum32(q);
      rstd = 1.0f / sqrtf(q / (float)outd + 1e-5f);
      if (a.stats && valid && h == 0) {
        a.stats[2 * (size_t)row] = mean;
        a.stats[2 * (size_t)row + 1] = rstd;
      }
    }
    T* hp = a.hpre ? reinterpret_cast<T*>(a.hpre) + (size_t)row * outd : nullptr;
    const T* rp = a.resid ? reinterpret_cast<const T*>(a.resid) + (size_t)rr * a.out_ld + gofs : nullptr;
    T* op = reinterpret_cast<T*>(a.out) + (size_t)row * a.out_ld + gofs;
    if constexpr (OUT_FULL) {
      uint4 ob[STAGE ? NR / 8 : 1];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
        if (a.use_ln) {
          if (hp) {
            if (a.tiled) store8_tiled<T, NR>(reinterpret_cast<T*>(a.hpre), i, row, h, v8, valid);
            else store8_w(hp, i, h, v8, valid);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int f0 = 16 * i + 8 * j + 4 * h;
            const f32x4 g4 = *reinterpret_cast<const f32x4*>(a.ln_g + f0);
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.ln_b + f0);
#pragma unroll
            for (int e = 0; e < 4; ++e) v8[4 * j + e] = ln_out(v8[4 * j + e], mean, rstd, g4[e], b4[e]);
          }
        }
        if (rp) {
          float r8[8];
          load8_w(r8, rp, i, h);
#pragma unroll
          for (int e = 0; e < 8; ++e) v8[e] = round_t<T>(v8[e]) + r8[e];
        }
        if constexpr (STAGE) ob[i] = pack8_w(v8, h);
        else store8_w(op, i, h, v8, valid);
      }
      if constexpr (STAGE)
        tile_store_chunks<4 * NT>(ob, reinterpret_cast<bf16*>(a.out) + (size_t)wave * 32 * a.out_ld + gofs,
                                  a.rows - wave * 32, stg[threadIdx.x >> 6], lane, a.out_ld / 8);
    } else {
      // M_NOUT: only the first 32 features (acc tile 0) exist; M_GEN: all, masked
      constexpr int NQ = (MODE == M_NOUT) ? 4 : NR / 4;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int f0 = 8 * q + 4 * h;
        f32x4 v = {acc[q / 4][4 * (q % 4)], acc[q / 4][4 * (q % 4) + 1], acc[q / 4][4 * (q % 4) + 2],
                   acc[q / 4][4 * (q % 4) + 3]};
        if (MODE != M_NOUT && a.use_ln) {
          if (hp && valid) {
            if (a.tiled) store4_tiled<T, NR>(reinterpret_cast<T*>(a.hpre), q, row, h, v);  // outd == H
            else store4_masked(hp, f0, outd, false, v);
          }
          f32x4 g4 = {1.f, 1.f, 1.f, 1.f}, b4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (f0 + e < outd) { g4[e] = a.ln_g[f0 + e]; b4[e] = a.ln_b[f0 + e]; }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ln_out(v[e], mean, rstd, g4[e], b4[e]);
        }
        if (rp) {
          const f32x4 r = load4_masked(rp, f0, outd, false);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = round_t<T>(v[e]) + r[e];
        }
        if (valid) store4_masked(op, f0, outd, false, v);
      }
    }
  }
}

// ------------------------------------------------------------------------- backward
template <typename T, int NR, int MODE>
AGN_DEV void load_grad(float (&g)[NR], const agn_mlp_bwd_args& a, int rr, bool valid, int h) {
  const T* g1 = a.g ? reinterpret_cast<const T*>(a.g) + (size_t)rr * a.out_dim : nullptr;
  const T* g2 = a.g2 ? reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim : nullptr;
  if constexpr (MODE == M_NOUT) {  // out_dim <= 32: acc tile 0 only
#pragma unroll
    for (int i = 0; i < NR; ++i) g[i] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 x = g1 ? load4_masked(g1, 8 * q + 4 * h, a.out_dim, false) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (g2) {
        const f32x4 y = load4_masked(g2, 8 * q + 4 * h, a.out_dim, false);
        x[0] += y[0]; x[1] += y[1]; x[2] += y[2]; x[3] += y[3];
      }
      g[4 * q] = x[0]; g[4 * q + 1] = x[1]; g[4 * q + 2] = x[2]; g[4 * q + 3] = x[3];
    }
  } else {
    if (g1) {
      load_row<T, NR, MODE == M_VEC>(g, g1, a.out_dim, h);
    } else {
#pragma unroll
      for (int i = 0; i < NR; ++i) g[i] = 0.f;
    }
    if (g2) add_row<T, NR, MODE == M_VEC>(g, g2, a.out_dim, h);
  }
  if (!valid) {
#pragma unroll
    for (int i = 0; i < NR; ++i) g[i] = 0.f;
  }
}

// GACT: a hidden activation other than ReLU (agn_mlp_*_args.act_fn); the ReLU instantiations
// carry none of its registers
template <typename T, int NT, int MODE, bool GACT>
__global__ __launch_bounds__(BLOCK, 2) void mlp_bwd_kernel(const agn_mlp_bwd_args a) {
  constexpr bool VEC = (MODE == M_VEC);
  constexpr int H = 32 * NT;
  constexpr int NR = 16 * NT;
  constexpr int NP = (NR >= 32) ? NR / 32 : 1;
  __shared__ uint4 wl[lds_units<T, NT>()];
  __shared__ float lnp[WPB][2][H];
  const int lane = threadIdx.x & 63;
  const int c = lane & 31, h = lane >> 5;
  const int wid = threadIdx.x >> 6;
  const int wave = blockIdx.x * WPB + wid;
  const int row = wave * 32 + c;
  const bool valid = row < a.rows;
  const int rr = valid ? row : a.rows - 1;
  const int M = a.out_dim;

  float A[NR];  // current dL/d(pre-activation)
  load_grad<T, NR, MODE>(A, a, rr, valid, h);
  if (MODE != M_NOUT && a.use_ln) {
    // LayerNorm backward, streamed 4 features at a time (hpre, gamma re-read per chunk)
    const float mean = a.stats[2 * (size_t)rr], rstd = a.stats[2 * (size_t)rr + 1];
    const T* hp = reinterpret_cast<const T*>(a.hpre) + (size_t)rr * M;
    float B[NR];
    float c1 = 0.f, c2 = 0.f;
#pragma unroll
    for (int q = 0; q < NR / 4; ++q) {
      const int f0 = 8 * q + 4 * h;
      const f32x4 hv = a.tiled ? load4_tiled<T, NR>(reinterpret_cast<const T*>(a.hpre), q, rr, h)  // M == H
                       : VEC ? load4(hp + f0) : load4_masked(hp, f0, M, false);
      f32x4 gm = {0.f, 0.f, 0.f, 0.f};
      if (VEC) gm = *reinterpret_cast<const f32x4*>(a.ln_g + f0);
      else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + e < M) gm[e] = a.ln_g[f0 + e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool in = VEC || f0 + e < M;
        const float xh = in ? (hv[e] - mean) * rstd : 0.f;
        ln_bwd_acc(c1, c2, A[4 * q + e], gm[e], xh);
        B[4 * q + e] = A[4 * q + e] * xh;  // g * xhat (LN weight-grad partial)
      }
    }
    c1 = sum32(c1);
    c2 = sum32(c2);
    c1 /= (float)M;
    c2 /= (float)M;
    if (a.ln_partial) {  // LayerNorm parameter partials over the wave's 32 rows (butterfly)
      butterfly_reduce<NR>(B, lane);
      float pg[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) pg[i] = B[i];
#pragma unroll
      for (int i = 0; i < NR; ++i) B[i] = A[i];
      butterfly_reduce<NR>(B, lane);
      const bool canon = (NR >= 32) || ((c % (32 / (NR < 32 ? NR : 32))) == 0);
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int f = feat_of((c * NR) / 32 + i, h);
        if (canon) { lnp[wid][0][f] = pg[i]; lnp[wid][1][f] = B[i]; }
      }
    }
#pragma unroll
    for (int q = 0; q < NR / 4; ++q) {
      const int f0 = 8 * q + 4 * h;
      const f32x4 hv = a.tiled ? load4_tiled<T, NR>(reinterpret_cast<const T*>(a.hpre), q, rr, h)  // M == H
                       : VEC ? load4(hp + f0) : load4_masked(hp, f0, M, false);
      f32x4 gm = {0.f, 0.f, 0.f, 0.f};
      if (VEC) gm = *reinterpret_cast<const f32x4*>(a.ln_g + f0);
      else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + e < M) gm[e] = a.ln_g[f0 + e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool in = VEC || f0 + e < M;
        const float xh = (hv[e] - mean) * rstd;
        A[4 * q + e] = in ? ln_bwd_out(A[4 * q + e], gm[e], c1, c2, xh, rstd) : 0.f;
      }
    }
  }
  // chain rule through the Linear / ReLU stack
  f32x16 acc[NT];
  BOp<T, NR> b;
  for (int l = a.nlin - 1; l >= 0; --l) {
    const int Ml = (l == a.nlin - 1) ? M : H;
    const int kuM = units_k<T>(Ml);
    if (a.gpre[l] && ((a.gpre_tiled >> l) & 1)) {
      store_row_tiled<T, NR>(reinterpret_cast<T*>(a.gpre[l]), A, row, h, valid);
    } else if (a.gpre[l]) {
      T* gp = reinterpret_cast<T*>(a.gpre[l]) + (size_t)row * Ml;
      if (VEC || (MODE == M_NOUT && l < a.nlin - 1)) store_row<T, NR, true>(gp, Ml, A, h, valid);
      else store_row<T, NR, false>(gp, Ml, A, h, valid);
    }
    b.set(A);
    if (l > 0) {
      __syncthreads();
      stage_block(wl, a.wtpk[l], kuM, 0, NT, 0, kuM);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
      __syncthreads();
      gemm<T, NT, NR, true>(acc, b, kuM, wl, kuM, NT, lane);
      cbarrier();
      acc_to_regs<NT, NR>(A, acc);
      if constexpr (!GACT) {
        // AGN_RELU_MASK sign bits (8 B per lane instead of the activation row)
        uint32_t mk[mask_dwords<NR>()];
        load_relu_mask<NR>(mk, a.mask[l - 1], min(wave, (a.rows - 1) / 32), lane);  // clamp: idle waves
#pragma unroll
        for (int i = 0; i < NR; ++i) A[i] = mask_sel(mk, i, A[i]);
      } else {
        // dL/dy rounded to T (the Linear backward's output in the storage type), times f'(x) at
        // the forward's saved pre-activation x
        const T* pb = reinterpret_cast<const T*>(a.pre[l - 1]);
#pragma unroll
        for (int q = 0; q < NR / 4; ++q) {
          const f32x4 x = a.tiled ? load4_tiled<T, NR>(pb, q, rr, h) : load4(pb + (size_t)rr * H + 8 * q + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) A[4 * q + e] = act_bwd<T>(a.act_fn, x[e], round_t<T>(A[4 * q + e]));
        }
      }
    } else {
      int koff = 0;
      for (int s = 0; s < a.din_nseg; ++s) {
        const int ks = a.din_k[s];
        if (a.din[s]) {
          const int otn = (ks + 31) / 32;
          __syncthreads();
          stage_block(wl, a.wtpk[0], kuM, koff / 32, otn, 0, kuM);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
          __syncthreads();
          gemm<T, NT, NR>(acc, b, kuM, wl, kuM, otn, lane);
          float v[NR];
          acc_to_regs<NT, NR>(v, acc);
          if (a.din_resid[s]) {
            cbarrier();
            float g[NR];
            load_grad<T, NR, MODE>(g, a, rr, valid, h);
#pragma unroll
            for (int i = 0; i < NR; ++i) v[i] += g[i];
          }
          T* dp = reinterpret_cast<T*>(a.din[s]) + (size_t)row * ks;
          if (MODE != M_GEN && ks == H) store_row<T, NR, true>(dp, ks, v, h, valid);
          else store_row<T, NR, false>(dp, ks, v, h, valid);
        }
        koff += ks;
      }
    }
  }
  if (a.use_ln && a.ln_partial) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * M; i += BLOCK) {
      const int q = i / M, f = i - q * M;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WPB; ++w) s += lnp[w][q][f];
      a.ln_partial[(size_t)blockIdx.x * 2 * M + i] = s;
    }
  }
}

// ------------------------------------------------------------------------- resident-weight kernels
// Persistent variants for the hot edge MLP (bf16, every layer H -> H, <= 4 Linears): all packed
// weights of the chain live in LDS for the whole launch (4 x 32 KB at H = 128), so the 8 waves of
// a block never synchronise after the prologue and each wave streams its own 32-row tiles —
// one wave's gathers overlap the other waves' MFMA chains. One block per CU.
constexpr int RES_WPB = 8;
constexpr int RES_BLOCK = 64 * RES_WPB;
constexpr int RES_MAXL = 4;
// LDS-staged g loads / de stores in the resident backward: coalesced, but at 256 VGPRs the extra
// live registers spill (measured: 2.55 -> 2.88 ms per launch with de staging), so both stay off
constexpr bool kStageGradIn = false;
constexpr bool kStageGradOut = false;

template <typename T, int NT>
constexpr int res_layer_units() { return NT * (nrk(32 * NT) / BOp<T, 16>::RPU) * 64; }

// XCD-aware tile walk: blocks b and b + 8 share an XCD (and its 4 MB L2), so each group of
// blocks {g, g+8, ...} walks one contiguous eighth of the tiles. Consecutive CSC edge tiles
// share receivers and nearby senders: their P_s/P_d rows are re-read from the same L2.
struct ResTiles {
  int first, end, step;
  AGN_DEV ResTiles(int ntiles, int wid) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int g = blockIdx.x & 7, bi = blockIdx.x >> 3, nb = gridDim.x >> 3;
      const int per = (ntiles + 7) / 8;
      first = g * per + bi * RES_WPB + wid;
      end = min(ntiles, (g + 1) * per);
      step = nb * RES_WPB;
    } else {
      first = blockIdx.x * RES_WPB + wid;
      end = ntiles;
      step = gridDim.x * RES_WPB;
    }
  }
};

// Diagnostic phase clocks of the resident edge forward (built with -DAGN_FWD_STAMPS into the
// separate stamps library only): the 8 waves of block 0 record s_memtime at 10 points of their
// first 8 tiles into agn_fwd_stamps[(wave * 8 + tile) * 16 + point].
#ifdef AGN_FWD_STAMPS
__device__ unsigned long long* agn_fwd_stamps;
#define FWD_STAMP(k)                                                                                   \
  do {                                                                                                 \
    if (agn_fwd_stamps && blockIdx.x == 0 && lane == 0 && ntile < 8)                                   \
      agn_fwd_stamps[((threadIdx.x >> 6) * 8 + ntile) * 16 + (k)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define FWD_STAMP(k) \
  do {               \
  } while (0)
#endif

#ifndef AGN_FWD_DEFER
#define AGN_FWD_DEFER 1  // resident edge forward: e' stores issue after the next tile's gathers
#endif

template <typename T, int NT>
__global__ __launch_bounds__(RES_BLOCK, 2) void mlp_fwd_res_kernel(const agn_mlp_fwd_args a) {
  constexpr int H = 32 * NT;
  constexpr int NR = 16 * NT;
  constexpr int NUH = nrk(H) / BOp<T, NR>::RPU;
  constexpr int LAYER = res_layer_units<T, NT>();
  __shared__ uint4 wres[RES_MAXL * LAYER];
  __shared__ __attribute__((aligned(16))) float pv[RES_MAXL + 2][H];  // biases, LN gamma, LN beta
  __shared__ uint4 stg[RES_WPB][8][H / 8 + STG_PAD];  // per-wave 8-row staging: coalesced e loads
  __shared__ int ids[RES_WPB][64];                     // per-wave next-tile src (lanes 0-31) / dst
  for (int l = 0; l < a.nlin; ++l) stage_block(wres + l * LAYER, a.wpk[l], NUH, 0, NT, 0, NUH);
  stage_params<H, RES_MAXL + 2>(pv, a.bias, a.nlin, a.ln_g, a.ln_b, RES_BLOCK);
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  const int ntiles = (a.rows + 31) / 32;
  const agn_seg& sg = a.seg[0];
  const ResTiles tw(ntiles, threadIdx.x >> 6);
  // The sender / receiver ids of the wave's next tile are loaded one tile ahead, so a tile's
  // projection-row gathers issue together with its e loads (one memory latency per tile, not two).
  // They reach the next tile through the wave's LDS slot, not a loop-carried register: a
  // loop-carried load result makes the compiler wait vmcnt(0) at the loop head, i.e. also for the
  // previous tile's e' stores. Lane l loads the src (l < 32) or dst (l >= 32) of row l & 31.
  int* wids = ids[threadIdx.x >> 6];
  const int32_t* const srcp = a.src;
  const int32_t* const dstp = a.dst;
  // (without projections the load reads the input rows instead: always a valid address, so the
  // next-id load below needs no branch - a conditional load leaves a register write at the loop
  // head that the compiler guards with vmcnt(0))
  const int32_t* const idp = a.proj ? (lane0 < 32 ? srcp : dstp) : reinterpret_cast<const int32_t*>(sg.ptr);
  auto tile_id = [&](int t) { return idp[min(t * 32 + (lane0 & 31), a.rows - 1)]; };
  if (a.proj && tw.first < tw.end) wids[lane0] = tile_id(tw.first);
#ifdef AGN_FWD_STAMPS
  int ntile = 0;
#endif
  // the previous tile's e' row, stored once this tile's loads have been consumed (PendingRow)
  PendingRow<NR / 8> pend;
  for (int tile = tw.first; tile < tw.end; tile += tw.step) {
    cbarrier();  // keep the (loop-invariant) LDS weight reads inside the loop: no LICM into VGPRs
    // the lane id behind a barrier each tile: lane-derived offsets (row addresses, staging and
    // weight-fragment offsets) are recomputed per tile instead of being hoisted and kept live
    const int lane = opaque_v(lane0);
    const int c = lane & 31, h = lane >> 5;
    FWD_STAMP(0);
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    f32x16 acc[NT];
    BOp<T, NR> b;
    // the projection rows are gathered and summed first, then the e tile goes through the staging
    // rows (issuing the e loads ahead of the gathers measured slower: DESIGN.md §9, round 3)
    const bool staged_in = sg.ld == H;
    uint4 eraw[NR / 8];
    const bool more = a.proj && tile + tw.step < tw.end;
    const int nid = tile_id(more ? tile + tw.step : tile);  // (unconditional: see tile_id)
    if (a.proj) {
      const int cs = wids[c], cd = wids[32 + c];
      const T* P = reinterpret_cast<const T*>(a.proj);
      // acc = P_s[src] + P_d[dst] on the matrix cores (exact fp32 add, common.hpp acc_add2_mfma)
      BOp<T, NR> xs, xd;
      {
        // gathers issued, then the previous tile's stores, then the gathered data used: the wait
        // for the gathers does not include the stores (PendingRow)
        uint4 rs[NR / 8], rd[NR / 8];
        const T* ps = P + (size_t)cs * (2 * H) + 8 * h;
        const T* pd = P + (size_t)cd * (2 * H) + H + 8 * h;
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) {
          rs[i] = *reinterpret_cast<const uint4*>(ps + 16 * i);
          rd[i] = *reinterpret_cast<const uint4*>(pd + 16 * i);
        }
        xs.set_w(rs);
        xd.set_w(rd);
      }
      bf16x8 f0, f1;
      ident_frags(f0, f1, lane);
      acc_add2_mfma<NT, NR>(acc, xs, xd, f0, f1);
    } else {
      acc_bias_lds<NT>(acc, pv[0], h);
    }
    FWD_STAMP(1);
    {
      if (staged_in) {  // coalesced 1-KB loads through the wave's LDS staging rows
        tile_load_issue<H / 8>(eraw, reinterpret_cast<const T*>(sg.ptr) + (size_t)tile * 32 * H, a.rows - tile * 32,
                               lane);
        uint4 mine[NR / 8];
        tile_load_finish<H / 8>(mine, eraw, stg[threadIdx.x >> 6], lane);
        b.set_w(mine);
      } else {
        b.load_w(reinterpret_cast<const T*>(sg.ptr) + (size_t)rr * sg.ld, h);
      }
    }
    // the residual is the layer input itself (e' = e + .., mgnLayer.py:205): keep the packed
    // operand instead of re-reading the row in the epilogue
    const bool res_in = a.resid == sg.ptr && a.out_ld == sg.ld;
    const BOp<T, NR> e0 = b;
    FWD_STAMP(2);
    gemm<T, NT, NR, true>(acc, b, NUH, wres, NUH, NT, lane);
    FWD_STAMP(3);
    if (AGN_FWD_DEFER) {
      // the previous tile's e' stores issue here, after this tile's loads have been consumed:
      // the next wait on a load is the next tile's, ~3/4 of a tile later, when they have completed
      cbarrier();
      pend.flush(h);
    }
    for (int l = 1; l < a.nlin; ++l) {
      cbarrier();
      b.template set_relu<NT>(acc);
      if (a.act[l - 1]) {
        if (a.tiled) b.store_tiled(reinterpret_cast<T*>(a.act[l - 1]), row, h, valid);
        else b.store(reinterpret_cast<T*>(a.act[l - 1]) + (size_t)row * H, h, valid);
      }
      if (a.mask[l - 1]) store_relu_mask<T, NR>(a.mask[l - 1], b, tile, lane);
      cbarrier();
      acc_bias_lds<NT>(acc, pv[l], h);
      FWD_STAMP(4 + 2 * (l - 1));
      gemm<T, NT, NR, true>(acc, b, NUH, wres + l * LAYER, NUH, NT, lane);
      FWD_STAMP(5 + 2 * (l - 1));
    }
    // epilogue: LayerNorm, residual, store (8 features per lane at a time)
    float mean = 0.f, rstd = 1.f;
    if (a.use_ln) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NR; ++i) s += acc[i / 16][i % 16];
      s = sum32(s);
      mean = s / (float)H;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < NR; i += 2) q = ln_sq_acc2(q, acc[i / 16][i % 16], acc[(i + 1) / 16][(i + 1) % 16], mean);
      q = sum32(q);
      rstd = 1.0f / sqrtf(q / (float)H + 1e-5f);
      if (a.stats && valid && h == 0) {
        a.stats[2 * (size_t)row] = mean;
        a.stats[2 * (size_t)row + 1] = rstd;
      }
    }
    FWD_STAMP(10);
    T* hp = a.hpre ? reinterpret_cast<T*>(a.hpre) + (size_t)row * H : nullptr;
    const T* rp = a.resid ? reinterpret_cast<const T*>(a.resid) + (size_t)rr * a.out_ld : nullptr;
    T* op = reinterpret_cast<T*>(a.out) + (size_t)row * a.out_ld;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
      if (a.use_ln) {
        if (hp) {
          if (a.tiled) store8_tiled<T, NR>(reinterpret_cast<T*>(a.hpre), i, row, h, v, valid);
          else store8_w(hp, i, h, v, valid);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int f0 = 16 * i + 8 * j + 4 * h;
          const f32x4 g4 = *reinterpret_cast<const f32x4*>(&pv[RES_MAXL][f0]);
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(&pv[RES_MAXL + 1][f0]);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {  // packed fp32: ln_out per element
            const f32x2 o = ln_out2(f2(v[4 * j + e], v[4 * j + e + 1]), mean, rstd, f2(g4[e], g4[e + 1]),
                                    f2(b4[e], b4[e + 1]));
            v[4 * j + e] = o[0];
            v[4 * j + e + 1] = o[1];
          }
        }
      }
      if (rp) {
        float r[8];
        if (res_in) e0.get8(r, i);
        else load8_w(r, rp, i, h);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {  // round_t(v) + r, the add packed
          const uint32_t p = pack2t<T>(v[e], v[e + 1]);
          const f32x2 o = f2(lo16<T>(p), hi16<T>(p)) + f2(r[e], r[e + 1]);
          v[e] = o[0];
          v[e + 1] = o[1];
        }
      }
      if (i == 0 && more) wids[lane] = nid;  // (the slot's reads are done: LDS is in order per wave)
      if (AGN_FWD_DEFER) pend.set(i, v);
      else store8_w(op, i, h, v, valid);  // direct 16-B stores (the staged 1-KB store measured slower)
    }
    if (AGN_FWD_DEFER) {
      pend.p = op;
      pend.valid = valid;
    }
    FWD_STAMP(11);
#ifdef AGN_FWD_STAMPS
    ++ntile;
#endif
  }
  if (AGN_FWD_DEFER) pend.flush(lane0 >> 5);
}

template <typename T, int NR>
AGN_DEV void load_grad_w(float (&g)[NR], const agn_mlp_bwd_args& a, int rr, bool valid, int h) {
  if (a.g) {
    load_row_w<T, NR>(g, reinterpret_cast<const T*>(a.g) + (size_t)rr * a.out_dim, h);
  } else {  // unused output: zero incoming gradient (no materialised zeros)
#pragma unroll
    for (int i = 0; i < NR; ++i) g[i] = 0.f;
  }
  if (a.g2) add_row_w<T, NR>(g, reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim, h);
  if (!valid) {
#pragma unroll
    for (int i = 0; i < NR; ++i) g[i] = 0.f;
  }
}

template <typename T, int NR>
AGN_DEV void add_grad_w(float (&v)[NR], const agn_mlp_bwd_args& a, int rr, int h) {
  // v += (g + g2): the incoming gradient is summed first, as autograd accumulates it
  const T* g = reinterpret_cast<const T*>(a.g) + (size_t)rr * a.out_dim;
  if (!a.g2 || !a.g) {
    if (a.g) add_row_w<T, NR>(v, g, h);
    else if (a.g2) add_row_w<T, NR>(v, reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim, h);
    return;
  }
  const T* g2 = reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim;
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    float x[8], y[8];
    load8_w(x, g, i, h);
    load8_w(y, g2, i, h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[8 * i + e] += x[e] + y[e];
  }
}

template <typename T, int NT>
__global__ __launch_bounds__(RES_BLOCK, 2) void mlp_bwd_res_kernel(const agn_mlp_bwd_args a) {
  static_assert(sizeof(T) == 2, "resident kernels are bf16-only");
  constexpr int H = 32 * NT;
  constexpr int NR = 16 * NT;
  constexpr int NP = (NR >= 32) ? NR / 32 : 1;
  constexpr int NUH = nrk(H) / BOp<T, NR>::RPU;
  constexpr int LAYER = res_layer_units<T, NT>();
  __shared__ uint4 wres[RES_MAXL * LAYER];
  __shared__ float lnp[RES_WPB][2][H];
  __shared__ __attribute__((aligned(16))) float pg_lds[H];  // LN gamma
  __shared__ uint4 stg[RES_WPB][8][H / 8 + STG_PAD];  // per-wave 8-row staging: coalesced g / de
  // layer 0's weights only serve dX: an encoder (narrow input, no input gradient) skips them
  // (res_bwd_ok: without dX every din pointer is NULL; with dX there is exactly one segment)
  for (int l = a.din[0] ? 0 : 1; l < a.nlin; ++l) stage_block(wres + l * LAYER, a.wtpk[l], NUH, 0, NT, 0, NUH);
  for (int i = threadIdx.x; i < H; i += RES_BLOCK) pg_lds[i] = a.use_ln ? a.ln_g[i] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int c = lane & 31, h = lane >> 5;
  const int wid = threadIdx.x >> 6;
  const int ntiles = (a.rows + 31) / 32;
  float pg[NP], pb[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const ResTiles tw(ntiles, wid);
  for (int tile = tw.first; tile < tw.end; tile += tw.step) {
    cbarrier();
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    float A[NR];
    if (kStageGradIn && a.g && a.out_dim == H) {  // incoming gradient: coalesced 1-KB loads through LDS
      uint4 mine[NR / 8];
      tile_load_chunks<H / 8>(mine, reinterpret_cast<const T*>(a.g) + (size_t)tile * 32 * H, a.rows - tile * 32,
                              stg[wid], lane);
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float o[8];
        unpack8_w(o, mine[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) A[8 * i + e] = o[e];
      }
      if (a.g2)
        add_row_w<T, NR>(A, reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim, h);
      if (!valid) {
#pragma unroll
        for (int i = 0; i < NR; ++i) A[i] = 0.f;
      }
    } else {
      load_grad_w<T, NR>(A, a, rr, valid, h);
    }
    if (a.use_ln) {
      const float mean = a.stats[2 * (size_t)rr], rstd = a.stats[2 * (size_t)rr + 1];
      const T* hp = reinterpret_cast<const T*>(a.hpre) + (size_t)rr * H;
      float B[NR];
      float c1 = 0.f, c2 = 0.f;
      // the pre-LN row is read once and kept packed (32 VGPRs) for both LN passes
      uint4 hraw[NR / 8];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        if (a.tiled) {
          hraw[i] = reinterpret_cast<const uint4*>(a.hpre)[tiled_unit<T, NR>(rr, i, h)];
        } else {
          float t8[8];
          load8_w(t8, hp, i, h);
          hraw[i] = __builtin_bit_cast(uint4, u32x4{pack2(t8[0], t8[1]), pack2(t8[2], t8[3]), pack2(t8[4], t8[5]),
                                                    pack2(t8[6], t8[7])});
        }
      }
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float hv[8];
        unpack8(hv, hraw[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 gm = *reinterpret_cast<const f32x4*>(pg_lds + 16 * i + 8 * j + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 8 * i + 4 * j + e;
            const float xh = (hv[4 * j + e] - mean) * rstd;
            ln_bwd_acc(c1, c2, A[r], gm[e], xh);
            B[r] = A[r] * xh;
          }
        }
      }
      c1 = sum32(c1);
      c2 = sum32(c2);
      c1 /= (float)H;
      c2 /= (float)H;
      if (a.ln_partial) {
        butterfly_reduce<NR>(B, lane);
#pragma unroll
        for (int i = 0; i < NP; ++i) pg[i] += B[i];
#pragma unroll
        for (int i = 0; i < NR; ++i) B[i] = A[i];
        butterfly_reduce<NR>(B, lane);
#pragma unroll
        for (int i = 0; i < NP; ++i) pb[i] += B[i];
      }
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float hv[8];
        unpack8(hv, hraw[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 gm = *reinterpret_cast<const f32x4*>(pg_lds + 16 * i + 8 * j + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 8 * i + 4 * j + e;
            const float xh = (hv[4 * j + e] - mean) * rstd;
            A[r] = ln_bwd_out(A[r], gm[e], c1, c2, xh, rstd);
          }
        }
      }
    }
    f32x16 acc[NT];
    BOp<T, NR> b;
    for (int l = a.nlin - 1; l >= 0; --l) {
      cbarrier();
      // AGN_RELU_MASK sign bits (res_bwd_ok: always given), issued before this layer's gpre store:
      // vmcnt retires in order, so a load issued after the store would wait for it to complete
      uint32_t mk[mask_dwords<NR>()];
      if (l > 0) load_relu_mask<NR>(mk, a.mask[l - 1], tile, lane);
      if (a.gpre[l]) {
        if ((a.gpre_tiled >> l) & 1) store_row_tiled<T, NR>(reinterpret_cast<T*>(a.gpre[l]), A, row, h, valid);
        else store_row_w<T, NR>(reinterpret_cast<T*>(a.gpre[l]) + (size_t)row * H, A, h, valid);
      }
      b.set(A);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
      if (l > 0) {
        gemm<T, NT, NR, true>(acc, b, NUH, wres + l * LAYER, NUH, NT, lane);
#pragma unroll
        for (int i = 0; i < NR; ++i) A[i] = mask_sel(mk, i, acc[i / 16][i % 16]);
      } else if (a.din[0]) {
        gemm<T, NT, NR, true>(acc, b, NUH, wres, NUH, NT, lane);
        if constexpr (!kStageGradOut) {
          float v[NR];
          acc_to_regs<NT, NR>(v, acc);
          if (a.din_resid[0]) add_grad_w<T, NR>(v, a, rr, h);
          store_row_w<T, NR>(reinterpret_cast<T*>(a.din[0]) + (size_t)row * H, v, h, valid);
          continue;
        }
        // de = W0^T gpre0 + (g + g2), packed pair by pair for the staged store
        const T* g1p = a.g ? reinterpret_cast<const T*>(a.g) + (size_t)rr * a.out_dim : nullptr;
        const T* g2p = a.g2 ? reinterpret_cast<const T*>(a.g2) + (size_t)(a.gidx ? a.gidx[rr] : rr) * a.out_dim
                            : nullptr;
        uint4 ob[NR / 8];
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = acc[(8 * i + e) / 16][(8 * i + e) % 16];
          if (a.din_resid[0]) {
            float x[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, y[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (g1p) load8_w(x, g1p, i, h);
            if (g2p) load8_w(y, g2p, i, h);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += x[e] + y[e];
          }
          ob[i] = pack8_w(o, h);
        }
        tile_store_chunks<H / 8>(ob, reinterpret_cast<T*>(a.din[0]) + (size_t)tile * 32 * H, a.rows - tile * 32,
                                 stg[wid], lane);
      }
    }
  }
  if (a.use_ln && a.ln_partial) {
    const bool canon = (NR >= 32) || ((c % (32 / (NR < 32 ? NR : 32))) == 0);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int f = feat_of((c * NR) / 32 + i, h);
      if (canon) { lnp[wid][0][f] = pg[i]; lnp[wid][1][f] = pb[i]; }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * H; i += RES_BLOCK) {
      const int q = i / H, f = i - q * H;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < RES_WPB; ++w) s += lnp[w][q][f];
      a.ln_partial[(size_t)blockIdx.x * 2 * H + i] = s;
    }
  }
}

// ------------------------------------------------------------------------- packing
// A operand of Y^T = A * X^T: A[r][k] = trans ? W[k][r] : W[r][k]  (W row-major, ld)
template <typename S>
AGN_DEV float wat(const S* w, int ld, int M, int K, int trans, int r, int k) {
  if (r >= M || k >= K) return 0.f;
  return trans ? to_f(w[(size_t)k * ld + r]) : to_f(w[(size_t)r * ld + k]);
}

template <typename S>
AGN_DEV void pack_one(const agn_pack_desc& d, int tid) {
  const S* w = reinterpret_cast<const S*>(d.src);
  if (d.rows == 0) {  // vector -> fp32
    if (tid < d.cols) reinterpret_cast<float*>(d.dst)[d.col_off + tid] = to_f(w[(size_t)tid * d.ld]);
    return;
  }
  const int OT = (d.rows + 31) / 32;
  const int lane = tid & 63;
  const int i = lane & 31, hh = lane >> 5;
  const int unit = tid >> 6;
  const int ot0 = d.row_off / 32;
  if (d.dst_dtype == AGN_BF16 || d.dst_dtype == AGN_F16) {
    const int KU = (d.cols + 15) / 16, KUT = (d.dst_cols + 15) / 16, ku0 = d.col_off / 16;
    if (unit >= OT * KU) return;
    const int ot = unit / KU, ku = unit % KU;
    const size_t at = ((size_t)(ot0 + ot) * KUT + ku0 + ku) * 64 + lane;
    if (d.dst_dtype == AGN_BF16) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (bf16)wat(w, d.ld, d.rows, d.cols, d.trans, 32 * ot + i, 16 * ku + 8 * (j >> 2) + 4 * hh + (j & 3));
      reinterpret_cast<bf16x8*>(d.dst)[at] = o;
    } else {
      f16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (f16)wat(w, d.ld, d.rows, d.cols, d.trans, 32 * ot + i, 16 * ku + 8 * (j >> 2) + 4 * hh + (j & 3));
      reinterpret_cast<f16x8*>(d.dst)[at] = o;
    }
  } else {
    const int KU = 2 * ((d.cols + 15) / 16), KUT = 2 * ((d.dst_cols + 15) / 16), ku0 = d.col_off / 8;
    if (unit >= OT * KU) return;
    const int ot = unit / KU, ku = unit % KU;
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = wat(w, d.ld, d.rows, d.cols, d.trans, 32 * ot + i, 8 * ku + 4 * hh + e);
    reinterpret_cast<f32x4*>(d.dst)[((size_t)(ot0 + ot) * KUT + ku0 + ku) * 64 + lane] = o;
  }
}

__global__ void pack_kernel(const agn_pack_desc* __restrict__ descs) {
  const agn_pack_desc d = descs[blockIdx.y];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  // only float32 / bfloat16 / float16 operands are packed (the descriptors live in device memory, so
  // the host wrapper (aerognn.core.Pack) rejects others; a stray one writes nothing here instead of
  // reinterpreting its bits)
  const auto ok = [](int t) { return t == AGN_F32 || t == AGN_BF16 || t == AGN_F16; };
  if (!ok(d.src_dtype) || !ok(d.dst_dtype)) return;
  if (d.src_dtype == AGN_BF16) pack_one<bf16>(d, tid);
  else if (d.src_dtype == AGN_F16) pack_one<f16>(d, tid);
  else pack_one<float>(d, tid);
}

__global__ void reduce_partials_kernel(const float* __restrict__ p, int nw, int n, float* __restrict__ out) {
  const int cidx = blockIdx.x * blockDim.x + threadIdx.x;
  if (cidx >= n) return;
  float s = 0.f;
  for (int w = 0; w < nw; ++w) s += p[(size_t)w * n + cidx];
  out[cidx] = s;
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

#define AGN_LAUNCH(KERNEL, T, NT, MODE)                                                              \
  do {                                                                                                \
    if (a->act_fn != AGN_ACT_RELU)                                                                    \
      hipLaunchKernelGGL((KERNEL<T, NT, MODE, true>), grid, dim3(BLOCK), 0, (hipStream_t)stream, *a);  \
    else                                                                                              \
      hipLaunchKernelGGL((KERNEL<T, NT, MODE, false>), grid, dim3(BLOCK), 0, (hipStream_t)stream, *a); \
  } while (0)

#define AGN_FWD_MODES(T, NT)                                   \
  switch (mode) {                                              \
    case M_VEC: AGN_LAUNCH(mlp_fwd_kernel, T, NT, M_VEC); break;   \
    case M_NIN: AGN_LAUNCH(mlp_fwd_kernel, T, NT, M_NIN); break;   \
    case M_NOUT: AGN_LAUNCH(mlp_fwd_kernel, T, NT, M_NOUT); break; \
    default: AGN_LAUNCH(mlp_fwd_kernel, T, NT, M_GEN); break;      \
  }
#define AGN_BWD_MODES(T, NT)                                   \
  switch (mode) {                                              \
    case M_VEC: AGN_LAUNCH(mlp_bwd_kernel, T, NT, M_VEC); break;   \
    case M_NOUT: AGN_LAUNCH(mlp_bwd_kernel, T, NT, M_NOUT); break; \
    default: AGN_LAUNCH(mlp_bwd_kernel, T, NT, M_GEN); break;      \
  }

#define AGN_DISPATCH(MODES)                                                   \
  do {                                                                        \
    if (a->dtype == AGN_F32) {                                                \
      if (a->hidden == 128) { MODES(float, 4) }                               \
      else if (a->hidden == 64) { MODES(float, 2) }                           \
      else if (a->hidden == 32) { MODES(float, 1) }                           \
      else return AGN_E_HIDDEN;                                               \
    } else if (a->dtype == AGN_BF16) {                                        \
      if (a->hidden == 128) { MODES(bf16, 4) }                                \
      else if (a->hidden == 64) { MODES(bf16, 2) }                            \
      else if (a->hidden == 32) { MODES(bf16, 1) }                            \
      else return AGN_E_HIDDEN;                                               \
    } else if (a->dtype == AGN_F16) {                                         \
      if (a->hidden == 128) { MODES(f16, 4) }                                 \
      else if (a->hidden == 64) { MODES(f16, 2) }                             \
      else if (a->hidden == 32) { MODES(f16, 1) }                             \
      else return AGN_E_HIDDEN;                                               \
    } else {                                                                  \
      return AGN_E_DTYPE;                                                     \
    }                                                                         \
  } while (0)

namespace {
int g_cus = 0;
int num_cus() {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) g_cus = p.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  return g_cus;
}
int res_blocks(int rows) {
  const int tiles = (rows + 31) / 32;
  const int need = (tiles + RES_WPB - 1) / RES_WPB;
  const int cap = num_cus();  // 128 KB of resident weights: one block per CU
  return need < cap ? (need > 0 ? need : 1) : cap;
}
inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }
bool fwd_ptrs_aligned(const agn_mlp_fwd_args* a) {
  bool ok = al16(a->out) && al16(a->resid) && al16(a->proj) && al16(a->hpre);
  for (int s = 0; s < a->nseg; ++s) ok = ok && al16(a->seg[s].ptr) && al16(a->seg[s].store);
  for (int l = 0; l < a->nlin; ++l) ok = ok && al16(a->act[l]);
  return ok;
}
bool bwd_ptrs_aligned(const agn_mlp_bwd_args* a) {
  bool ok = al16(a->g) && al16(a->g2) && al16(a->hpre);
  for (int s = 0; s < a->din_nseg; ++s) ok = ok && al16(a->din[s]);
  for (int l = 0; l < a->nlin; ++l) ok = ok && al16(a->gpre[l]);
  return ok;
}
int g_opt_resident = 1;
bool res_fwd_ok(const agn_mlp_fwd_args* a, bool vec) {
  return g_opt_resident && vec && a->act_fn == AGN_ACT_RELU && a->dtype == AGN_BF16 && a->hidden == 128 && a->nlin <= RES_MAXL && a->nseg == 1 &&
         a->seg[0].kind == AGN_SEG_PLAIN && a->seg[0].k == 128 && a->out_dim == 128 && a->out_ld == 128 &&
         a->seg[0].ld % 8 == 0 && a->rows >= 64 * 1024;
}
bool res_bwd_ok(const agn_mlp_bwd_args* a, bool vec) {
  // edge/node chains with an H-wide dX, or any chain without dX (the edge encoder: d_e = 4 in)
  bool need_dx = false;
  for (int s = 0; s < a->din_nseg; ++s) need_dx |= a->din[s] != nullptr;
  // nlin == 1 with LayerNorm and no dX: the LayerNorm backward alone (G3 for agn_edge_bwd_fused)
  const bool din_ok = need_dx ? (a->din_nseg == 1 && a->in_dim == 128 && a->din_k[0] == 128)
                              : (a->nlin > 1 || a->use_ln);
  return g_opt_resident && vec && a->act_fn == AGN_ACT_RELU && a->dtype == AGN_BF16 && a->hidden == 128 &&
         a->nlin <= RES_MAXL && a->out_dim == 128 && din_ok && a->rows >= 64 * 1024;
}
}  // namespace

#ifdef AGN_FWD_STAMPS
extern "C" int agn_debug_fwd_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(agn_fwd_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

namespace agn {
bool node32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc);  // node32_fwd.hip
bool enc32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc);   // enc32_fwd.hip
bool dec32_fwd_try(const agn_mlp_fwd_args* a, void* stream, int* rc);   // enc32_fwd.hip
bool node32_bwd_try(const agn_mlp_bwd_args* a, void* stream, int* rc, int* ln_rows);  // node32_bwd.hip
bool dec32_bwd_try(const agn_mlp_bwd_args* a, void* stream, int* rc);                  // node32_bwd.hip
}

extern "C" {

int agn_version(void) { return 1; }

int agn_set_option(int key, int value) {
  if (key == AGN_OPT_RESIDENT) {
    const int old = g_opt_resident;
    g_opt_resident = value ? 1 : 0;
    return old;
  }
  return AGN_E_ARG;
}

const char* agn_error_string(int code) {
  switch (code) {
    case 0: return "success";
    case AGN_E_ARG: return "invalid argument";
    case AGN_E_DTYPE: return "unsupported dtype (f32 / bf16 / f16)";
    case AGN_E_HIDDEN: return "unsupported hidden size (32, 64, 128)";
    case AGN_E_SHAPE: return "unsupported shape";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

size_t agn_packed_bytes(int m, int k, int dtype) {
  return (size_t)((m + 31) / 32) * ((k + 15) / 16) * 1024 * (dtype == AGN_F32 ? 2 : 1);
}

int agn_pack(const agn_pack_desc* descs_device, int n, int max_threads, void* stream) {
  if (n <= 0) return 0;
  if (max_threads <= 0) return AGN_E_ARG;
  dim3 grid((max_threads + 255) / 256, n);
  hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, (hipStream_t)stream, descs_device);
  return launch_status();
}

int agn_mlp_bwd_nwaves(int rows) {
  const int waves = (rows + 31) / 32;
  return (waves + WPB - 1) / WPB;
}

int agn_mlp_forward(const agn_mlp_fwd_args* a, void* stream) {
  if (!a || a->rows < 0 || a->nlin < 1 || a->nlin > AGN_MAX_LIN || a->nseg < 1 || a->nseg > AGN_MAX_SEG)
    return AGN_E_ARG;
  if (a->rows == 0) return 0;
  const bool out_full =
      (a->out_ld % 8 == 0) && (a->nlin == 1 ? (a->out_dim % a->hidden == 0) : (a->out_dim == a->hidden));
  bool in_full = true;
  for (int s = 0; s < a->nseg; ++s) {
    if (a->seg[s].k < 1 || a->seg[s].k > a->hidden) return AGN_E_SHAPE;
    if (s + 1 < a->nseg && (a->seg[s].k % 32) != 0) return AGN_E_SHAPE;
    if (a->seg[s].k != a->hidden || a->seg[s].ld % 8 != 0) in_full = false;
  }
  if (a->nlin > 1 && a->out_dim > a->hidden) return AGN_E_SHAPE;
  if (a->use_ln && a->out_dim > a->hidden) return AGN_E_SHAPE;
  if (a->act_fn < AGN_ACT_RELU || a->act_fn > AGN_ACT_TANH) return AGN_E_ARG;
  for (int l = 0; l < a->nlin; ++l)
    if (!al16(a->act[l]) || !al16(a->pre[l])) return AGN_E_ARG;  // activation buffers are always 16-B accessed
  int mode = M_GEN;
  if (fwd_ptrs_aligned(a)) {
    if (in_full && out_full) mode = M_VEC;
    else if (out_full && a->nseg == 1 && (a->seg[0].kind == AGN_SEG_PLAIN || a->seg[0].kind == AGN_SEG_GATHER) &&
             a->seg[0].k <= 16)
      mode = M_NIN;
    else if (in_full && a->nlin > 1 && a->out_dim <= 32 && !a->use_ln) mode = M_NOUT;
  }
  const bool vec = mode == M_VEC;
  if (g_opt_resident && vec) {  // a processor layer's node MLP: resident weights, aggregation walked in
    int rc = 0;
    if (agn::node32_fwd_try(a, stream, &rc)) return rc;
  }
  if (g_opt_resident && mode == M_NIN) {  // an encoder on narrow rows: resident weights
    int rc = 0;
    if (agn::enc32_fwd_try(a, stream, &rc)) return rc;
  }
  if (g_opt_resident && mode == M_NOUT) {  // the decoder to <= 32 outputs: resident weights
    int rc = 0;
    if (agn::dec32_fwd_try(a, stream, &rc)) return rc;
  }
  if (res_fwd_ok(a, vec)) {
    dim3 g(res_blocks(a->rows));
    hipLaunchKernelGGL((mlp_fwd_res_kernel<bf16, 4>), g, dim3(RES_BLOCK), 0, (hipStream_t)stream, *a);
    return launch_status();
  }
  dim3 grid(agn_mlp_bwd_nwaves(a->rows));
  AGN_DISPATCH(AGN_FWD_MODES);
  return launch_status();
}

int agn_mlp_backward(const agn_mlp_bwd_args* a, void* stream) {
  if (!a || a->rows < 0 || a->nlin < 1 || a->nlin > AGN_MAX_LIN || a->din_nseg < 0 || a->din_nseg > AGN_MAX_SEG)
    return AGN_E_ARG;
  if (a->rows == 0) return 0;
  if (a->out_dim > a->hidden) return AGN_E_SHAPE;
  for (int s = 0; s < a->din_nseg; ++s) {
    if (a->din_k[s] > a->hidden) return AGN_E_SHAPE;
    if (s + 1 < a->din_nseg && (a->din_k[s] % 32) != 0) return AGN_E_SHAPE;
  }
  if (a->act_fn < AGN_ACT_RELU || a->act_fn > AGN_ACT_TANH) return AGN_E_ARG;
  for (int l = 0; l + 1 < a->nlin; ++l) {
    // the ReLU backward reads the sign bits (AGN_RELU_MASK), the others the saved pre-activation
    if (a->act_fn == AGN_ACT_RELU ? !a->mask[l] : (!a->pre[l] || !al16(a->pre[l]))) return AGN_E_ARG;
    if (a->act_fn != AGN_ACT_RELU && a->tiled == 0 && a->hidden % 4) return AGN_E_SHAPE;
  }
  int mode = M_GEN;
  if (bwd_ptrs_aligned(a)) {
    if (a->out_dim == a->hidden) mode = M_VEC;
    else if (a->out_dim <= 32 && !a->use_ln) mode = M_NOUT;
  }
  const bool vec = mode == M_VEC;
  agn_mlp_bwd_args* am = const_cast<agn_mlp_bwd_args*>(a);
  if (g_opt_resident && vec) {  // a processor layer's node MLP: resident weights
    int rc = 0, lr = 0;
    if (agn::node32_bwd_try(a, stream, &rc, &lr)) {
      am->ln_rows = lr;
      return rc;
    }
  }
  if (g_opt_resident && mode == M_NOUT) {  // the decoder from H-wide rows: resident weights
    int rc = 0;
    if (agn::dec32_bwd_try(a, stream, &rc)) {
      am->ln_rows = (int)agn_mlp_bwd_nwaves(a->rows);
      return rc;
    }
  }
  if (res_bwd_ok(a, vec)) {
    dim3 g(res_blocks(a->rows));
    am->ln_rows = (int)g.x;
    hipLaunchKernelGGL((mlp_bwd_res_kernel<bf16, 4>), g, dim3(RES_BLOCK), 0, (hipStream_t)stream, *a);
    return launch_status();
  }
  dim3 grid(agn_mlp_bwd_nwaves(a->rows));
  am->ln_rows = (int)grid.x;
  AGN_DISPATCH(AGN_BWD_MODES);
  return launch_status();
}

int agn_reduce_partials(const float* partial, int nw, int n, float* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     partial, nw, n, out);
  return launch_status();
}

}  // extern "C"
