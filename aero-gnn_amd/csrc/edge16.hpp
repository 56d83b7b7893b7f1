// Shared device code of the 16-row-tile sum-trick edge chain (gfx950, bf16, H = 128):
// the forward (edge16_fwd.hip) and the fused training backward (edge16_bwd.hip).
//
// Reference chain (models/mgnLayer.py:72-105, residual :205):
//   h0 = e W_e^T + P_s[src] + P_d[dst];  a1 = relu(h0); h1 = a1 W1^T + b1; a2 = relu(h1);
//   h2 = a2 W2^T + b2; a3 = relu(h2); h3 = a3 W3^T + b3; e' = e + LN(h3).
//
// Tile layout ("16-row tiles"): a wave owns 16 rows; lane l holds row r = l & 15 and column
// group g = l >> 4. Every product runs on v_mfma_f32_16x16x32_bf16 as the TRANSPOSED product
// Y^T = W X^T (cdna_hip_programming.md §3: A[m = l&15][k = 8g + j], B[k = 8g + j][n = l&15],
// D[4g + i][l&15]):
//   * operand (Op): k-step t holds features 32t + 8g + j (j = 0..7) of the lane's row: natural
//     order, so a row's 16-B chunk 4t + g IS the fragment (no lane exchange on loads / stores);
//   * accumulator (acc[ob], ob = 0..7): register i holds feature 32(ob>>1) + 8g + 4(ob&1) + i,
//     i.e. the A rows of output block ob are the weight rows o(ob, m) = 32(ob>>1) + 8(m>>2) +
//     4(ob&1) + (m&3), chosen so that blocks 2s and 2s+1 ARE the next layer's k-step s operand.
// Both kernels call the same helpers in the same order, so the backward's forward recompute is
// bitwise the forward kernel's h0..h3, LayerNorm statistics and ReLU masks.
//
// LDS weight image (one per Linear, 32 KB, natural [out][in] rows of 256 B): 8-byte piece hf of
// 16-B chunk c of row o at  256 o + 16 (c ^ fw(o)) + 8 (hf ^ (o & 1)),  fw(o) = 4 o1 ^ 8 o3 ^ 2 o4
// (o_b = bit b of o). Row-fragment reads (two ds_read_b64 per forward A fragment) and transposed
// reads (ds_read_b64_tr_b16 pairs for the backward's W^T fragments) are both conflict-free
// (checked against the MI355X_MICROARCH.md §LDS lane groups). The swizzle only involves lane
// bits, so every read is (lane base) XOR (a k-step / block constant) + an immediate.
#pragma once
#include "common.hpp"

namespace agn {
namespace e16 {

constexpr int H = 128;
constexpr int IMG_B = H * H * 2;  // one 128 x 128 bf16 image (32 KB)
#ifndef AGN_E16_PF
#define AGN_E16_PF 2
#endif
constexpr int PF = AGN_E16_PF;    // weight fragments in flight per product (4 registers each)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct Op {
  bf16x8 u[4];
};

AGN_DEV int fw_swz(int o) { return (((o >> 1) & 1) << 2) ^ (((o >> 3) & 1) << 3) ^ (((o >> 4) & 1) << 1); }
AGN_DEV int wimg(int o, int c, int hf) { return 256 * o + 16 * (c ^ fw_swz(o)) + 8 * (hf ^ (o & 1)); }

// weight images from the packed forward operands (agn_pack trans = 0: unit (ot, ku, lane) holds
// W[32 ot + lane%32][16 ku + 8(j>>2) + 4(lane/32) + (j&3)], j = 0..7): the two 4-feature pieces of a
// unit are natural chunks 2ku (j < 4) and 2ku + 1, half lane/32
AGN_DEV void load_images(char* lds, const void* const (&wpk)[4], int tid, int nthr) {
  for (int l = 0; l < 4; ++l) {
    const uint4* src = reinterpret_cast<const uint4*>(wpk[l]);
    char* img = lds + l * IMG_B;
    for (int u = tid; u < 2048; u += nthr) {
      const int ln = u & 63, unit = u >> 6;
      const int o = 32 * (unit >> 3) + (ln & 31), ku = unit & 7, hh = ln >> 5;
      const uint4 v = src[u];
      *reinterpret_cast<uint2*>(img + wimg(o, 2 * ku, hh)) = uint2{v.x, v.y};
      *reinterpret_cast<uint2*>(img + wimg(o, 2 * ku + 1, hh)) = uint2{v.z, v.w};
    }
  }
}

AGN_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
AGN_DEV bf16x8 frag2(uint2 lo, uint2 hi) { return __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y}); }
AGN_DEV uint2 tr64(const char* p) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p)));
}

AGN_DEV int fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
// a wave-uniform byte offset kept in an SGPR behind a compiler barrier: image bases past the 16-bit
// ds offset range are then added per use (v_add with an SGPR) instead of being materialised once
// into VGPRs that stay live across the whole tile loop
AGN_DEV int sfresh(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
// acc[ob] += W[rows of block ob] . X^T over k-steps t = 0..3 (each element sums its k-steps in
// ascending t). Lane (m, g) reads row o(ob, m), chunk 4t + g: the lane base of t = 0 XOR 64 t,
// the block as an immediate (its row offset leaves the swizzle bits alone).
AGN_DEV void gemm_fwd(f32x4 (&acc)[8], const Op& x, const char* lds, int img_off, int lane) {
  const char* img = lds + sfresh(img_off);
  const int m = lane & 15, g = lane >> 4;
  const int base = wimg(8 * (m >> 2) + (m & 3), g, 0);
  // fragments stream two (t, ob) steps ahead (8 registers in flight); the scheduling barriers keep
  // the compiler from hoisting all 64 reads of the product (registers it does not have)
  auto frag = [&](int idx) {
    const int t = idx >> 3, ob = idx & 7;
    const int ro = 256 * (32 * (ob >> 1) + 4 * (ob & 1));
#ifdef AGN_E16_NOLDS  // diagnostic: no fragment reads (timing only; results wrong)
    return __builtin_bit_cast(bf16x8, uint4{(uint32_t)(base + ro), (uint32_t)t, 0u, 0u});
#endif
    const uint2 lo = *reinterpret_cast<const uint2*>(img + (base ^ (64 * t)) + ro);
    const uint2 hi = *reinterpret_cast<const uint2*>(img + (base ^ (64 * t) ^ 8) + ro);
    return frag2(lo, hi);
  };
  bf16x8 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = frag(i);
#pragma unroll
  for (int idx = 0; idx < 32; ++idx) {
    const bf16x8 cur = f[idx % PF];
    if (idx + PF < 32) f[idx % PF] = frag(idx + PF);
    acc[idx & 7] = mfma16(cur, x.u[idx >> 3], acc[idx & 7]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// gemm_fwd for NH 16-row halves of a wave at once: each weight fragment read from LDS feeds NH
// MFMAs (one per half), so the LDS traffic per row falls by NH. Every accumulator sums its k-steps
// in gemm_fwd's order: the results are bitwise gemm_fwd's.
template <int NH>
AGN_DEV void gemm_fwd_n(f32x4 (&acc)[NH][8], const Op (&x)[NH], const char* lds, int img_off, int lane) {
  const char* img = lds + sfresh(img_off);
  const int m = lane & 15, g = lane >> 4;
  const int base = wimg(8 * (m >> 2) + (m & 3), g, 0);
  auto frag = [&](int idx) {
    const int t = idx >> 3, ob = idx & 7;
    const int ro = 256 * (32 * (ob >> 1) + 4 * (ob & 1));
    const uint2 lo = *reinterpret_cast<const uint2*>(img + (base ^ (64 * t)) + ro);
    const uint2 hi = *reinterpret_cast<const uint2*>(img + (base ^ (64 * t) ^ 8) + ro);
    return frag2(lo, hi);
  };
  bf16x8 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = frag(i);
#pragma unroll
  for (int idx = 0; idx < 32; ++idx) {
    const bf16x8 cur = f[idx % PF];
    if (idx + PF < 32) f[idx % PF] = frag(idx + PF);
#pragma unroll
    for (int h = 0; h < NH; ++h) acc[h][idx & 7] = mfma16(cur, x[h].u[idx >> 3], acc[h][idx & 7]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// acc[ib] = W^T[rows of block ib] . G^T (from zero; t ascending). A[m][k = 8g + j] =
// W[32t + 8g + j][in(ib, m)]: per 16-lane group g, lane 4q + p supplies row 32t + 8g + q (+4 for
// j >= 4) at the 4 columns in(ib, 4p..4p+3) = 32(ib>>1) + 8p + 4(ib&1) + 0..3 (chunk 4(ib>>1) + p,
// half ib&1); lane m receives column m of the 4 rows (element q = row q).
AGN_DEV void gemm_bwd(f32x4 (&acc)[8], const Op& gop, const char* lds, int img_off, int lane) {
  const char* img = lds + sfresh(img_off);
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int base = wimg(8 * g + q, p, 0);
  auto frag = [&](int idx) {
    const int ib = idx >> 2, t = idx & 3;
#ifdef AGN_E16_NOLDS
    return __builtin_bit_cast(bf16x8, uint4{(uint32_t)(base + ib), (uint32_t)t, 0u, 0u});
#endif
    const char* pb = img + (base ^ (64 * (ib >> 1)) ^ (8 * (ib & 1)));
    return frag2(tr64(pb + 8192 * t), tr64(pb + 8192 * t + 1024));
  };
  bf16x8 f[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) f[i] = frag(i);
#pragma unroll
  for (int idx = 0; idx < 32; ++idx) {
    const bf16x8 cur = f[idx % PF];
    if (idx + PF < 32) f[idx % PF] = frag(idx + PF);
    const int ib = idx >> 2, t = idx & 3;
    acc[ib] = t == 0 ? mfma16(cur, gop.u[0], f32x4{}) : mfma16(cur, gop.u[t], acc[ib]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// acc = a bias vector (fp32 [H] in LDS): block ob's 4 features are contiguous
AGN_DEV void bias_init(f32x4 (&acc)[8], const float* pv, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) acc[ob] = *reinterpret_cast<const f32x4*>(pv + 32 * (ob >> 1) + 8 * g + 4 * (ob & 1));
}

AGN_DEV uint32_t pk(float x, float y) { return pack2(x, y); }
// the next k-step operand from blocks 2s, 2s+1 (bf16 RNE, one v_cvt_pk per pair)
AGN_DEV void pack_op(Op& o, const f32x4 (&acc)[8]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
    o.u[s] = __builtin_bit_cast(bf16x8, u32x4{pk(acc[2 * s][0], acc[2 * s][1]), pk(acc[2 * s][2], acc[2 * s][3]),
                                              pk(acc[2 * s + 1][0], acc[2 * s + 1][1]),
                                              pk(acc[2 * s + 1][2], acc[2 * s + 1][3])});
}
// relu(round(acc)) packed (common.hpp relu_pk16: int16 max with 0 on the packed pair)
AGN_DEV void relu_op(Op& o, const f32x4 (&acc)[8]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
    o.u[s] = __builtin_bit_cast(
        bf16x8, u32x4{relu_pk16(pk(acc[2 * s][0], acc[2 * s][1])), relu_pk16(pk(acc[2 * s][2], acc[2 * s][3])),
                      relu_pk16(pk(acc[2 * s + 1][0], acc[2 * s + 1][1])),
                      relu_pk16(pk(acc[2 * s + 1][2], acc[2 * s + 1][3]))});
}
// G_{L-1} = round(dA) . [a_L > 0]: relu outputs are +0 or positive int16 patterns, so (0 - a) >> 15
// is 0xffff exactly where a > 0 (built on the whole short8 vector: the per-dword short2 form is
// miscompiled by this hipcc)
AGN_DEV void relu_select(Op& o, const f32x4 (&acc)[8], const Op& act) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const u32x4 m = __builtin_bit_cast(u32x4, (s16x8{} - __builtin_bit_cast(s16x8, act.u[s])) >> 15);
    const u32x4 w = {pk(acc[2 * s][0], acc[2 * s][1]) & m[0], pk(acc[2 * s][2], acc[2 * s][3]) & m[1],
                     pk(acc[2 * s + 1][0], acc[2 * s + 1][1]) & m[2], pk(acc[2 * s + 1][2], acc[2 * s + 1][3]) & m[3]};
    o.u[s] = __builtin_bit_cast(bf16x8, w);
  }
}

// a row's 64 bytes of this lane (chunks 4t + g) as the operand
AGN_DEV void load_op(Op& o, const bf16* rowp, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) o.u[t] = *reinterpret_cast<const bf16x8*>(rowp + 32 * t + 8 * g);
}
AGN_DEV void load_raw(uint4 (&o)[4], const bf16* rowp, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = *reinterpret_cast<const uint4*>(rowp + 32 * t + 8 * g);
}
AGN_DEV void store_raw(bf16* rowp, const uint4 (&o)[4], int lane, bool valid) {
  const int g = lane >> 4;
  if (valid) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<uint4*>(rowp + 32 * t + 8 * g) = o[t];
  }
}
AGN_DEV void store_op(bf16* rowp, const Op& o, int lane, bool valid) {
  const int g = lane >> 4;
  if (valid) {
#pragma unroll
    for (int t = 0; t < 4; ++t) *reinterpret_cast<bf16x8*>(rowp + 32 * t + 8 * g) = o.u[t];
  }
}
// element e (0..3) of block ob from a raw chunk set: chunk ob>>1, elements 4(ob&1) + e
AGN_DEV float raw_el(const uint4 (&r)[4], int ob, int e) {
  const u32x4 x = __builtin_bit_cast(u32x4, r[ob >> 1]);
  const uint32_t w = x[2 * (ob & 1) + (e >> 1)];
  return (e & 1) ? hi_bf16(w) : lo_bf16(w);
}
AGN_DEV float op_el(const Op& o, int ob, int e) {
  const u32x4 x = __builtin_bit_cast(u32x4, o.u[ob >> 1]);
  const uint32_t w = x[2 * (ob & 1) + (e >> 1)];
  return (e & 1) ? hi_bf16(w) : lo_bf16(w);
}

// acc = P_s[src] + P_d[dst] (exact fp32 sums of the bf16 rows)
AGN_DEV void acc_sum2(f32x4 (&acc)[8], const uint4 (&x)[4], const uint4 (&y)[4]) {
#pragma unroll
  for (int ob = 0; ob < 8; ++ob)
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
      const f32x2 s = f2(raw_el(x, ob, e), raw_el(x, ob, e + 1)) + f2(raw_el(y, ob, e), raw_el(y, ob, e + 1));
      acc[ob][e] = s[0];
      acc[ob][e + 1] = s[1];
    }
}

// sum of v over the 4 lanes of a row (l, l^16, l^32, l^48): (v_g0 + v_g1) + (v_g2 + v_g3) on every
// lane, bitwise equal across the four (v_permlane16/32_swap of v with itself, no selects)
AGN_DEV float sum4(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// LayerNorm statistics of the row in acc (eps 1e-5, mgnLayer.py / nn.LayerNorm), explicit fmas
// (common.hpp ln_sq_acc2) so every kernel rounds alike
AGN_DEV void ln_stats(const f32x4 (&acc)[8], float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int ob = 0; ob < 8; ++ob)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += acc[ob][e];
  s = sum4(s);
  mean = s / (float)H;
  float q = 0.f;
#pragma unroll
  for (int ob = 0; ob < 8; ++ob)
#pragma unroll
    for (int e = 0; e < 4; e += 2) q = ln_sq_acc2(q, acc[ob][e], acc[ob][e + 1], mean);
  q = sum4(q);
  rstd = 1.0f / sqrtf(q / (float)H + 1e-5f);
}

// XCD-grouped walk over units of work (blocks b and b + 8 share an XCD and its L2): each group
// {g, g+8, ...} of workgroups takes one contiguous eighth of the units
struct Walk {
  int first, end, step;
  AGN_DEV Walk(int nunits, int sub, int nsub) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int grp = blockIdx.x & 7, per = (nunits + 7) / 8;
      first = grp * per + (blockIdx.x >> 3) * nsub + sub;
      end = min(nunits, (grp + 1) * per);
      step = (gridDim.x >> 3) * nsub;
    } else {
      first = blockIdx.x * nsub + sub;
      end = nunits;
      step = gridDim.x * nsub;
    }
  }
};

AGN_DEV void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
template <typename V> AGN_DEV void opaque(V& v) { asm volatile("" : "+v"(v)); }
AGN_DEV void pin(Op& o) {
#pragma unroll
  for (int i = 0; i < 4; ++i) opaque(o.u[i]);
}

}  // namespace e16
}  // namespace agn
