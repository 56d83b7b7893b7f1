// Common device helpers for the aero-gnn MI355X (gfx950) kernels.
//
// Fragment convention used by every fused MLP kernel ("rows on lanes"):
//   A wave owns 32 data rows (edges or nodes). Lane l holds data row c = l & 31 and
//   feature half h = l >> 5. A [32 x F] activation tile lives in registers as
//   "acc layout": register rho holds feature f(rho, h) = 8*(rho >> 2) + 4*h + (rho & 3).
//   That is exactly the C/D layout of v_mfma_f32_32x32x{16_bf16, 2_f32} when the MFMA
//   computes the TRANSPOSED product  Y^T[out x rows] = W[out x K] * X^T[K x rows]
//   (col = lane & 31 = data row, row = out feature), so a layer's accumulator is fed
//   to the next layer's MFMA as its B operand with no LDS round trip and no shuffles
//   (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
//   The K order inside each MFMA step is permuted accordingly; weights are pre-packed
//   into that order (pack kernel) so each lane reads its A fragment with one 16-B load.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "aerognn.h"

typedef __bf16 bf16;
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16;
typedef f16 f16x2 __attribute__((ext_vector_type(2)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define AGN_DEV __device__ __forceinline__

namespace agn {

enum { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

// ---------------------------------------------------------------- element access
AGN_DEV float to_f(float v) { return v; }
AGN_DEV float to_f(bf16 v) { return (float)v; }
AGN_DEV float to_f(f16 v) { return (float)v; }
template <typename T> AGN_DEV T from_f(float v);
template <> AGN_DEV float from_f<float>(float v) { return v; }
template <> AGN_DEV bf16 from_f<bf16>(float v) { return (bf16)v; }
template <> AGN_DEV f16 from_f<f16>(float v) { return (f16)v; }

// round-trip through storage type T (what a stored-then-reloaded value looks like)
template <typename T> AGN_DEV float round_t(float v) { return to_f(from_f<T>(v)); }

AGN_DEV f32x4 load4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
AGN_DEV f32x4 load4(const bf16* p) {
  bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
AGN_DEV f32x4 load4(const f16* p) {
  f16x4 v = *reinterpret_cast<const f16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
AGN_DEV void store4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
AGN_DEV void store4(f16* p, f32x4 v) {
  f16x4 b = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
  *reinterpret_cast<f16x4*>(p) = b;
}
AGN_DEV void store4(bf16* p, f32x4 v) {
  bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *reinterpret_cast<bf16x4*>(p) = b;
}

// Masked 4-wide load: features f0..f0+3 of a row with `k` valid features.
template <typename T>
AGN_DEV f32x4 load4_masked(const T* row, int f0, int k, bool vec_ok) {
  if (vec_ok && f0 + 3 < k) return load4(row + f0);
  f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (f0 + q < k) r[q] = to_f(row[f0 + q]);
  return r;
}
template <typename T>
AGN_DEV void store4_masked(T* row, int f0, int k, bool vec_ok, f32x4 v) {
  if (vec_ok && f0 + 3 < k) { store4(row + f0, v); return; }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (f0 + q < k) row[f0 + q] = from_f<T>(v[q]);
}

// ---------------------------------------------------------------- 16-B row I/O (acc layout)
// A full row of H features in acc layout is split over lanes c and c+32 in 4-feature chunks
// (group q: features 8q+4h..8q+4h+3). For bf16 that is 8 B per lane per access; exchanging
// halves with v_permlane32_swap (cdna_hip_programming.md T21) lets each lane move 8
// contiguous features (16 B) instead: pair i = groups (2i, 2i+1) = features 16i..16i+15,
// lane half h reads/writes features 16i+8h..16i+8h+7. Every lane must execute these
// (uniform control flow); `valid` only masks the final store.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef bf16 bf16x2 __attribute__((ext_vector_type(2)));

AGN_DEV void swap_halves(uint32_t& a, uint32_t& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
// One v_cvt_pk_bf16_f32 per pair (RNE per element, the same rounding as two scalar casts). Built
// with a vector convert: the scalar-cast form {(bf16)x, (bf16)y} lowers to two single-source
// conversions plus a v_perm once the pair feeds integer ops (relu_pk16), 3 VALU instead of 1.
typedef float f32x2 __attribute__((ext_vector_type(2)));
AGN_DEV uint32_t pack2(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{x, y}, bf16x2));
}
AGN_DEV float lo_bf16(uint32_t u) { return __uint_as_float(u << 16); }
AGN_DEV float hi_bf16(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// the same for either 16-bit storage type (T = bf16 / f16; fp16 converts, bf16 shifts)
// ReLU of two packed 16-bit floats as int16 max with 0 (v_pk_max_i16): a set sign bit (negative,
// -0) gives +0, everything else is kept. relu(round(x)) == round(relu(x)) bit for bit for every
// non-NaN x (a value that rounds to -0 was negative), and a NaN stays NaN as in torch.relu,
// where fmaxf(NaN, 0) would give 0. Replaces the canonicalising v_max_f32 pair per element.
typedef short s16x2 __attribute__((ext_vector_type(2)));
AGN_DEV uint32_t relu_pk16(uint32_t x) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, x), s16x2{0, 0}));
}
template <typename T> AGN_DEV uint32_t pack2t(float x, float y);
template <> AGN_DEV uint32_t pack2t<bf16>(float x, float y) { return pack2(x, y); }
template <> AGN_DEV uint32_t pack2t<f16>(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{x, y}, f16x2));
}
template <typename T> AGN_DEV float lo16(uint32_t u);
template <typename T> AGN_DEV float hi16(uint32_t u);
template <> AGN_DEV float lo16<bf16>(uint32_t u) { return lo_bf16(u); }
template <> AGN_DEV float hi16<bf16>(uint32_t u) { return hi_bf16(u); }
template <> AGN_DEV float lo16<f16>(uint32_t u) { return (float)__builtin_bit_cast(f16x2, u)[0]; }
template <> AGN_DEV float hi16<f16>(uint32_t u) { return (float)__builtin_bit_cast(f16x2, u)[1]; }

// ---------------------------------------------------------------- MLP hidden activations
// (AGN_ACT_*, mlp.py:37 getattr(F, activation_fn)). fp32 forms of torch's kernels: F.gelu with
// approximate='none', F.silu, torch.tanh; their backward formulas are torch's GeluBackward,
// SiluBackward (from the input) and TanhBackward (from the output, rounded as the forward stored it).
AGN_DEV float act_fwd(int k, float x) {
  if (k == AGN_ACT_GELU) return x * 0.5f * (1.f + erff(x * 0.70710678118654752440f));
  if (k == AGN_ACT_SILU) return x / (1.f + expf(-x));
  if (k == AGN_ACT_TANH) return tanhf(x);
  return fmaxf(x, 0.f);
}
// dy * f'(x), x the (rounded) pre-activation, dy the gradient of the (rounded) output
template <typename T>
AGN_DEV float act_bwd(int k, float x, float dy) {
  if (k == AGN_ACT_GELU) {
    const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752440f));
    const float pdf = expf(-0.5f * x * x) * 0.39894228040143267794f;  // M_2_SQRTPI * M_SQRT1_2 / 2
    return dy * (cdf + x * pdf);
  }
  if (k == AGN_ACT_SILU) {
    const float s = 1.f / (1.f + expf(-x));
    return dy * s * (1.f + x * (1.f - s));
  }
  if (k == AGN_ACT_TANH) {
    const float y = round_t<T>(tanhf(x));
    return dy * (1.f - y * y);
  }
  return x > 0.f ? dy : 0.f;
}

// o[0..3] = features 16i+4h.., o[4..7] = 16i+8+4h.. (acc registers 8i..8i+7)
AGN_DEV void load8_w(float (&o)[8], const bf16* rowp, int i, int h) {
  const u32x4 x = *reinterpret_cast<const u32x4*>(rowp + 16 * i + 8 * h);
  uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  o[0] = lo_bf16(a0); o[1] = hi_bf16(a0); o[2] = lo_bf16(a1); o[3] = hi_bf16(a1);
  o[4] = lo_bf16(b0); o[5] = hi_bf16(b0); o[6] = lo_bf16(b1); o[7] = hi_bf16(b1);
}
AGN_DEV void load8_w(float (&o)[8], const f16* rowp, int i, int h) {
  const u32x4 x = *reinterpret_cast<const u32x4*>(rowp + 16 * i + 8 * h);
  uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  o[0] = lo16<f16>(a0); o[1] = hi16<f16>(a0); o[2] = lo16<f16>(a1); o[3] = hi16<f16>(a1);
  o[4] = lo16<f16>(b0); o[5] = hi16<f16>(b0); o[6] = lo16<f16>(b1); o[7] = hi16<f16>(b1);
}
AGN_DEV void load8_w(float (&o)[8], const float* rowp, int i, int h) {
  const f32x4 x = load4(rowp + 16 * i + 4 * h), y = load4(rowp + 16 * i + 8 + 4 * h);
#pragma unroll
  for (int e = 0; e < 4; ++e) { o[e] = x[e]; o[4 + e] = y[e]; }
}
// ---------------------------------------------------------------- LDS-staged coalesced tile I/O
// A wave's 32-row tile of a row-major [rows][H] bf16 matrix (H = 8 * NC chunks of 16 B) moves
// through an 8-row LDS staging area `stg` (8 x NC uint4, private to the wave) in 4 passes, so
// every global access instruction covers 1 KB contiguous. In registers each lane keeps the
// row's chunks in "exchanged" form: chunk 2i + h of row c (what pack8_w produces).
// Staging rows are padded by STG_PAD chunks: with a 256-B stride the 16 (row, half) addresses
// one wave touches per chunk step all fall into the same 4 banks (8-way conflicts, measured
// 1.6e8 SQ_LDS_BANK_CONFLICT cycles per 3 edge forwards); 288 B spreads them over 64 banks.
constexpr int STG_PAD = 2;
// split form: tile_load_issue puts the tile's global loads in flight (32 registers of raw chunks),
// tile_load_finish routes them through the staging rows; other work can sit in between
template <int NC>
AGN_DEV void tile_load_issue(uint4 (&raw)[NC / 2], const bf16* tile_base, int nvalid, int lane, int ldc = NC) {
  static_assert(NC >= 8 && NC <= 64, "staged tile I/O needs 8..64 chunks per row");
  constexpr int PER = 64 / NC;  // rows covered by one 1-KB instruction
  static_assert(32 / PER == NC / 2, "raw chunk count");
  const uint4* gb = reinterpret_cast<const uint4*>(tile_base);
#pragma unroll
  for (int k = 0; k < 32 / PER; ++k) {
    const int q = lane + 64 * k, r = q / NC;
    raw[k] = (r < nvalid) ? gb[(size_t)r * ldc + q % NC] : uint4{0u, 0u, 0u, 0u};
  }
}
template <int NC>
AGN_DEV void tile_load_finish(uint4 (&mine)[NC / 2], const uint4 (&raw)[NC / 2], uint4 (*stg)[NC + STG_PAD], int lane) {
  constexpr int PER = 64 / NC;
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int k = 0; k < 8 / PER; ++k) {
      const int q = lane + 64 * k;  // chunk within the 8-row block
      stg[q / NC][q % NC] = raw[p * (8 / PER) + k];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < NC / 2; ++i) {
      const uint4 v = stg[c & 7][2 * i + h];
      if ((c >> 3) == p) mine[i] = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}
template <int NC>
AGN_DEV void tile_load_chunks(uint4 (&mine)[NC / 2], const bf16* tile_base, int nvalid, uint4 (*stg)[NC + STG_PAD], int lane,
                              int ldc = NC) {
  uint4 raw[NC / 2];
  tile_load_issue<NC>(raw, tile_base, nvalid, lane, ldc);
  tile_load_finish<NC>(mine, raw, stg, lane);
}
template <int NC>
AGN_DEV void tile_store_chunks(const uint4 (&mine)[NC / 2], bf16* tile_base, int nvalid, uint4 (*stg)[NC + STG_PAD], int lane,
                               int ldc = NC) {
  static_assert(NC >= 8 && NC <= 64, "staged tile I/O needs 8..64 chunks per row");
  constexpr int PER = 64 / NC;
  const int c = lane & 31, h = lane >> 5;
  uint4* gb = reinterpret_cast<uint4*>(tile_base);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if ((c >> 3) == p) {
#pragma unroll
      for (int i = 0; i < NC / 2; ++i) stg[c & 7][2 * i + h] = mine[i];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 8 / PER; ++k) {
      const int q = lane + 64 * k, r = 8 * p + q / NC;
      const uint4 v = stg[q / NC][q % NC];
      if (r < nvalid) gb[(size_t)r * ldc + q % NC] = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}
// exchanged chunk -> acc-layout floats (the lane-half exchange of load8_w)
AGN_DEV void unpack8_w(float (&o)[8], uint4 u) {
  const u32x4 x = __builtin_bit_cast(u32x4, u);
  uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  o[0] = lo_bf16(a0); o[1] = hi_bf16(a0); o[2] = lo_bf16(a1); o[3] = hi_bf16(a1);
  o[4] = lo_bf16(b0); o[5] = hi_bf16(b0); o[6] = lo_bf16(b1); o[7] = hi_bf16(b1);
}

// pack + lane-half exchange of store8_w without the store: chunk (2i + h) of the row
AGN_DEV uint4 pack8_w(const float (&v)[8], int h) {
  uint32_t a0 = pack2(v[0], v[1]), a1 = pack2(v[2], v[3]), b0 = pack2(v[4], v[5]), b1 = pack2(v[6], v[7]);
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  return __builtin_bit_cast(uint4, u32x4{a0, a1, b0, b1});
}
AGN_DEV void store8_w(bf16* rowp, int i, int h, const float (&v)[8], bool valid) {
  uint32_t a0 = pack2(v[0], v[1]), a1 = pack2(v[2], v[3]), b0 = pack2(v[4], v[5]), b1 = pack2(v[6], v[7]);
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  if (valid) *reinterpret_cast<u32x4*>(rowp + 16 * i + 8 * h) = u32x4{a0, a1, b0, b1};
}
AGN_DEV void store8_w(f16* rowp, int i, int h, const float (&v)[8], bool valid) {
  uint32_t a0 = pack2t<f16>(v[0], v[1]), a1 = pack2t<f16>(v[2], v[3]), b0 = pack2t<f16>(v[4], v[5]),
           b1 = pack2t<f16>(v[6], v[7]);
  swap_halves(a0, b0);
  swap_halves(a1, b1);
  if (valid) *reinterpret_cast<u32x4*>(rowp + 16 * i + 8 * h) = u32x4{a0, a1, b0, b1};
}
AGN_DEV void store8_w(float* rowp, int i, int h, const float (&v)[8], bool valid) {
  if (!valid) return;
  store4(rowp + 16 * i + 4 * h, f32x4{v[0], v[1], v[2], v[3]});
  store4(rowp + 16 * i + 8 + 4 * h, f32x4{v[4], v[5], v[6], v[7]});
}
template <typename T, int NR>
AGN_DEV void load_row_w(float (&v)[NR], const T* rowp, int h) {
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    float o[8];
    load8_w(o, rowp, i, h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[8 * i + e] = o[e];
  }
}
template <typename T, int NR>
AGN_DEV void add_row_w(float (&v)[NR], const T* rowp, int h) {
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    float o[8];
    load8_w(o, rowp, i, h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[8 * i + e] += o[e];
  }
}
template <typename T, int NR>
AGN_DEV void store_row_w(T* rowp, const float (&v)[NR], int h, bool valid) {
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = v[8 * i + e];
    store8_w(rowp, i, h, o, valid);
  }
}

// A tile row's output held back as store-ready 16-B chunks, so that its stores issue once the
// NEXT tile's loads have been waited for: vmcnt counts loads and stores together in issue order,
// so a wait for a load also waits for every store issued before it (the edge kernels spent 10-18 %
// of their time there). p == nullptr: nothing pending.
template <int N>
struct PendingRow {
  u32x4 d[N];
  bf16* p = nullptr;
  bool valid = false;
  // chunk i of a row in store8_w's layout (features 16 i + 8 h .. +7)
  AGN_DEV void set(int i, const float (&v)[8]) {
    uint32_t a0 = pack2(v[0], v[1]), a1 = pack2(v[2], v[3]), b0 = pack2(v[4], v[5]), b1 = pack2(v[6], v[7]);
    swap_halves(a0, b0);
    swap_halves(a1, b1);
    d[i] = u32x4{a0, a1, b0, b1};
  }
  // the chunks of a packed operand (BOp<bf16>::store's layout)
  template <class B>
  AGN_DEV void set_op(const B& b) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, b.u[i]);
      uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
      swap_halves(a0, b0);
      swap_halves(a1, b1);
      d[i] = u32x4{a0, a1, b0, b1};
    }
  }
  AGN_DEV void flush(int h) {
    if (p && valid) {
#pragma unroll
      for (int i = 0; i < N; ++i) *reinterpret_cast<u32x4*>(p + 16 * i + 8 * h) = d[i];
    }
    p = nullptr;
  }
};

// ---------------------------------------------------------------- AGN_TILED saves (aerognn.h)
// 16-B unit index of (row, unit i of the lane's NR registers, half h); U = units per lane-row.
template <typename T, int NR>
AGN_DEV size_t tiled_unit(int row, int i, int h) {
  constexpr int U = NR * (int)sizeof(T) / 16;
  return ((size_t)(row >> 5) * U + i) * 64 + (row & 31) + 32 * h;
}
template <typename T, int NR>
AGN_DEV void store_row_tiled(T* base, const float (&v)[NR], int row, int h, bool valid) {
  if (!valid) return;
  uint4* b = reinterpret_cast<uint4*>(base);
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i)
      b[tiled_unit<T, NR>(row, i, h)] = __builtin_bit_cast(
          uint4, u32x4{pack2t<T>(v[8 * i], v[8 * i + 1]), pack2t<T>(v[8 * i + 2], v[8 * i + 3]),
                       pack2t<T>(v[8 * i + 4], v[8 * i + 5]), pack2t<T>(v[8 * i + 6], v[8 * i + 7])});
  } else {
#pragma unroll
    for (int i = 0; i < NR / 4; ++i)
      b[tiled_unit<T, NR>(row, i, h)] = __builtin_bit_cast(uint4, f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]});
  }
}
template <typename T, int NR>
AGN_DEV void load_row_tiled(float (&v)[NR], const T* base, int row, int h) {
  const uint4* b = reinterpret_cast<const uint4*>(base);
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, b[tiled_unit<T, NR>(row, i, h)]);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[8 * i + 2 * j] = lo16<T>(x[j]); v[8 * i + 2 * j + 1] = hi16<T>(x[j]); }
    }
  } else {
#pragma unroll
    for (int i = 0; i < NR / 4; ++i) {
      const f32x4 x = __builtin_bit_cast(f32x4, b[tiled_unit<T, NR>(row, i, h)]);
      v[4 * i] = x[0]; v[4 * i + 1] = x[1]; v[4 * i + 2] = x[2]; v[4 * i + 3] = x[3];
    }
  }
}
AGN_DEV void unpack8(float (&v)[8], uint4 u) {
  const u32x4 x = __builtin_bit_cast(u32x4, u);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf16(x[j]); v[2 * j + 1] = hi_bf16(x[j]); }
}
// register quad q (features 8q+4h..+3) of a tiled row
template <typename T, int NR>
AGN_DEV f32x4 load4_tiled(const T* base, int q, int row, int h) {
  if constexpr (sizeof(T) == 2) {
    const T* p = base + tiled_unit<T, NR>(row, q >> 1, h) * 8 + 4 * (q & 1);
    return load4(p);
  } else {
    return load4(base + tiled_unit<T, NR>(row, q, h) * 4);
  }
}
template <typename T, int NR>
AGN_DEV void store4_tiled(T* base, int q, int row, int h, f32x4 v) {
  if constexpr (sizeof(T) == 2) store4(base + tiled_unit<T, NR>(row, q >> 1, h) * 8 + 4 * (q & 1), v);
  else store4(base + tiled_unit<T, NR>(row, q, h) * 4, v);
}
// unit i of a pair loop (8 registers 8i..8i+7): bf16 = one unit, fp32 = units 2i, 2i+1
template <typename T, int NR>
AGN_DEV void store8_tiled(T* base, int i, int row, int h, const float (&v)[8], bool valid) {
  if (!valid) return;
  uint4* b = reinterpret_cast<uint4*>(base);
  if constexpr (sizeof(T) == 2) {
    b[tiled_unit<T, NR>(row, i, h)] =
        __builtin_bit_cast(uint4, u32x4{pack2t<T>(v[0], v[1]), pack2t<T>(v[2], v[3]), pack2t<T>(v[4], v[5]),
                                        pack2t<T>(v[6], v[7])});
  } else {
    b[tiled_unit<T, NR>(row, 2 * i, h)] = __builtin_bit_cast(uint4, f32x4{v[0], v[1], v[2], v[3]});
    b[tiled_unit<T, NR>(row, 2 * i + 1, h)] = __builtin_bit_cast(uint4, f32x4{v[4], v[5], v[6], v[7]});
  }
}
template <typename T, int NR>
AGN_DEV void load8_tiled(float (&v)[8], const T* base, int i, int row, int h) {
  const uint4* b = reinterpret_cast<const uint4*>(base);
  if constexpr (sizeof(T) == 2) {
    const u32x4 x = __builtin_bit_cast(u32x4, b[tiled_unit<T, NR>(row, i, h)]);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[2 * j] = lo16<T>(x[j]); v[2 * j + 1] = hi16<T>(x[j]); }
  } else {
    const f32x4 x = __builtin_bit_cast(f32x4, b[tiled_unit<T, NR>(row, 2 * i, h)]);
    const f32x4 y = __builtin_bit_cast(f32x4, b[tiled_unit<T, NR>(row, 2 * i + 1, h)]);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = x[j]; v[4 + j] = y[j]; }
  }
}

// Compiler-only barrier: keeps hipcc from hoisting later global loads (LN params, residual
// rows) above the MFMA chain, where they would sit live in registers across every layer.
AGN_DEV void cbarrier() { asm volatile("" ::: "memory"); }

// a value behind a compiler barrier: per-lane offsets derived from it are recomputed where used
// instead of being hoisted out of a tile loop (where they would sit in registers and spill)
AGN_DEV int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// feature index held in register rho by lane half h (acc layout)
AGN_DEV int feat_of(int rho, int h) { return 8 * (rho >> 2) + 4 * h + (rho & 3); }

// Per-feature fp32 parameter vector (bias, LN gamma/beta) in acc layout: 4-wide loads of the
// 4 consecutive features each register quad holds. Features >= n (or p == NULL) read as 0.
template <int NR, bool FULL = false>
AGN_DEV void load_param(float (&v)[NR], const float* p, int n, int h) {
#pragma unroll
  for (int q = 0; q < NR / 4; ++q) {
    const int f0 = 8 * q + 4 * h;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (FULL) {
      x = *reinterpret_cast<const f32x4*>(p + f0);
    } else if (p) {
      if (f0 + 3 < n) x = *reinterpret_cast<const f32x4*>(p + f0);
      else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + e < n) x[e] = p[f0 + e];
      }
    }
    v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
  }
}

// ---------------------------------------------------------------- MFMA traits
// Packed A fragments: unit u = ((ot * KU) + ku) * 64 + lane, 16 bytes per lane.
//   bf16: one unit = one v_mfma_f32_32x32x16_bf16 k-step (16 K), KU = ceil(K/16)
//   f32 : one unit = four v_mfma_f32_32x32x2_f32 k-steps (4 regs of B), KU = 2*ceil(K/16)
// The number of activation registers for K features is NRK(K) = 8 * ceil(K/16).
AGN_DEV constexpr int nrk(int k) { return 8 * ((k + 15) / 16); }

// Activation operand of the next GEMM (B operand), built from acc-layout registers:
// bf16 packs the 8 registers of one MFMA k-step (16 K) into a bf16x8; f32 keeps floats
// (one register per v_mfma_f32_32x32x2_f32 k-step).
template <typename T, int NR> struct BOp;
template <int NR> struct BOp<bf16, NR> {
  static constexpr int RPU = 8;   // registers per packed A unit
  bf16x8 u[NR / 8];
  AGN_DEV void set(const float (&v)[NR]) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i)
      u[i] = __builtin_bit_cast(bf16x8, u32x4{pack2(v[8 * i], v[8 * i + 1]), pack2(v[8 * i + 2], v[8 * i + 3]),
                                              pack2(v[8 * i + 4], v[8 * i + 5]), pack2(v[8 * i + 6], v[8 * i + 7])});
  }
  AGN_DEV void mfma(f32x16& acc, const uint4& a_raw, int unit) const {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(&a_raw);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, u[unit], acc, 0, 0, 0);
  }
  // relu(acc) straight into the packed operand (register rho = 16*t + r of acc tile t)
  template <int NT>
  AGN_DEV void set_relu(const f32x16 (&acc)[NT]) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      u32x4 w;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = relu_pk16(pack2(acc[(8 * i + 2 * k) / 16][(8 * i + 2 * k) % 16],
                               acc[(8 * i + 2 * k + 1) / 16][(8 * i + 2 * k + 1) % 16]));
      u[i] = __builtin_bit_cast(bf16x8, w);
    }
  }
  // From a row's 16-B chunks as loaded (chunk i of lane half h = features 16i+8h..+7) or as the
  // staging rows hand them over ("exchanged": tile_load_finish): the lane-half swap of load8_w /
  // unpack8_w puts the acc-order pairs in place, so the operand is the swapped dwords themselves,
  // not an unpack to fp32 and a repack (identical bits: bf16 -> fp32 -> bf16 is exact; only a
  // signalling NaN would come back quieted by the repack, which this path skips).
  AGN_DEV void set_w(const uint4 (&mine)[NR / 8]) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, mine[i]);
      uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
      swap_halves(a0, b0);
      swap_halves(a1, b1);
      u[i] = __builtin_bit_cast(bf16x8, u32x4{a0, a1, b0, b1});
    }
  }
  AGN_DEV void load_w(const bf16* rowp, int h) {
    uint4 raw[NR / 8];
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) raw[i] = *reinterpret_cast<const uint4*>(rowp + 16 * i + 8 * h);
    set_w(raw);
  }
  // registers 8i..8i+7 (acc order) as floats
  AGN_DEV void get8(float (&o)[8], int i) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)u[i][j];
  }
  // AGN_TILED store: the packed registers as they are (no lane exchange)
  AGN_DEV void store_tiled(bf16* base, int row, int h, bool valid) const {
    if (!valid) return;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i)
      reinterpret_cast<uint4*>(base)[tiled_unit<bf16, NR>(row, i, h)] = __builtin_bit_cast(uint4, u[i]);
  }
  // store the packed activations as a row of `H` bf16, 16 B per lane (see store8_w)
  AGN_DEV void store(bf16* rowp, int h, bool valid) const {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, u[i]);
      uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
      swap_halves(a0, b0);
      swap_halves(a1, b1);
      if (valid) *reinterpret_cast<u32x4*>(rowp + 16 * i + 8 * h) = u32x4{a0, a1, b0, b1};
    }
  }
};
template <int NR> struct BOp<f16, NR> {
  static constexpr int RPU = 8;
  f16x8 u[NR / 8];
  AGN_DEV void set(const float (&v)[NR]) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) u[i][j] = (f16)v[8 * i + j];
  }
  AGN_DEV void mfma(f32x16& acc, const uint4& a_raw, int unit) const {
    f16x8 a = *reinterpret_cast<const f16x8*>(&a_raw);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, u[unit], acc, 0, 0, 0);
  }
  template <int NT>
  AGN_DEV void set_relu(const f32x16 (&acc)[NT]) {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      u32x4 w;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = relu_pk16(pack2t<f16>(acc[(8 * i + 2 * k) / 16][(8 * i + 2 * k) % 16],
                                     acc[(8 * i + 2 * k + 1) / 16][(8 * i + 2 * k + 1) % 16]));
      u[i] = __builtin_bit_cast(f16x8, w);
    }
  }
  AGN_DEV void get8(float (&o)[8], int i) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)u[i][j];
  }
  AGN_DEV void store_tiled(f16* base, int row, int h, bool valid) const {
    if (!valid) return;
#pragma unroll
    for (int i = 0; i < NR / 8; ++i)
      reinterpret_cast<uint4*>(base)[tiled_unit<f16, NR>(row, i, h)] = __builtin_bit_cast(uint4, u[i]);
  }
  AGN_DEV void store(f16* rowp, int h, bool valid) const {
#pragma unroll
    for (int i = 0; i < NR / 8; ++i) {
      const u32x4 x = __builtin_bit_cast(u32x4, u[i]);
      uint32_t a0 = x[0], a1 = x[1], b0 = x[2], b1 = x[3];
      swap_halves(a0, b0);
      swap_halves(a1, b1);
      if (valid) *reinterpret_cast<u32x4*>(rowp + 16 * i + 8 * h) = u32x4{a0, a1, b0, b1};
    }
  }
};
template <int NR> struct BOp<float, NR> {
  static constexpr int RPU = 4;
  float u[NR];
  AGN_DEV void set(const float (&v)[NR]) {
#pragma unroll
    for (int i = 0; i < NR; ++i) u[i] = v[i];
  }
  AGN_DEV void mfma(f32x16& acc, const uint4& a_raw, int unit) const {
    f32x4 a = *reinterpret_cast<const f32x4*>(&a_raw);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], u[4 * unit + e], acc, 0, 0, 0);
  }
  template <int NT>
  AGN_DEV void set_relu(const f32x16 (&acc)[NT]) {
#pragma unroll
    for (int i = 0; i < NR; ++i) u[i] = fmaxf(acc[i / 16][i % 16], 0.f);
  }
  AGN_DEV void get8(float (&o)[8], int i) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = u[8 * i + j];
  }
  AGN_DEV void store_tiled(float* base, int row, int h, bool valid) const {
    store_row_tiled<float, NR>(base, u, row, h, valid);
  }
  AGN_DEV void store(float* rowp, int h, bool valid) const {
    if (!valid) return;
#pragma unroll
    for (int q = 0; q < NR / 4; ++q)
      *reinterpret_cast<f32x4*>(rowp + 8 * q + 4 * h) = f32x4{u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]};
  }
};

// Packed A fragments: unit u = ((ot * KU) + ku) * 64 + lane, 16 bytes per lane.
//   bf16: one unit = one v_mfma_f32_32x32x16_bf16 k-step (16 K), KU = ceil(K/16)
//   f32 : one unit = four v_mfma_f32_32x32x2_f32 k-steps, KU = 2*ceil(K/16)
// The number of activation registers for K features is nrk(K) = 8 * ceil(K/16).
template <typename T> AGN_DEV constexpr int units_k(int k) { return nrk(k) / BOp<T, 16>::RPU; }

// ---------------------------------------------------------------- AGN_RELU_MASK (aerognn.h)
// The backward only needs sign(relu output) of a hidden layer: one bit per activation register.
// Dword d of lane `lane` in 32-row tile t sits at (t * ND + d) * 64 + lane (one 256-B coalesced
// access per dword); bit j = register 32d + j of the packed operand is > 0 (the stored value,
// i.e. after rounding to T, exactly the test the backward applied to the re-read activation).
template <int NR> AGN_DEV constexpr int mask_dwords() { return (NR + 31) / 32; }
// bit i = (register i > 0). bf16: integer tests on the packed pairs (a bf16 in the top 16 bits of
// a dword is > 0 as a signed int iff it is a positive nonzero value), no float conversions.
template <int NR> AGN_DEV bool bop_pos(const BOp<bf16, NR>& b, int i) {
  const uint32_t w = __builtin_bit_cast(u32x4, b.u[i / 8])[(i % 8) / 2];
  return (int32_t)((i & 1) ? (w & 0xffff0000u) : (w << 16)) > 0;
}
template <int NR> AGN_DEV bool bop_pos(const BOp<f16, NR>& b, int i) { return (float)b.u[i / 8][i % 8] > 0.f; }
template <int NR> AGN_DEV bool bop_pos(const BOp<float, NR>& b, int i) { return b.u[i] > 0.f; }
template <typename T, int NR>
AGN_DEV void store_relu_mask(void* base, const BOp<T, NR>& b, int tile, int lane) {
  constexpr int ND = mask_dwords<NR>();
  uint32_t* p = reinterpret_cast<uint32_t*>(base) + (size_t)tile * ND * 64 + lane;
  if constexpr (sizeof(T) == 2) {
    // relu outputs are >= 0 or -0: per bf16 half, (magnitude + 0x7fff) carries into the sign
    // position iff the magnitude is nonzero; & ~sign drops -0. Bits are placed with v_bfe +
    // v_lshl_or (inline shift constants: no per-bit literal masks held in VGPRs).
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      uint32_t w = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = 32 * d + 2 * k;  // registers i, i+1 share one packed dword
        if (i < NR) {
          const uint32_t x = __builtin_bit_cast(u32x4, b.u[i / 8])[(i % 8) / 2];
          const uint32_t q = ((x & 0x7fff7fffu) + 0x7fff7fffu) & ~x;
          w |= __builtin_amdgcn_ubfe(q, 15, 1) << (2 * k);
          w |= __builtin_amdgcn_ubfe(q, 31, 1) << (2 * k + 1);
        }
      }
      p[d * 64] = w;
    }
  } else {
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (32 * d + j < NR) w |= (bop_pos<NR>(b, 32 * d + j) ? 1u : 0u) << j;
      p[d * 64] = w;
    }
  }
}
template <int NR>
AGN_DEV void load_relu_mask(uint32_t (&m)[mask_dwords<NR>()], const void* base, int tile, int lane) {
  constexpr int ND = mask_dwords<NR>();
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base) + (size_t)tile * ND * 64 + lane;
#pragma unroll
  for (int d = 0; d < ND; ++d) m[d] = p[d * 64];
}
// v * bit i of the mask (the relu backward select): v_bfe_i32 gives 0 / all-ones, then an AND of
// the float's bits (no per-bit literal constants, no compares)
AGN_DEV float mask_sel(const uint32_t* m, int i, float v) {
  const int32_t s = __builtin_amdgcn_sbfe((int32_t)m[i >> 5], i & 31, 1);
  return __uint_as_float(__float_as_uint(v) & (uint32_t)s);
}

// acc[ot] += A[ot tile, units 0..nu-1] * B, A fragments staged in LDS as [ot][ku_total][64]
// (16 B per lane, linear: one conflict-free ds_read_b128 per lane per unit). The next unit's
// fragments are read while the current unit's MFMAs issue.
template <typename T, int NT, int NR, bool FULL = false>
AGN_DEV void gemm(f32x16 (&acc)[NT], const BOp<T, NR>& b, int nu, const uint4* lds, int ku_total,
                  int otn, int lane) {
  constexpr int NUMAX = NR / BOp<T, NR>::RPU;
  uint4 ac[NT], an[NT];
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) ac[ot] = lds[(ot * ku_total) * 64 + lane];
#pragma unroll
  for (int u = 0; u < NUMAX; ++u) {
    if (u < nu) {
      if (u + 1 < nu) {
#pragma unroll
        for (int ot = 0; ot < NT; ++ot) an[ot] = lds[(ot * ku_total + u + 1) * 64 + lane];
      }
#pragma unroll
      for (int ot = 0; ot < NT; ++ot)
        if (FULL || ot < otn) b.mfma(acc[ot], ac[ot], u);
#pragma unroll
      for (int ot = 0; ot < NT; ++ot) ac[ot] = an[ot];
    }
  }
}

// ---------------------------------------------------------------- exact row sums on the MFMA
// x + y of two bf16 rows, into acc-layout fp32 registers, by the matrix cores: an identity A
// fragment times the row operand (acc order, BOp::set_w) is the row itself, exactly (one nonzero
// product per output); four MFMAs per 32-feature tile give acc = x exactly, then round(x + y) -
// the fp32 add of the VALU path, bit for bit (a -0 sum comes out +0, equal as a value; a NaN or
// inf in one feature reaches the 15 other features of its k-step through 0 * inf).
// A operand lane map (cdna_hip_programming.md: lane l holds A[row l&31][k = 8(l>>5) + j]); the
// operand's k order is the acc-register order (feature 16u + 8(j>>2) + 4(l>>5) + (j&3) at k-step
// u), so the identity's one for output row i < 16 of k-step 2 ot sits at j = 4(i>>3) + (i&3) of the
// lanes with (i>>2)&1 == l>>5; rows 16..31 take the same pattern in k-step 2 ot + 1.
AGN_DEV void ident_frags(bf16x8& f0, bf16x8& f1, int lane) {
  const int i = lane & 31, il = i & 15;
  const int j = 4 * (il >> 3) + (il & 3);
  const uint32_t one = (((il >> 2) & 1) == (lane >> 5)) ? (0x3F80u << (16 * (j & 1))) : 0u;
  const int d = j >> 1;
  const u32x4 w = {d == 0 ? one : 0u, d == 1 ? one : 0u, d == 2 ? one : 0u, d == 3 ? one : 0u};
  const u32x4 z = {0u, 0u, 0u, 0u};
  f0 = __builtin_bit_cast(bf16x8, i < 16 ? w : z);
  f1 = __builtin_bit_cast(bf16x8, i < 16 ? z : w);
}
// The same identity for operands in ROW order, as 16-B loads of a row-major bf16 row deliver them
// (lane half h holds features 16 u + 8 h .. + 7 of k-step u: no lane-half exchange, set_w): the one
// for output row i < 16 of k-step 2 ot sits at j = i & 7 of the lanes with (i >> 3) & 1 == l >> 5.
// The products and sums are the acc-order identity's, so acc_add2_mfma_rows(x raw, y raw) is
// acc_add2_mfma(set_w(x), set_w(y)) bit for bit, without the 96 moves / swaps of the exchange.
AGN_DEV void ident_frags_rows(bf16x8& f0, bf16x8& f1, int lane) {
  const int i = lane & 31, il = i & 15;
  const int j = il & 7;
  const uint32_t one = (((il >> 3) & 1) == (lane >> 5)) ? (0x3F80u << (16 * (j & 1))) : 0u;
  const int d = j >> 1;
  const u32x4 w = {d == 0 ? one : 0u, d == 1 ? one : 0u, d == 2 ? one : 0u, d == 3 ? one : 0u};
  const u32x4 z = {0u, 0u, 0u, 0u};
  f0 = __builtin_bit_cast(bf16x8, i < 16 ? w : z);
  f1 = __builtin_bit_cast(bf16x8, i < 16 ? z : w);
}
template <int NT, int NU>
AGN_DEV void acc_add2_mfma_rows(f32x16 (&acc)[NT], const uint4 (&x)[NU], const uint4 (&y)[NU], const bf16x8& f0,
                                const bf16x8& f1) {
  static_assert(NU == 2 * NT, "two raw 16-B chunks per output tile");
  auto u = [](const uint4& v) { return __builtin_bit_cast(bf16x8, v); };
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, u(x[2 * ot]), f32x16{}, 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, u(x[2 * ot + 1]), acc[ot], 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, u(y[2 * ot]), acc[ot], 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, u(y[2 * ot + 1]), acc[ot], 0, 0, 0);
}
template <int NT, int NR>
AGN_DEV void acc_add2_mfma(f32x16 (&acc)[NT], const BOp<bf16, NR>& x, const BOp<bf16, NR>& y, const bf16x8& f0,
                           const bf16x8& f1) {
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, x.u[2 * ot], f32x16{}, 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, x.u[2 * ot + 1], acc[ot], 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f0, y.u[2 * ot], acc[ot], 0, 0, 0);
#pragma unroll
  for (int ot = 0; ot < NT; ++ot) acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f1, y.u[2 * ot + 1], acc[ot], 0, 0, 0);
}

// ---------------------------------------------------------------- LayerNorm element steps
// Written with explicit fused operations: under -ffp-contract=fast the compiler's SLP
// vectorisation otherwise contracts some elements of a row (fma) and not others (packed mul +
// add), per kernel, so two kernels evaluating the same LayerNorm would round differently. Every
// kernel that computes or differentiates the chain's LayerNorm uses these.
AGN_DEV float ln_sq_acc(float q, float d) { return __builtin_fmaf(d, d, q); }  // q + d^2
// backward pass 1: c1 += g*gamma, c2 += (g*gamma) * xhat
AGN_DEV void ln_bwd_acc(float& c1, float& c2, float g, float gm, float xh) {
  const float gg = g * gm;
  c1 = c1 + gg;
  c2 = __builtin_fmaf(gg, xh, c2);
}
// backward pass 2: (g*gamma - c1 - xhat*c2) * rstd
AGN_DEV float ln_bwd_out(float g, float gm, float c1, float c2, float xh, float rstd) {
  const float t = __builtin_fmaf(g, gm, -c1);
  return __builtin_fmaf(-xh, c2, t) * rstd;
}
// The same steps on two consecutive registers with the elementwise work in packed fp32
// (v_pk_mul / v_pk_add / v_pk_fma: one instruction per pair, the scalar rounding per element;
// a lone wave issues them at the scalar rate, so they halve its VALU time). The running sums c1,
// c2 still take the elements in register order. Contraction off: no fma the scalar forms lack.
AGN_DEV f32x2 ln_xhat2(f32x2 hv, float mean, float rstd) {
#pragma clang fp contract(off)
  return (hv - f32x2{mean, mean}) * f32x2{rstd, rstd};
}
AGN_DEV void ln_bwd_acc2(float& c1, float& c2, f32x2 g, f32x2 gm, f32x2 xh) {
#pragma clang fp contract(off)
  const f32x2 gg = g * gm;
  c1 = c1 + gg[0];
  c2 = __builtin_fmaf(gg[0], xh[0], c2);
  c1 = c1 + gg[1];
  c2 = __builtin_fmaf(gg[1], xh[1], c2);
}
AGN_DEV f32x2 ln_bwd_out2(f32x2 g, f32x2 gm, float c1, float c2, f32x2 xh, float rstd) {
#pragma clang fp contract(off)
  const f32x2 t = __builtin_elementwise_fma(g, gm, f32x2{-c1, -c1});
  return __builtin_elementwise_fma(-xh, f32x2{c2, c2}, t) * f32x2{rstd, rstd};
}
AGN_DEV f32x2 f2(float x, float y) { return f32x2{x, y}; }
// variance pass of the statistics on a register pair: q += d0^2, q += d1^2 (ln_sq_acc in register
// order), the two subtractions of the mean in one v_pk_add
AGN_DEV float ln_sq_acc2(float q, float v0, float v1, float mean) {
#pragma clang fp contract(off)
  const f32x2 d = f32x2{v0, v1} - f32x2{mean, mean};
  q = __builtin_fmaf(d[0], d[0], q);
  return __builtin_fmaf(d[1], d[1], q);
}
// LayerNorm output gamma * xhat + beta as an explicit fma of the rounded xhat (every kernel)
AGN_DEV float ln_out(float v, float mean, float rstd, float g, float b) {
#pragma clang fp contract(off)
  return __builtin_fmaf((v - mean) * rstd, g, b);
}
AGN_DEV f32x2 ln_out2(f32x2 v, float mean, float rstd, f32x2 g, f32x2 b) {
#pragma clang fp contract(off)
  return __builtin_elementwise_fma((v - f32x2{mean, mean}) * f32x2{rstd, rstd}, g, b);
}

// ---------------------------------------------------------------- wave reductions
// The value a butterfly partner at distance M holds, with VALU cross-lane operations (no LDS
// round trip, unlike __shfl_xor's ds_bpermute). M = 1, 2: DPP quad_perm (lane ^ M); M = 4: DPP
// row_half_mirror (lane ^ 7 within 8 lanes: it differs from this lane in bit 2, which is all a
// reduce step over bit 2 needs; the summation tree changes, not the set summed); M = 8: DPP
// row_ror:8 (lane ^ 8 within a 16-lane row); M = 16 / 32: v_permlane16_swap / v_permlane32_swap.
template <int M> AGN_DEV float partner(float v) {
  const int x = __float_as_int(v);
  if constexpr (M == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  else if constexpr (M == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  else if constexpr (M == 4) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
  else if constexpr (M == 8) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false));
  else if constexpr (M == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)x, false, false);
    return __uint_as_float((__lane_id() & 16) ? r[0] : r[1]);
  } else {
    static_assert(M == 32, "butterfly distance");
    const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)x, (uint32_t)x, false, false);
    return __uint_as_float((__lane_id() & 32) ? r[0] : r[1]);
  }
}
AGN_DEV float xor32(float v) { return partner<32>(v); }
// v + (the value lane l ^ 32 holds): one v_permlane32_swap of v with itself leaves the lower half's
// value in r[0] and the upper half's in r[1] on every lane, so the sum needs no lane select
// (and a + b == b + a: bitwise v + xor32(v) on both halves)
AGN_DEV float sum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Transpose-reduce NR per-lane values over the 32 lanes of each half (lanes c = l & 31).
// On return lane c holds in v[i] (i < max(NR/32,1)) the 32-lane sum of register
// rho = floor(c*NR/32) + i; for NR < 32 the 32/NR lanes sharing a rho hold identical sums.
template <int NR, int N, int M>
struct Butterfly {
  // one exchange step: keep half of the N live registers, add the partner's other half
  static AGN_DEV void run(float (&v)[NR], int c) {
    if constexpr (M >= 1) {
      if constexpr (N >= 2) {
        constexpr int HALF = N / 2;
        if constexpr (M == 16) {
          // v_permlane16_swap(x = v[i], y = v[HALF + i]) leaves (x_lo, x_up) on the lower row's
          // lanes and (y_lo, y_up) on the upper row's: each row's keep + partner sum, no selects
#pragma unroll
          for (int i = 0; i < HALF; ++i) {
            const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[HALF + i]),
                                                            false, false);
            v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
          }
        } else {
          const bool upper = (c & M) != 0;
#pragma unroll
          for (int i = 0; i < HALF; ++i) {
            const float keep = upper ? v[HALF + i] : v[i];
            const float send = upper ? v[i] : v[HALF + i];
            v[i] = keep + partner<M>(send);
          }
        }
        Butterfly<NR, HALF, M / 2>::run(v, c);
      } else {
        v[0] += partner<M>(v[0]);
        Butterfly<NR, 1, M / 2>::run(v, c);
      }
    }
  }
};

template <int NR>
AGN_DEV void butterfly_reduce(float (&v)[NR], int lane) {
  Butterfly<NR, NR, 16>::run(v, lane & 31);
}

}  // namespace agn
