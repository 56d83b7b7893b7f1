// Fused training backward of the sum-trick edge MLP (gfx950, bf16, H = 128): forward recompute,
// chain rule and in-kernel weight gradients in ONE persistent launch.
//
// Reference chain (models/mgnLayer.py:72-105, residual :205):
//   h0 = e W_e^T + P_s[src] + P_d[dst];  a1 = relu(h0); h1 = a1 W1^T + b1; a2 = relu(h1);
//   h2 = a2 W2^T + b2; a3 = relu(h2); h3 = a3 W3^T + b3; e' = e + LN(h3).
// Backward of one 32-edge tile (S = dL/de' = g + dAgg[dst]):
//   G3 = LN'(S);  dW3 += G3^T a3, db3 += sum G3;  G2 = (G3 W3) . [a3 > 0];  ... ;
//   G0 = (G1 W1) . [a1 > 0];  de = G0 W_e + S.
//   G0 is written (its sender / receiver segment sums are dP_s / dP_d, dW_e = G0^T e goes to
//   agn_wgrad); G1..G3, a2, a3 and h3 never reach HBM.
//
// Work split (one 512-thread workgroup per CU, two waves per SIMD):
//  * waves 0-3 ("chain waves", one per SIMD) each own a 32-edge tile per round. They start from
//    the forward's saved a1 and LayerNorm statistics (agn_edge_forward32's training saves; without
//    them h0 is recomputed from e, P_s[src], P_d[dst] and W_e), recompute h1..h3 bitwise the
//    forward kernel's values (same operands, same MFMA order), keep a2 and a3 in registers, run the
//    LayerNorm backward and the chain rule, and hand each layer's (G_L, a_L) to the dW waves in
//    16-row items through an LDS ring;
//  * waves 4-7 ("dW waves", one per SIMD) own a 64x64 quarter of dW1..dW3 each (192 accumulator
//    registers for the whole launch) and consume every item in a fixed order (round, wave group,
//    layer, wave, half): the fp32 sums are deterministic;
//  * Lin1..Lin3 live in LDS as ONE image each, read both ways: rows (ds_read_b128, the forward's
//    A = W fragments) and columns (ds_read_b64_tr_b16, the backward's A = W^T fragments). The image
//    is layout (a) of cdna_hip_programming.md T10 over the packed forward operand (agn_pack,
//    trans = 0), whose k order is the acc-register order of common.hpp; the transposed reads pick
//    their 8-byte pieces so that each lane gets the same 8 values, in the same order, as the split
//    path's packed W^T fragments (agn_pack, trans = 1). W_e's packed fragments are read from L2.
// The ring holds NSLOT (7) slots of 8 KB (G_L and a_L for 16 rows, layout (a) images read with
// ds_read_b64_tr_b16 by the dW MFMAs, k = rows). A chain wave writes item n into slot n % NSLOT
// once item n - NSLOT has been consumed by all four dW waves; LDS counters (filled / consumed)
// order the hand-offs, no workgroup barrier runs inside the main loops.
// Per-workgroup partials (dW, db, LayerNorm) go to slabs that agn_wgrad_reduce / agn_colsum sum in
// fixed order: no atomics on HBM.
#include "common.hpp"
#include "aerognn.h"

using namespace agn;

namespace {

constexpr int H = 128;
constexpr int NT = 4;                  // 32-feature tiles per row
constexpr int NR = 64;                 // acc registers per row half
constexpr int CW = 4;                  // chain waves
constexpr int NWAVE = 8;               // chain + dW waves
constexpr int NTHR = 64 * NWAVE;
#ifndef AGN_EB_NSLOT
#define AGN_EB_NSLOT 7
#endif
constexpr int NSLOT = AGN_EB_NSLOT;    // ring slots (8 KB each; a tile's hand-off pair takes two)
#ifndef AGN_EB_GROUP
#define AGN_EB_GROUP 2  // chain waves per hand-off group (item order, chain_wave)
#endif
constexpr int GROUP = AGN_EB_GROUP;
constexpr int IMG_B = H * H * 2;       // one 128 x 128 bf16 image (32 KB)
constexpr int HALF_B = 16 * H * 2;     // 16 rows of one item matrix (4 KB)
constexpr int SLOT_B = 2 * HALF_B;     // G half + a half
// LDS images of Lin1..Lin3 at (l - 1) * IMG_B; W_e is read from L2 (packed fragments, 32 KB shared by
// every CU): its 32 KB of LDS went to the ring, 3 -> 7 slots (round 6)
constexpr int OFF_RING = 3 * IMG_B;
constexpr int OFF_PV = OFF_RING + NSLOT * SLOT_B;  // fp32 [4][H]: b1, b2, b3, LN gamma
constexpr int OFF_FLAG = OFF_PV + 4 * H * 4;       // int filled[NSLOT], consumed[NSLOT]
constexpr int OFF_LNP = OFF_FLAG + 8 * ((2 * NSLOT + 7) / 8) * 4;  // fp32 [CW][2][H]: LayerNorm partials per chain wave
constexpr int OFF_IDS = OFF_LNP + CW * 2 * H * 4;   // int [CW][64]: next tile's src (lanes 0-31) / dst
constexpr int LDS_B = OFF_IDS + CW * 64 * 4;
static_assert(LDS_B <= 160 * 1024, "LDS budget");

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Layout (a) of a [rows][128] bf16 image: 8-row x 32-column subtiles of 512 B, 16-B chunk ch of
// row r at the byte offset below. Row reads of a 32x32x16 operand (one 16-B chunk per lane, 32
// rows) and transposed reads (4 rows x 32 columns per 32-lane half) are both conflict-free, and
// the offsets split into a per-lane part plus immediates (4096 per 16 rows, 512 per 32 columns).
AGN_DEV int aoff(int r, int ch) {
  return 2048 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}

// feature held at image position p (the acc-register order of common.hpp swaps bits 2 and 3
// within each 16-feature block); an involution
AGN_DEV int phi(int p) { return (p & ~12) | ((p & 4) << 1) | ((p & 8) >> 1); }

AGN_DEV bf16x8 tr_pair(const char* lo, const char* hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lo));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(hi));
  const bf16x4 x = __builtin_bit_cast(bf16x4, a), y = __builtin_bit_cast(bf16x4, b);
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

AGN_DEV void mfma(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}

// acc[ot] += W[ot rows] . X^T for the 8 k-steps of an H-wide operand (A = W row fragments of an
// LDS image): the order of common.hpp gemm(), so the sums are bitwise the forward kernel's
AGN_DEV void gemm_rows(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const char* img, int lane) {
  const int i = lane & 31, hh = lane >> 5;
  const int base = 2048 * (i >> 3) + 64 * (i & 7);
  const int x = (i >> 2) & 3;
  const char* pe = img + base + 16 * (hh ^ x);        // k-steps u even: chunk 2u + hh, (ch & 3) = hh
  const char* po = img + base + 16 * ((2 + hh) ^ x);  // u odd: (ch & 3) = 2 + hh
  // fragments stream two (u, ot) steps ahead (8 registers in flight)
  auto frag = [&](int idx) {
    const int u = idx >> 2, ot = idx & 3;
    return *reinterpret_cast<const uint4*>((u & 1 ? po : pe) + 512 * (u >> 1) + 8192 * ot);
  };
  uint4 f0 = frag(0), f1 = frag(1);
#pragma unroll
  for (int idx = 0; idx < 8 * NT; ++idx) {
    const uint4 cur = f0;
    f0 = f1;
    if (idx + 2 < 8 * NT) f1 = frag(idx + 2);
    b.mfma(acc[idx & 3], cur, idx >> 2);
    __builtin_amdgcn_sched_barrier(0);  // keep the 2-deep prefetch: no hoisting of all 32 reads
  }
}

// acc[ot] = W^T[ot rows] . G^T (accumulators start at zero): A = W^T fragments by transposed reads of the same image. Lane
// (i, hh) of k-step u needs W[16u + 8(j>>2) + 4hh + (j&3)][32ot + i], j = 0..7 (agn_pack trans = 1):
// rows 16u + 4hh + q (q = 0..3) and 16u + 8 + 4hh + q; lane 4q + p of its 16-lane group g supplies
// the 8-byte piece (chunk 4ot + 2(g&1) + (p&1), half p>>1), so the column lane t of the group
// receives is position 32ot + 16(g&1) + phi(t), i.e. feature 32ot + i.
AGN_DEV void gemm_cols(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const char* img, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, hh = lane >> 5;
  const int xx = 2 * (g & 1) + (p & 1);
  const char* r1 = img + 64 * (4 * hh + q) + 16 * (xx ^ hh) + 8 * (p >> 1);
  const char* r2 = img + 2048 + 64 * (4 * hh + q) + 16 * (xx ^ (hh + 2)) + 8 * (p >> 1);
  auto frag = [&](int idx) {
    const int u = idx >> 2, ot = idx & 3;
    return tr_pair(r1 + 4096 * u + 512 * ot, r2 + 4096 * u + 512 * ot);
  };
  bf16x8 f0 = frag(0), f1 = frag(1);
#pragma unroll
  for (int idx = 0; idx < 8 * NT; ++idx) {
    const bf16x8 cur = f0;
    f0 = f1;
    if (idx + 2 < 8 * NT) f1 = frag(idx + 2);
    if (idx < NT) acc[idx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, b.u[0], f32x16{}, 0, 0, 0);
    else mfma(acc[idx & 3], cur, b.u[idx >> 2]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// gemm_rows and gemm_cols with the A fragments from global memory (L2): W_e's packed operands,
// forward (agn_pack trans = 0) and transposed (trans = 1), unit ((ot * 8) + u) * 64 + lane. These are
// the values the LDS image reads give (the image is built from the trans = 0 operand; the transposed
// reads reproduce the trans = 1 operand, see gemm_cols), in the same MFMA order: bitwise the same sums.
// Fragments stream PFG deep (L2 latency under the MFMAs).
constexpr int PFG = 8;
AGN_DEV void gemm_rows_g(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* w, int lane) {
  uint4 f[PFG];
#pragma unroll
  for (int i = 0; i < PFG; ++i) f[i] = w[((i & 3) * 8 + (i >> 2)) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < 8 * NT; ++idx) {
    const uint4 cur = f[idx % PFG];
    const int nx = idx + PFG;
    if (nx < 8 * NT) f[idx % PFG] = w[((nx & 3) * 8 + (nx >> 2)) * 64 + lane];
    b.mfma(acc[idx & 3], cur, idx >> 2);
    __builtin_amdgcn_sched_barrier(0);
  }
}
AGN_DEV void gemm_cols_g(f32x16 (&acc)[NT], const BOp<bf16, NR>& b, const uint4* wt, int lane) {
  uint4 f[PFG];
#pragma unroll
  for (int i = 0; i < PFG; ++i) f[i] = wt[((i & 3) * 8 + (i >> 2)) * 64 + lane];
#pragma unroll
  for (int idx = 0; idx < 8 * NT; ++idx) {
    const bf16x8 cur = __builtin_bit_cast(bf16x8, f[idx % PFG]);
    const int nx = idx + PFG;
    if (nx < 8 * NT) f[idx % PFG] = wt[((nx & 3) * 8 + (nx >> 2)) * 64 + lane];
    if (idx < NT) acc[idx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, b.u[0], f32x16{}, 0, 0, 0);
    else mfma(acc[idx & 3], cur, b.u[idx >> 2]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// acc = bias (fp32 [H] in LDS), acc layout
AGN_DEV void acc_bias(f32x16 (&acc)[NT], const float* pv, int h) {
#pragma unroll
  for (int q = 0; q < 4 * NT; ++q) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(pv + 8 * q + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
  }
}

// Spin on an LDS counter. Bounded (about half a second) so that a protocol error can never leave
// a wave spinning forever; a wait that gives up is recorded in the device fault word (one lane,
// a vector atomic OR), which agn_fault_status reports: the launch's dW / db are then wrong and
// the caller must not use them.
__device__ int g_agn_fault = 0;
AGN_DEV void wait_ge(int* p, int v) {
  bool ok = false;
  for (int spin = 0; spin < (1 << 24); ++spin) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) {
      ok = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (!ok && __lane_id() == 0) __hip_atomic_fetch_or(&g_agn_fault, AGN_FAULT_RING_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("" ::: "memory");
}
// scheduling fence: keeps the machine scheduler from hoisting the next phase's LDS reads (bias,
// gamma) above the current phase's register work, where they would all be live at once
AGN_DEV void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
AGN_DEV void lgkm_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// the lane id behind a compiler barrier: per-lane LDS offsets derived from it are recomputed in
// each phase instead of being hoisted out of the tile loop (where they would sit in registers
// across the whole chain and spill)
template <typename V> AGN_DEV void opaque(V& v) { asm volatile("" : "+v"(v)); }
// pin a packed operand in place: IR passes must not sink its computation (and every input it
// reads) down to the first use, which would keep those inputs live across the work in between
AGN_DEV void pin(BOp<bf16, NR>& b) {
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) opaque(b.u[i]);
}
AGN_DEV int fresh_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

struct Rounds {  // XCD-grouped round walk (blocks b and b + 8 share an XCD and its L2)
  int first, end, step;
  AGN_DEV Rounds(int nrounds) {
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
      const int grp = blockIdx.x & 7, per = (nrounds + 7) / 8;
      first = grp * per + (blockIdx.x >> 3);
      end = min(nrounds, (grp + 1) * per);
      step = gridDim.x >> 3;
    } else {
      first = blockIdx.x;
      end = nrounds;
      step = gridDim.x;
    }
  }
};

// ------------------------------------------------------------------------------ chain wave
// Item n = (round, wave group, L, chain wave, half) (chain_wave's nbase): G_L and a_L of
// rows 16 half .. 16 half + 15 of the wave's tile, as two layout (a) images: unit i of lane
// (c, hh) = positions 16i + 8hh..+7 (chunk 2i + hh) of row c & 15. A chain wave hands both halves
// over at once (items n0, n0 + 1): every lane writes, each half into its own slot.
// an item pair's filled flags, once this wave's writes of it have retired (LDS in order per wave)
AGN_DEV void produce_flag(char* lds, int n0, int lane) {
#ifdef AGN_EB_NORING
  return;
#endif
  int* filled = reinterpret_cast<int*>(lds + OFF_FLAG);
  lgkm_drain();
  if (lane == 0) {
    __hip_atomic_store(&filled[n0 % NSLOT], n0 / NSLOT + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&filled[(n0 + 1) % NSLOT], (n0 + 1) / NSLOT + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
AGN_DEV void produce_pair(char* lds, int n0, const BOp<bf16, NR>& G, const BOp<bf16, NR>& X, int lane,
                          unsigned long long* ist = nullptr) {
#ifdef AGN_EB_NORING
  return;  // diagnostic build only: the chain alone (no hand-offs; dW / db are not computed)
#endif
  int* filled = reinterpret_cast<int*>(lds + OFF_FLAG);
  int* consumed = filled + NSLOT;
  const int k0 = n0 % NSLOT, j0 = n0 / NSLOT;
  const int k1 = (n0 + 1) % NSLOT, j1 = (n0 + 1) / NSLOT;
#ifdef AGN_EB_STAMPS
  if (ist && lane == 0) ist[0] = __builtin_amdgcn_s_memtime();
#endif
  wait_ge(&consumed[k0], 4 * j0);
  wait_ge(&consumed[k1], 4 * j1);
#ifdef AGN_EB_STAMPS
  if (ist && lane == 0) ist[1] = __builtin_amdgcn_s_memtime();
#endif
  const int c = lane & 31, hh = lane >> 5;
  char* sb = lds + OFF_RING + ((c >> 4) ? k1 : k0) * SLOT_B;
  const int r = c & 15, x = (r >> 2) & 3;
  const int base = 2048 * (r >> 3) + 64 * (r & 7);
  const int oe = base + 16 * (hh ^ x), oo = base + 16 * ((2 + hh) ^ x);  // aoff(r, 2i + hh), i even / odd
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int o = (i & 1 ? oo : oe) + 512 * (i >> 1);
    *reinterpret_cast<uint4*>(sb + o) = __builtin_bit_cast(uint4, G.u[i]);
    *reinterpret_cast<uint4*>(sb + HALF_B + o) = __builtin_bit_cast(uint4, X.u[i]);
  }
  // the flags are set by produce_flag after the chain step that follows (its LDS waits retire these
  // writes, so that drain costs nothing; round 6: -0.8 % per launch)
#ifdef AGN_EB_STAMPS
  if (ist && lane == 0) ist[2] = __builtin_amdgcn_s_memtime();
#endif
}

// G_{L-1} = dA . [a_L > 0] (the split path's AGN_RELU_MASK select), packed: each pair of dA is
// rounded to bf16 by one v_cvt_pk and ANDed with a 16-bit mask per half built from the packed
// activation (relu outputs are +0 or positive int16 patterns: 0 - a is negative exactly when a > 0,
// and its arithmetic shift by 15 is 0xffff or 0). Bitwise the select-then-round of the split path:
// a dropped element is 0x0000 either way, a kept one is the same rounding of dA.
// The mask is built on the whole 8-lane short vector: the per-dword form
// bit_cast<short2>(bit_cast<uint4>(act)[k]) is miscompiled by this hipcc (ROCm 7.2, -O3: dword 0's
// mask is applied to all four dwords of the unit; caught by test_fused_edge_bwd_matches_split and
// the bf16 oracle tests, reproduced in a 20-line kernel).
typedef short s16x8v __attribute__((ext_vector_type(8)));
AGN_DEV void relu_select_pk(BOp<bf16, NR>& out, const f32x16 (&acc)[NT], const BOp<bf16, NR>& act) {
#pragma unroll
  for (int i = 0; i < NR / 8; ++i) {
    // relu outputs are +0 or positive int16 patterns: min(a, 1) as unsigned 16-bit is 1 exactly when
    // a > 0, and the rounded dA times that 0 / 1 is the masked value bit for bit (3 VALU per dword
    // instead of v_pk_sub + v_pk_ashr + v_and + v_cvt_pk). Inline asm: written with 16-bit vector
    // builtins, this hipcc applied dword 0's mask to all four dwords of the unit (the miscompile above)
    const u32x4 a4 = __builtin_bit_cast(u32x4, act.u[i]);
    u32x4 w;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = 8 * i + 2 * k;
      const uint32_t g = pack2(acc[r / 16][r % 16], acc[(r + 1) / 16][(r + 1) % 16]);
      uint32_t m;
      asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(m) : "v"(a4[k]));  // (the constant 1 for both halves)
      asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(w[k]) : "v"(g), "v"(m));
    }
    out.u[i] = __builtin_bit_cast(bf16x8, w);
  }
}

// Diagnostic phase clocks (built with -DAGN_EB_STAMPS into a separate library; the product build
// has none): chain wave w of blocks 0 and 128 stamps s_memtime at 16 points of its first 8 tiles
// into a.stamps[((sel * 8 + w) * 8 + tile) * 16 + point]; dW wave d stores its total wait and
// total cycles at point 0 / 1 of slot (sel * 8 + 4 + d) * 8 * 16.
#ifdef AGN_EB_STAMPS
#ifndef AGN_EB_STAMP_MASK
#define AGN_EB_STAMP_MASK 0xfff  // which of the 12 points are stamped (1: the tile starts only)
#endif
#define EB_STAMP(k)                                                                                     \
  do {                                                                                                  \
    if (((AGN_EB_STAMP_MASK >> (k)) & 1) && stp && ntile_done < 8 && (lane0 & 63) == 0)                \
      stp[ntile_done * 16 + (k)] = __builtin_amdgcn_s_memtime();                                        \
  } while (0)
// item-level clocks of produce(): tiles 1 and 2 of block 0's chain waves, at 2048 + 576 + ..
#define EB_IST(pi) \
  ((AGN_EB_STAMP_MASK == 0xfff && stp && blockIdx.x == 0 && (ntile_done == 1 || ntile_done == 2)) \
       ? a.stamps + 2048 + 576 + ((cw * 2 + ntile_done - 1) * 6 + (pi)) * 3 : nullptr)
#else
#define EB_STAMP(k) \
  do {              \
  } while (0)
#define EB_IST(pi) nullptr
#endif

// SAVED: the tile starts from the forward's a1 (AGN_TILED) and LayerNorm statistics
// (agn_edge_forward32's training saves) instead of recomputing h0 from e, P_s[src], P_d[dst] and
// W_e; every value downstream is bitwise the same. a3 stays in registers from the forward recompute
// to its hand-off. SAVED keeps a2 as well and drops a1 after Lin1, re-reading it from the forward's
// save for the L1 hand-off; otherwise a2 is recomputed from a1 for its hand-off (32 MFMAs plus its
// bias / ReLU work per tile), or with SCR parked in the wave's 8-KB slice of a.scratch and read
// back (opt-in: the same time, and the slices do not stay in L2).
// ENC: the same chain as an encoder MLP (models/mlp.py:40-51 on the node / edge features,
// models/bsms_mgn.py:138-139): h0 = x W0^T + b0 on k <= 16 input features (a.e, rows gathered by
// a.src when set), S = g (no receiver term), and no input gradient: the tile ends with G0's store
// (dW0 = G0^T x and db0 go to agn_wgrad). Bitwise the split path's (mlp_bwd_res_kernel) G's.
template <bool SAVED, bool SCR, bool ENC = false>
AGN_DEV void chain_wave(const agn_edge_bwd_args& a, char* lds, int cw, int lane0) {
#ifdef AGN_EB_STAMPS
  unsigned long long* stp = nullptr;
  if (a.stamps && (blockIdx.x == 0 || blockIdx.x == 128)) stp = a.stamps + ((blockIdx.x == 0 ? 0 : 8) + cw) * 8 * 16;
  int ntile_done = 0;
#endif
  const int ntiles = (a.rows + 31) / 32;
  const int nrounds = (ntiles + CW - 1) / CW;
  const Rounds rw(nrounds);
  const float* pv = reinterpret_cast<const float*>(lds + OFF_PV);
  const bf16* P = reinterpret_cast<const bf16*>(a.proj);
  int rcount = 0;
  // The node ids of a wave's next tile are loaded one tile ahead (the tile's P_s / P_d gathers
  // then wait for one memory latency instead of two dependent ones) and handed to the next tile
  // through the wave's LDS slot, not a loop-carried register: a loop-carried load result makes
  // the compiler's wait at the loop head vmcnt(0), i.e. for this tile's de / G0 stores as well.
  // Lane l loads the src (l < 32) or dst (l >= 32) of row l & 31.
  int* ids = reinterpret_cast<int*>(lds + OFF_IDS) + cw * 64;
  const int32_t* const srcp = a.src;  // (scalar copies: a per-lane choice of the struct field made
  const int32_t* const dstp = a.dst;  // the compiler load the pointer itself, behind a full wait)
  auto tile_id = [&](int rd) {
    const int row = (rd * CW + cw) * 32 + (lane0 & 31);
    const int rr = row < a.rows ? row : a.rows - 1;
    if constexpr (ENC) return srcp ? srcp[rr] : rr;  // the input row (gathered or not)
    const int32_t* p = (lane0 < 32 && !SAVED) ? srcp : dstp;  // (SAVED reads no src)
    return p[rr];
  };
  // this wave's scratch slice (a2): unit i of lane l at 16 (64 i + l) (1 KB per wave instruction)
  uint4* const scr = SCR ? reinterpret_cast<uint4*>(a.scratch) + (size_t)(blockIdx.x * CW + cw) * 512 : nullptr;
  if (rw.first < rw.end) ids[lane0] = tile_id(rw.first);
  for (int rd = rw.first; rd < rw.end; rd += rw.step, ++rcount) {
    const int cmax = min(CW, ntiles - rd * CW);
    if (cw >= cmax) continue;
    EB_STAMP(0);
    // Item order within a round: wave group g (waves 2g, 2g+1), then layer, then wave, then half.
    // The ring hands over one group's whole backward before the other's, so the two groups run
    // half a tile apart and the hand-offs of one group overlap the other's forward recompute.
    const int gsz = GROUP == 2 ? (cw < 2 ? min(2, cmax) : cmax - 2) : 1;  // waves in this group
    const int nbase = GROUP == 2 ? rcount * 6 * CW + (cw < 2 ? 0 : 6 * min(2, cmax)) + 2 * (cw & 1)
                                 : rcount * 6 * CW + 6 * cw;
    // (only a workgroup's last round can be partial)
    const int tile = rd * CW + cw;
    cbarrier();
    // per-tile lane id: nothing lane-derived (row addresses, LDS offsets) is hoisted out of the
    // tile loop, where it would stay live across the whole chain
    const int lane = fresh_lane(lane0);
    const int c = lane & 31, h = lane >> 5;
    const int row = tile * 32 + c;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const int sid = SAVED ? 0 : ids[c], did = ENC ? 0 : ids[32 + c];
    const bool more = rd + rw.step < rw.end;
    const int nid = tile_id(more ? rd + rw.step : rd);  // stored to the slot before the tile's stores
    // incoming gradient rows g and dAgg[dst]: loaded now, kept raw (64 registers) through the
    // forward recompute
    // SAVED: a1 and the statistics first (the recompute starts on a1)
    BOp<bf16, NR> a1;  // the only activation kept in registers from the forward pass
    f32x2 st{0.f, 0.f};
    if constexpr (SAVED) {
      const uint4* ap = reinterpret_cast<const uint4*>(a.a1);
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) a1.u[i] = __builtin_bit_cast(bf16x8, ap[tiled_unit<bf16, NR>(rr, i, h)]);
      st = *reinterpret_cast<const f32x2*>(a.stats + 2 * (size_t)rr);
    }
    uint4 graw[NR / 8], g2raw[NR / 8];
    if constexpr (ENC) {
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) g2raw[i] = uint4{0u, 0u, 0u, 0u};
    } else {
      const bf16* g2p = reinterpret_cast<const bf16*>(a.g2) + (size_t)did * H;
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) g2raw[i] = *reinterpret_cast<const uint4*>(g2p + 16 * i + 8 * h);
    }
    if (a.g) {
      const bf16* gp = reinterpret_cast<const bf16*>(a.g) + (size_t)rr * H;
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) graw[i] = *reinterpret_cast<const uint4*>(gp + 16 * i + 8 * h);
    } else {
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) graw[i] = uint4{0u, 0u, 0u, 0u};
    }
    // ---- forward recompute (mlp_fwd_res_kernel's operations, in its order)
    f32x16 acc[NT];
    if constexpr (ENC) {
      // h0 = x W0^T + b0 (enc32_fwd_kernel's layer 0: the row's k <= 16 features in registers
      // 4q..4q+3 = features 8q + 4h .. +3 of one k-step, one MFMA per output tile onto the bias)
      bf16x8 xu;
      {
        const bf16* rowp = reinterpret_cast<const bf16*>(a.e) + (size_t)sid * a.xld;
        float v[8];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 x = load4_masked(rowp, 8 * q + 4 * h, a.xk, false);
          v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
        }
        xu = __builtin_bit_cast(bf16x8, u32x4{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])});
      }
      EB_STAMP(1);
      const float* b0 = a.bias[0];
#pragma unroll
      for (int q = 0; q < 4 * NT; ++q) {
        const f32x4 x = b0 ? *reinterpret_cast<const f32x4*>(b0 + 8 * q + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q / 4][4 * (q % 4) + e] = x[e];
      }
      const uint4* w0 = reinterpret_cast<const uint4*>(a.wpk[0]);
#pragma unroll
      for (int ot = 0; ot < NT; ++ot)
        acc[ot] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w0[ot * 64 + lane]), xu, acc[ot], 0, 0, 0);
      cbarrier();
      a1.template set_relu<NT>(acc);
    } else if constexpr (!SAVED) {
      {
        {  // acc = P_s[src] + P_d[dst] on the matrix cores (the forward kernel's exact add)
          uint4 xs[NR / 8], xd[NR / 8];  // rows as loaded (row-order identity: no lane-half exchange)
          const bf16* ps = P + (size_t)sid * (2 * H) + 8 * h;
          const bf16* pd = P + (size_t)did * (2 * H) + H + 8 * h;
#pragma unroll
          for (int i = 0; i < NR / 8; ++i) {
            xs[i] = *reinterpret_cast<const uint4*>(ps + 16 * i);
            xd[i] = *reinterpret_cast<const uint4*>(pd + 16 * i);
          }
          bf16x8 f0, f1;
          ident_frags_rows(f0, f1, fresh_lane(lane));
          acc_add2_mfma_rows<NT, NR / 8>(acc, xs, xd, f0, f1);
        }
        BOp<bf16, NR> eop;
        eop.load_w(reinterpret_cast<const bf16*>(a.e) + (size_t)rr * H, h);
        EB_STAMP(1);
        gemm_rows_g(acc, eop, reinterpret_cast<const uint4*>(a.wpk[0]), fresh_lane(lane));
      }
      cbarrier();
      a1.template set_relu<NT>(acc);
    } else {
      EB_STAMP(1);
    }
    pin(a1);
    sched_fence();
    acc_bias(acc, pv + 0 * H, h);
    gemm_rows(acc, a1, lds + 0 * IMG_B, fresh_lane(lane));
    cbarrier();
    // SAVED: a2 stays in registers to its hand-off and a1 is dropped here (re-read from the
    // forward's save for the L1 hand-off); otherwise a2 is recomputed from a1 (or parked in the
    // scratch) and a1 stays
    constexpr bool KEEP2 = SAVED;
    BOp<bf16, NR> a2;
    {
      a2.template set_relu<NT>(acc);
      pin(a2);
      if constexpr (SCR && !KEEP2) {
        const int l = fresh_lane(lane);
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) scr[64 * i + l] = __builtin_bit_cast(uint4, a2.u[i]);
      }
      sched_fence();
      acc_bias(acc, pv + 1 * H, h);
      gemm_rows(acc, a2, lds + 1 * IMG_B, fresh_lane(lane));
    }
    cbarrier();
    // a3 stays in registers from here to its hand-off (the chain recomputes only a2: one GEMM
    // instead of two, round 6)
    BOp<bf16, NR> a3;
    a3.template set_relu<NT>(acc);
    pin(a3);
    sched_fence();
    acc_bias(acc, pv + 2 * H, h);
    gemm_rows(acc, a3, lds + 2 * IMG_B, fresh_lane(lane));
    EB_STAMP(2);
    // LayerNorm statistics (mlp_fwd_res_kernel's epilogue)
    float mean, rstd;
    if constexpr (SAVED) {
      mean = st[0];
      rstd = st[1];
    } else {
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
    }
    // the pre-LN row as the split path stores it (bf16, acc order)
    BOp<bf16, NR> hpk;
    {
      float v[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) v[i] = acc[i / 16][i % 16];
      hpk.set(v);
      pin(hpk);
    }
    cbarrier();
    // ---- incoming gradient S = g + dAgg[dst] (mlp_bwd_res_kernel's load_grad_w)
    float A[NR];
    if constexpr (ENC) {  // S = g (mlp_bwd_res_kernel's load_grad_w without a second term)
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float x[8];
        unpack8_w(x, graw[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) A[8 * i + e] = x[e];
      }
    } else {  // S = g + g2 on the matrix cores (exact fp32 add): acc is free once h3 is packed
      bf16x8 f0, f1;
      ident_frags_rows(f0, f1, fresh_lane(lane));
      acc_add2_mfma_rows<NT, NR / 8>(acc, graw, g2raw, f0, f1);
#pragma unroll
      for (int i = 0; i < NR; ++i) A[i] = acc[i / 16][i % 16];
    }
    if (!valid) {
#pragma unroll
      for (int i = 0; i < NR; ++i) A[i] = 0.f;
    }
    // ---- LayerNorm backward (mlp_bwd_res_kernel, its expressions; partials in 16-register
    // chunks: the butterfly's XOR order 16, 8, 4, 2, 1 gives each feature the same sums)
    {
      const float* gmv = pv + 3 * H;
      // this wave's LayerNorm parameter partials: lane c adds sum g * xhat (c < 16) or sum g
      // (c >= 16) of register 16 kk + (c & 15)
      float* lnp = reinterpret_cast<float*>(lds + OFF_LNP) + cw * 2 * H + (c >> 4) * H;
      float c1 = 0.f, c2 = 0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        sched_fence();
        float B[32];  // [0, 16): g * xhat of registers 16 kk.., [16, 32): g of the same registers
#pragma unroll
        for (int i = 2 * kk; i < 2 * kk + 2; ++i) {
          float hv[8];
          unpack8(hv, __builtin_bit_cast(uint4, hpk.u[i]));
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const f32x4 gm = *reinterpret_cast<const f32x4*>(gmv + 16 * i + 8 * j + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const int r = 8 * i + 4 * j + e;
              const f32x2 xh = ln_xhat2(f2(hv[4 * j + e], hv[4 * j + e + 1]), mean, rstd);
              const f32x2 g = f2(A[r], A[r + 1]);
              ln_bwd_acc2(c1, c2, g, f2(gm[e], gm[e + 1]), xh);
              const f32x2 bx = g * xh;
              B[r - 16 * kk] = bx[0];
              B[r + 1 - 16 * kk] = bx[1];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) B[16 + i] = A[16 * kk + i];
        // lane c holds the 32-row sum of B[c]: sum g * xhat (c < 16) or sum g (c >= 16) of register
        // 16 kk + (c & 15); each feature's rows are added in the butterfly's XOR order 16, 8, 4, 2, 1
        butterfly_reduce<32>(B, lane);
        // running sum over the wave's tiles in its LDS slot (one lane per address, no-return LDS
        // add: nothing waits on it; the sum is ((0 + t0) + t1) + .. in tile order)
        __hip_atomic_fetch_add(lnp + feat_of(16 * kk + (c & 15), h), B[0], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        opaque(c1);  // the running sums are due now: nothing of this chunk stays live for later
        opaque(c2);
      }
      c1 = sum32(c1);
      c2 = sum32(c2);
      c1 /= (float)H;
      c2 /= (float)H;
      // pass 2 unpacks h3 and recomputes xhat again: opaque copies keep the compiler from holding
      // pass 1's 64 unpacked / normalised values live in between
      opaque(mean);
      opaque(rstd);
      int goff = 0;
      opaque(goff);  // gamma and A * gamma re-read / recomputed, not kept from pass 1
      const float* gmv2 = gmv + goff;
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        sched_fence();
        float hv[8];
        u32x4 hr = __builtin_bit_cast(u32x4, hpk.u[i]);
        opaque(hr);  // unpacked again, not kept from pass 1
        unpack8(hv, __builtin_bit_cast(uint4, hr));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 gm = *reinterpret_cast<const f32x4*>(gmv2 + 16 * i + 8 * j + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const int r = 8 * i + 4 * j + e;
            const f32x2 xh = ln_xhat2(f2(hv[4 * j + e], hv[4 * j + e + 1]), mean, rstd);
            const f32x2 o = ln_bwd_out2(f2(A[r], A[r + 1]), f2(gm[e], gm[e + 1]), c1, c2, xh, rstd);
            A[r] = o[0];
            A[r + 1] = o[1];
          }
        }
      }
    }
    EB_STAMP(3);
    // ---- chain rule; every layer's (G_L, a_L) goes to the dW waves
    BOp<bf16, NR> op;
    cbarrier();
    op.set(A);  // G3
    pin(op);
    if constexpr (!SCR && !KEEP2) {  // a2 = relu(a1 W1^T + b1) again (the forward's operations)
      sched_fence();
      acc_bias(acc, pv + 0 * H, h);
      gemm_rows(acc, a1, lds + 0 * IMG_B, fresh_lane(lane));
      cbarrier();
      a2.template set_relu<NT>(acc);
      pin(a2);
    }
    pin(a3);
    sched_fence();
    EB_STAMP(4);
    produce_pair(lds, nbase + 0 * gsz, op, a3, fresh_lane(lane), EB_IST(0));
    if constexpr (SCR && !KEEP2) {  // a2 back from the scratch, under the chain step
      const int l = fresh_lane(lane);
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) a2.u[i] = __builtin_bit_cast(bf16x8, scr[64 * i + l]);
    }
    EB_STAMP(5);
    gemm_cols(acc, op, lds + 2 * IMG_B, fresh_lane(lane));
    cbarrier();
    relu_select_pk(op, acc, a3);  // G2
    produce_flag(lds, nbase + 0 * gsz, fresh_lane(lane));
    if constexpr (KEEP2) {  // a1 again, into a3's registers, two chain steps ahead of its use
      int rr3 = rr;
      opaque(rr3);  // (a new load, not the first one's value kept live)
      const uint4* ap = reinterpret_cast<const uint4*>(a.a1);
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) a1.u[i] = __builtin_bit_cast(bf16x8, ap[tiled_unit<bf16, NR>(rr3, i, h)]);
    }
    EB_STAMP(6);
    pin(op);
    produce_pair(lds, nbase + 2 * gsz, op, a2, fresh_lane(lane), EB_IST(2));
    EB_STAMP(7);
    gemm_cols(acc, op, lds + 1 * IMG_B, fresh_lane(lane));
    cbarrier();
    relu_select_pk(op, acc, a2);  // G1
    produce_flag(lds, nbase + 2 * gsz, fresh_lane(lane));
    EB_STAMP(8);
    pin(op);
    // de = G0 W_e + (g + g2) (mlp_bwd_res_kernel's add_grad_w order) needs the incoming rows
    // again: re-read now (L2) so the loads complete under the L1 hand-off and chain step.
    // Opaque indices keep the compiler from holding the first reads' values live since the LN.
    auto reload_g = [&]() {
      int did2 = did, rr2 = rr;
      opaque(did2);
      opaque(rr2);
      const bf16* g2p = reinterpret_cast<const bf16*>(a.g2) + (size_t)did2 * H;
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) g2raw[i] = *reinterpret_cast<const uint4*>(g2p + 16 * i + 8 * h);
      if (a.g) {
        const bf16* gp = reinterpret_cast<const bf16*>(a.g) + (size_t)rr2 * H;
#pragma unroll
        for (int i = 0; i < NR / 8; ++i) graw[i] = *reinterpret_cast<const uint4*>(gp + 16 * i + 8 * h);
      }
    };
    if constexpr (!ENC) reload_g();
    produce_pair(lds, nbase + 4 * gsz, op, a1, fresh_lane(lane), EB_IST(4));
    EB_STAMP(9);
    gemm_cols(acc, op, lds + 0 * IMG_B, fresh_lane(lane));
    cbarrier();
    relu_select_pk(op, acc, a1);  // G0
    produce_flag(lds, nbase + 4 * gsz, fresh_lane(lane));
    EB_STAMP(10);
    pin(op);
    if (more) ids[lane] = nid;  // (this tile's reads of the slot are done: LDS is in order per wave)
    if constexpr (ENC) {  // no input gradient: G0 for agn_wgrad's dW0 / db0 ends the tile
      op.store(reinterpret_cast<bf16*>(a.g0) + (size_t)row * H, h, valid);
      EB_STAMP(11);
#ifdef AGN_EB_STAMPS
      ++ntile_done;
#endif
      continue;
    }
    // de = G0 W_e first, G0's stores after it: vmcnt retires loads and stores in issue order, so W_e's
    // fragment loads issued behind the G0 stores would each wait for those stores too
    gemm_cols_g(acc, op, reinterpret_cast<const uint4*>(a.wtpk0), fresh_lane(lane));
    sched_fence();
    op.store(reinterpret_cast<bf16*>(a.g0) + (size_t)row * H, h, valid);
    {
      float v[NR];
#pragma unroll
      for (int i = 0; i < NR / 8; ++i) {
        float x[8], y[8];
        unpack8_w(x, graw[i]);
        unpack8_w(y, g2raw[i]);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 t = f2(acc[(8 * i + e) / 16][(8 * i + e) % 16], acc[(8 * i + e + 1) / 16][(8 * i + e + 1) % 16]);
          const f32x2 o = a.g ? t + (f2(x[e], x[e + 1]) + f2(y[e], y[e + 1])) : t + f2(y[e], y[e + 1]);
          v[8 * i + e] = o[0];
          v[8 * i + e + 1] = o[1];
        }
      }
      store_row_w<bf16, NR>(reinterpret_cast<bf16*>(a.de) + (size_t)row * H, v, h, valid);
    }
    EB_STAMP(11);
#ifdef AGN_EB_STAMPS
    ++ntile_done;
#endif
  }
}

// ------------------------------------------------------------------------------ dW wave
AGN_DEV void dw_wave(const agn_edge_bwd_args& a, char* lds, int d, int lane) {
#ifdef AGN_EB_NORING
  return;  // diagnostic build only (see produce_pair)
#endif
  int* filled = reinterpret_cast<int*>(lds + OFF_FLAG);
  int* consumed = filled + NSLOT;
  const int ntiles = (a.rows + 31) / 32;
  const int nrounds = (ntiles + CW - 1) / CW;
  const Rounds rw(nrounds);
  const int ob = 2 * (d >> 1), ib = 2 * (d & 1);  // position blocks: o 32ob.., i 32ib.. (two each)
  // transposed reads of an item image: rows 8hh + q (+4), positions 32 blk + 16(g&1) + 4p..
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, hh = lane >> 5;
  const int xx = 2 * (g & 1) + (p >> 1);
  const int t1 = 2048 * hh + 64 * q + 16 * (xx ^ (2 * hh)) + 8 * (p & 1);
  const int t2 = 2048 * hh + 64 * (4 + q) + 16 * (xx ^ (2 * hh + 1)) + 8 * (p & 1);
  f32x16 dw[3][2][2];
  float dbs[3][2];
#pragma unroll
  for (int l = 0; l < 3; ++l)
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      dbs[l][x] = 0.f;
#pragma unroll
      for (int y = 0; y < 2; ++y) dw[l][x][y] = f32x16{};
    }
  int n = 0, pre0 = 0, pre1 = 0;
  // (no s_setprio: until round 6 the dW waves ran at priority 2 so that their MFMAs issued between
  // the chain's; with the faster chain, equal priority is 2.7 % faster per launch)
#ifdef AGN_EB_STAMPS
  unsigned long long waited = 0;
  const unsigned long long tstart = __builtin_amdgcn_s_memtime();
#endif
  for (int rd = rw.first; rd < rw.end; rd += rw.step) {
    const int cmax = min(CW, ntiles - rd * CW);
    for (int grp = 0; grp < CW / GROUP; ++grp) {  // the chain waves' item order (chain_wave): group, layer, wave
    const int gsz = GROUP == 2 ? (grp == 0 ? min(2, cmax) : max(0, cmax - 2)) : (grp < cmax ? 1 : 0);
#pragma unroll
    for (int li = 0; li < 3; ++li) {  // 0: L = 3, 1: L = 2, 2: L = 1
      for (int cc = 0; cc < gsz; ++cc, n += 2) {
        // a chain wave's pair (items n, n + 1: both halves of its tile) is taken at once: one
        // LDS round trip for its 16 reads instead of two
        const int k0 = n % NSLOT, j0 = n / NSLOT;
        const int k1 = (n + 1) % NSLOT, j1 = (n + 1) / NSLOT;
#ifdef AGN_EB_STAMPS
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
        if (pre0 < j0 + 1) wait_ge(&filled[k0], j0 + 1);
        if (pre1 < j1 + 1) wait_ge(&filled[k1], j1 + 1);
#ifdef AGN_EB_STAMPS
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        waited += t1 - t0;
        unsigned long long* ist = (a.stamps && blockIdx.x == 0 && n >= 24 && n < 72)
                                      ? a.stamps + 2048 + (d * 48 + n - 24) * 3 : nullptr;
        if (ist && lane == 0) {
          ist[0] = ist[3] = t0;
          ist[1] = ist[4] = t1;
        }
#endif
        bf16x8 gf[2][2], xf[2][2];
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          const char* sb = lds + OFF_RING + (q2 ? k1 : k0) * SLOT_B;
          gf[q2][0] = tr_pair(sb + 512 * ob + t1, sb + 512 * ob + t2);
          gf[q2][1] = tr_pair(sb + 512 * (ob + 1) + t1, sb + 512 * (ob + 1) + t2);
          xf[q2][0] = tr_pair(sb + HALF_B + 512 * ib + t1, sb + HALF_B + 512 * ib + t2);
          xf[q2][1] = tr_pair(sb + HALF_B + 512 * (ib + 1) + t1, sb + HALF_B + 512 * (ib + 1) + t2);
        }
        lgkm_drain();
        if (lane == 0) {
          __hip_atomic_fetch_add(&consumed[k0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(&consumed[k1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#ifdef AGN_EB_STAMPS
        if (ist && lane == 0) ist[2] = ist[5] = __builtin_amdgcn_s_memtime();
#endif
        // the next pair's flags are read now, their latency under this pair's MFMAs
        pre0 = __hip_atomic_load(&filled[(n + 2) % NSLOT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        pre1 = __hip_atomic_load(&filled[(n + 3) % NSLOT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          mfma(dw[li][0][0], gf[q2][0], xf[q2][0]);
          mfma(dw[li][0][1], gf[q2][0], xf[q2][1]);
          mfma(dw[li][1][0], gf[q2][1], xf[q2][0]);
          mfma(dw[li][1][1], gf[q2][1], xf[q2][1]);
          if ((d & 1) == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              dbs[li][0] += (float)gf[q2][0][e];
              dbs[li][1] += (float)gf[q2][1][e];
            }
          }
        }
      }
    }
    }
  }
#ifdef AGN_EB_STAMPS
  if (a.stamps && (blockIdx.x == 0 || blockIdx.x == 128) && lane == 0) {
    unsigned long long* sp = a.stamps + ((blockIdx.x == 0 ? 0 : 8) + 4 + d) * 8 * 16;
    sp[0] = waited;
    sp[1] = __builtin_amdgcn_s_memtime() - tstart;
    sp[2] = (unsigned long long)n;
  }
#endif
  // partial slabs (true feature order): dW_L of workgroup b at dw_partial[(L-1) nblk + b][o][i]
  const size_t slab = (size_t)H * H;
#pragma unroll
  for (int li = 0; li < 3; ++li) {
    float* Pw = a.dw_partial + ((size_t)(2 - li) * a.nblk + blockIdx.x) * slab;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int op = 32 * (ob + x) + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const int ip = 32 * (ib + y) + (lane & 31);
          Pw[(size_t)phi(op) * H + phi(ip)] = dw[li][x][y][r];
        }
    if ((d & 1) == 0) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const float t = dbs[li][x] + __shfl_xor(dbs[li][x], 32, 64);  // rows 8hh.. of both halves
        if (hh == 0) a.db_partial[((size_t)(2 - li) * a.nblk + blockIdx.x) * H + phi(32 * (ob + x) + lane)] = t;
      }
    }
  }
}

template <bool SAVED, bool SCR, bool ENC = false>
__global__ __launch_bounds__(NTHR, 2) void edge_bwd_fused_kernel(const agn_edge_bwd_args a) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_B];
  // weight images from the packed forward operands: unit (ot, ku, lane) -> row 32ot + lane%32,
  // chunk 2ku + lane/32
  for (int l = 1; l < 4; ++l) {
    const uint4* src = reinterpret_cast<const uint4*>(a.wpk[l]);
    for (int u = threadIdx.x; u < 2048; u += NTHR) {
      const int ln = u & 63, unit = u >> 6;
      const int o = 32 * (unit >> 3) + (ln & 31), ch = 2 * (unit & 7) + (ln >> 5);
      *reinterpret_cast<uint4*>(lds + (l - 1) * IMG_B + aoff(o, ch)) = src[u];
    }
  }
  float* pv = reinterpret_cast<float*>(lds + OFF_PV);
  for (int i = threadIdx.x; i < 4 * H; i += NTHR) {
    const int l = i / H, f = i - l * H;
    pv[i] = l < 3 ? (a.bias[l + 1] ? a.bias[l + 1][f] : 0.f) : a.ln_g[f];
  }
  if (threadIdx.x < 2 * NSLOT) reinterpret_cast<int*>(lds + OFF_FLAG)[threadIdx.x] = 0;
  for (int i = threadIdx.x; i < CW * 2 * H; i += NTHR) reinterpret_cast<float*>(lds + OFF_LNP)[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < CW) chain_wave<SAVED, SCR, ENC>(a, lds, wave, lane);
  else dw_wave(a, lds, wave - CW, lane);
  __syncthreads();
  // LayerNorm parameter partials of the four chain waves, summed in wave order
  const float* lnp = reinterpret_cast<const float*>(lds + OFF_LNP);  // [CW][2][H]
  for (int i = threadIdx.x; i < 2 * H; i += NTHR) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < CW; ++w) s += lnp[w * 2 * H + i];
    a.ln_partial[(size_t)blockIdx.x * 2 * H + i] = s;
  }
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int g_cus = 0;

}  // namespace

extern "C" {

int agn_edge_bwd_blocks(int rows) {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) g_cus = pr.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  const int rounds = ((rows + 31) / 32 + CW - 1) / CW;
  if (rounds >= g_cus) return g_cus;
  const int n = (rounds + 7) / 8 * 8;
  return n < 8 ? 8 : n;
}

size_t agn_edge_bwd_scratch_bytes(int nblk) { return nblk > 0 ? (size_t)nblk * CW * 32 * H * 2 : 0; }

int agn_fault_status_async(int* host_pinned, void* stream) {
  if (!host_pinned) return AGN_E_ARG;
  const hipError_t e = hipMemcpyFromSymbolAsync(host_pinned, HIP_SYMBOL(g_agn_fault), sizeof(int), 0,
                                                hipMemcpyDeviceToHost, (hipStream_t)stream);
  return e == hipSuccess ? 0 : (int)e;
}

int agn_debug_set_fault(int value) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_agn_fault), &value, sizeof(int)) == hipSuccess ? 0 : AGN_E_ARG;
}

int agn_fault_status(int* value, int reset) {
  if (!value) return AGN_E_ARG;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(value, HIP_SYMBOL(g_agn_fault), sizeof(int));
  if (e == hipSuccess && reset) {
    const int zero = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_agn_fault), &zero, sizeof(int));
  }
  return e == hipSuccess ? 0 : (int)e;
}

int agn_edge_bwd_fused(const agn_edge_bwd_args* a, void* stream) {
  if (!a || a->rows < 1 || a->nblk < 1 || !a->dst || !a->g2 || !a->ln_g || !a->de || !a->g0 || !a->dw_partial ||
      !a->db_partial || !a->ln_partial)
    return AGN_E_ARG;
  // either the forward's saves (a1 AGN_TILED, 16-B aligned; stats 8-B aligned) or the recompute's inputs
  if ((a->a1 != nullptr) != (a->stats != nullptr)) return AGN_E_ARG;
  if (a->a1 ? ((reinterpret_cast<uintptr_t>(a->a1) & 15) || (reinterpret_cast<uintptr_t>(a->stats) & 7))
            : (!a->e || !a->proj || !a->src))
    return AGN_E_ARG;
  if (a->scratch && (reinterpret_cast<uintptr_t>(a->scratch) & 15)) return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wpk[l]) return AGN_E_ARG;
  if (!a->wtpk0) return AGN_E_ARG;
  const bool saved = a->a1 != nullptr, scr = a->scratch != nullptr;
  const dim3 grid(a->nblk), blk(NTHR);
  if (saved) hipLaunchKernelGGL((edge_bwd_fused_kernel<true, false>), grid, blk, 0, (hipStream_t)stream, *a);  // (keeps a2: no scratch)
  else if (scr) hipLaunchKernelGGL((edge_bwd_fused_kernel<false, true>), grid, blk, 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((edge_bwd_fused_kernel<false, false>), grid, blk, 0, (hipStream_t)stream, *a);
  return launch_status();
}

int agn_encoder_bwd_fused(const agn_edge_bwd_args* a, void* stream) {
  if (!a || a->rows < 1 || a->nblk < 1 || !a->e || !a->g || !a->ln_g || !a->g0 || !a->dw_partial || !a->db_partial ||
      !a->ln_partial || a->xk < 1 || a->xk > 16 || a->xld < a->xk)
    return AGN_E_ARG;
  if ((reinterpret_cast<uintptr_t>(a->scratch) & 15) || (reinterpret_cast<uintptr_t>(a->g) & 15) ||
      (reinterpret_cast<uintptr_t>(a->g0) & 15))
    return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wpk[l] || (reinterpret_cast<uintptr_t>(a->wpk[l]) & 15)) return AGN_E_ARG;
  if (a->scratch) hipLaunchKernelGGL((edge_bwd_fused_kernel<false, true, true>), dim3(a->nblk), dim3(NTHR), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((edge_bwd_fused_kernel<false, false, true>), dim3(a->nblk), dim3(NTHR), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
