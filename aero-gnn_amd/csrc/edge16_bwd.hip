// Fused training backward of the sum-trick edge MLP on 16-row tiles (gfx950, bf16, H = 128):
// forward recompute, LayerNorm backward, chain rule and in-kernel weight gradients in ONE
// persistent launch.
//
// Backward of one 16-edge tile (S = dL/de' = g + dAgg[dst], mgnLayer.py:93-105, residual :205):
//   G3 = LN'(S);  dW3 += G3^T a3, db3 += sum G3;  G2 = (G3 W3) . [a3 > 0];  ... ;
//   G0 = (G1 W1) . [a1 > 0];  de = G0 W_e + S.
//   G0 is written (its sender / receiver segment sums are dP_s / dP_d; dW_e = G0^T e goes to
//   agn_wgrad); G1..G3, a1..a3 and h3 never reach HBM, and the training forward saves nothing.
//
// Work split (one 1024-thread workgroup per CU, 16 waves at <= 128 registers, four per SIMD):
//  * waves 0-7, the chain waves (two per SIMD, so one's loads, LayerNorm and hand-offs overlap
//    the other's MFMA phases), each own a 16-edge tile per round: they recompute h0..h3 with the
//    forward kernel's helpers (edge16.hpp, bitwise its values), run the LayerNorm backward and the
//    chain rule, and hand each layer's (G_L, a_L) to the dW waves through that layer's LDS slot;
//  * waves 8-15, the dW waves, own a 32 x 64 block of each of dW1..dW3 (96 accumulator registers
//    for the whole launch, v_mfma_f32_32x32x16_bf16 with k = the item's 16 rows) and consume every
//    item of every layer in a fixed order (round, chain wave): the fp32 sums are deterministic.
// One 8-KB slot per layer (G_L and a_L of 16 rows): item m of layer L is written once all eight
// dW waves have consumed item m - 1 of that layer. The three layers' sequences are independent, so
// a chain wave only ever waits for the previous chain wave's item of the same layer (the waves
// settle half a tile apart; no cycle: every wait is on a smaller item index).
// Per-workgroup partials (dW, db, LayerNorm) go to slabs that agn_wgrad_reduce / agn_colsum sum in
// fixed order: no atomics on HBM.
#include "edge16.hpp"
#include "aerognn.h"

using namespace agn;
using namespace agn::e16;

namespace {

constexpr int CW = 8;                        // chain waves
constexpr int DW = 8;                        // dW waves
#ifdef AGN_E16_CHAINONLY  // diagnostic: the chain waves alone at 256 registers (no dW waves launched)
constexpr int NTHR = 64 * CW;
#else
constexpr int NTHR = 64 * (CW + DW);
#endif
constexpr int ITEM_B = 2 * 16 * H * 2;       // G_L and a_L of 16 rows
constexpr int OFF_RING = 4 * IMG_B;          // [3][ITEM_B], slot L-1
constexpr int OFF_PV = OFF_RING + 3 * ITEM_B;  // fp32 [4][H]: b1, b2, b3, LN gamma
constexpr int OFF_FLAG = OFF_PV + 4 * H * 4;   // int filled[4], consumed[4] (index L-1)
constexpr int OFF_IDS = OFF_FLAG + 32;         // int [CW][32]: next tile's src (0-15) / dst (16-31)
constexpr int LDS_B = OFF_IDS + CW * 32 * 4;
static_assert(LDS_B <= 160 * 1024, "LDS budget");
static_assert(CW * 2 * H * 4 <= 3 * ITEM_B, "LayerNorm partials reuse the ring");

// Ring item image: 16 rows of 256 B; 8-byte piece hf of chunk c of row r at
// 256 r + 16 (c ^ fr(r)) + 8 (hf ^ r3), fr(r) = 4 r0 ^ 9 r1 ^ 2 r2: the chain wave's two
// ds_write_b64 per chunk and the dW waves' transposed reads are conflict-free.
AGN_DEV int fr_swz(int r) { return ((r & 1) << 2) ^ ((r & 2) ? 9 : 0) ^ ((r & 4) >> 1); }
AGN_DEV int rimg(int r, int c, int hf) { return 256 * r + 16 * (c ^ fr_swz(r)) + 8 * (hf ^ ((r >> 3) & 1)); }

AGN_DEV void lgkm_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Spin on an LDS counter, bounded (about half a second) so that a protocol error can never leave a
// wave spinning forever; a wait that gives up sets the device fault word (one lane, a vector
// atomic OR), which agn_fault_status reports: the launch's dW / db are then wrong.
__device__ int g_e16_fault = 0;  // (one per code object: read by agn_fault_status)
AGN_DEV bool wait_ge(const int* p, int v) {
  for (int spin = 0; spin < (1 << 24); ++spin) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) {
      asm volatile("" ::: "memory");
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (__lane_id() == 0) __hip_atomic_fetch_or(&g_e16_fault, AGN_FAULT_RING_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("" ::: "memory");
  return false;
}

// item m of layer L: (G, A) of the wave's tile into slot L-1 once item m-1 is consumed
AGN_DEV void produce_wait(char* lds, int L, int m) {
#ifndef AGN_E16_NORING
  const int* consumed = reinterpret_cast<const int*>(lds + OFF_FLAG) + 4;
  wait_ge(&consumed[L - 1], DW * m);
#endif
}
AGN_DEV void produce_write(char* lds, int L, int m, const Op& G, const Op& A, int lane) {
#ifdef AGN_E16_NORING
  return;  // diagnostic build only: the chain alone (no hand-offs; dW / db are not computed)
#endif
  int* filled = reinterpret_cast<int*>(lds + OFF_FLAG);
  char* sb = lds + OFF_RING + (L - 1) * ITEM_B;
  const int base = rimg(lane & 15, lane >> 4, 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int o = base ^ (64 * t);
    const u32x4 gv = __builtin_bit_cast(u32x4, G.u[t]);
    const u32x4 av = __builtin_bit_cast(u32x4, A.u[t]);
    *reinterpret_cast<uint2*>(sb + o) = uint2{gv[0], gv[1]};
    *reinterpret_cast<uint2*>(sb + (o ^ 8)) = uint2{gv[2], gv[3]};
    *reinterpret_cast<uint2*>(sb + 4096 + o) = uint2{av[0], av[1]};
    *reinterpret_cast<uint2*>(sb + 4096 + (o ^ 8)) = uint2{av[2], av[3]};
  }
  lgkm_drain();
  if (lane == 0) __hip_atomic_store(&filled[L - 1], m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Diagnostic phase clocks (a -DAGN_E16_STAMPS build into a separate library; the product build has
// none): wave w of blocks 0 and 128 stamps s_memtime at 16 points of its first 8 tiles into
// a.stamps[((sel * 16 + w) * 8 + tile) * 16 + point]; a dW wave stores its idle-loop cycles, its
// total cycles and its item count at points 0..2 of its tile-0 slot.
#ifdef AGN_E16_STAMPS
#define E16_STAMP(k)                                                                         \
  do {                                                                                       \
    if (stp && ntile < 8 && lane0 == 0) stp[ntile * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define E16_STAMP(k) \
  do {               \
  } while (0)
#endif

// LayerNorm parameter partials: 8 values (features 32s + 8g + v of chunk s) summed over the 16 rows
// of the lane's column group (DPP butterfly within the 16-lane row, common.hpp Butterfly): lane r
// ends with the sum of value r >> 1 (lanes r and r ^ 1 alike; the even / odd lane keeps the even /
// odd chunk, so a lane's two running sums per quantity cover distinct features)
AGN_DEV float rowsum8(float (&v)[8], int lane) {
  Butterfly<8, 8, 8>::run(v, lane & 15);
  return v[0];
}

// ------------------------------------------------------------------------------ chain wave
template <bool HAS_G>
AGN_DEV void chain_wave(const agn_edge_bwd_args& a, char* lds, int cw, int lane0) {
  const int ntiles = (a.rows + 15) / 16;
  const int nrounds = (ntiles + CW - 1) / CW;
  const Walk rw(nrounds, 0, 1);
  const float* pv = reinterpret_cast<const float*>(lds + OFF_PV);
  const bf16* P = reinterpret_cast<const bf16*>(a.proj);
  const bf16* E = reinterpret_cast<const bf16*>(a.e);
  const bf16* Gi = reinterpret_cast<const bf16*>(a.g);
  const bf16* G2 = reinterpret_cast<const bf16*>(a.g2);
  int* ids = reinterpret_cast<int*>(lds + OFF_IDS) + cw * 32;
  const int32_t* const srcp = a.src;
  const int32_t* const dstp = a.dst;
  auto tile_id = [&](int rd) {
    const int rr = min((rd * CW + cw) * 16 + (lane0 & 15), a.rows - 1);
    return ((lane0 & 16) ? dstp : srcp)[rr];
  };
  if (rw.first < rw.end && lane0 < 32) ids[lane0] = tile_id(rw.first);
  float run[4];  // running LayerNorm partials: sum g * xhat (0-1), sum g (2-3) of chunk 2 sp + (r & 1)
#pragma unroll
  for (int i = 0; i < 4; ++i) run[i] = 0.f;
  int rcount = 0;
#ifdef AGN_E16_STAMPS
  unsigned long long* stp = nullptr;
  if (a.stamps && (blockIdx.x == 0 || blockIdx.x == 128)) stp = a.stamps + ((blockIdx.x == 0 ? 0 : 16) + cw) * 8 * 16;
  int ntile = 0;
#endif
  for (int rd = rw.first; rd < rw.end; rd += rw.step, ++rcount) {
    const int cmax = min(CW, ntiles - rd * CW);  // (only a workgroup's last round can be partial)
    if (cw >= cmax) continue;
    const int m = rcount * CW + cw;  // item index of this tile in every layer's sequence
    cbarrier();
    E16_STAMP(0);
    const int lane = fresh(lane0);
    const int r = lane & 15, g = lane >> 4;
    const int row = (rd * CW + cw) * 16 + r;
    const bool valid = row < a.rows;
    const int rr = valid ? row : a.rows - 1;
    const bool more = rd + rw.step < rw.end;
    const int nid = tile_id(more ? rd + rw.step : rd);
    const int sid = ids[r], did = ids[16 + r];
    // ---- forward recompute (edge16_fwd_kernel's operations, in its order)
    f32x4 acc[8];
    Op a1;
    {
      uint4 xs[4], xd[4];
      Op e0;
      load_raw(xs, P + (size_t)sid * (2 * H), lane);
      load_raw(xd, P + (size_t)did * (2 * H) + H, lane);
      load_op(e0, E + (size_t)rr * H, lane);
      acc_sum2(acc, xs, xd);
      if (lane < 32 && more) ids[lane] = nid;
      E16_STAMP(1);
      gemm_fwd(acc, e0, lds, 0 * IMG_B, fresh(lane));
    }
    cbarrier();
    relu_op(a1, acc);
    pin(a1);
    bias_init(acc, pv + 0 * H, lane);
    gemm_fwd(acc, a1, lds, 1 * IMG_B, fresh(lane));
    cbarrier();
    {  // a2, a3 are not kept (recomputed after the LayerNorm backward)
      Op a2;
      relu_op(a2, acc);
      pin(a2);
      bias_init(acc, pv + 1 * H, lane);
      gemm_fwd(acc, a2, lds, 2 * IMG_B, fresh(lane));
    }
    cbarrier();
    {
      Op a3;
      relu_op(a3, acc);
      pin(a3);
      bias_init(acc, pv + 2 * H, lane);
      gemm_fwd(acc, a3, lds, 3 * IMG_B, fresh(lane));
    }
    cbarrier();
    E16_STAMP(2);
    float mean, rstd;
    ln_stats(acc, mean, rstd);
    Op hpk;  // the pre-LN row in bf16 (what the split path saves and its LN backward reads)
    pack_op(hpk, acc);
    pin(hpk);
    // ---- incoming gradient S = g + dAgg[dst] (fp32, into acc)
    {
      uint4 gr[4], g2r[4];
      load_raw(g2r, G2 + (size_t)did * H, fresh(lane));
      if (HAS_G) load_raw(gr, Gi + (size_t)rr * H, fresh(lane));
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 y = f2(raw_el(g2r, ob, e), raw_el(g2r, ob, e + 1));
          const f32x2 s = HAS_G ? f2(raw_el(gr, ob, e), raw_el(gr, ob, e + 1)) + y : y;
          acc[ob][e] = valid ? s[0] : 0.f;
          acc[ob][e + 1] = valid ? s[1] : 0.f;
        }
    }
    E16_STAMP(3);
    // ---- LayerNorm backward (mlp_bwd_res_kernel's expressions, common.hpp helpers)
    {
      const float* gmv = pv + 3 * H;
      float c1 = 0.f, c2 = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sched_fence();
        float B1[8], B2[8];
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          const int ob = 2 * s + hb;
          const f32x4 gm = *reinterpret_cast<const f32x4*>(gmv + 32 * s + 8 * g + 4 * hb);
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 xh = ln_xhat2(f2(op_el(hpk, ob, e), op_el(hpk, ob, e + 1)), mean, rstd);
            const f32x2 gv = f2(acc[ob][e], acc[ob][e + 1]);
            ln_bwd_acc2(c1, c2, gv, f2(gm[e], gm[e + 1]), xh);
            const f32x2 bx = gv * xh;
            B1[4 * hb + e] = bx[0];
            B1[4 * hb + e + 1] = bx[1];
            B2[4 * hb + e] = gv[0];
            B2[4 * hb + e + 1] = gv[1];
          }
        }
        const float v1 = rowsum8(B1, lane), v2 = rowsum8(B2, lane);
        const bool mine = (r & 1) == (s & 1);
        run[s >> 1] += mine ? v1 : 0.f;
        run[2 + (s >> 1)] += mine ? v2 : 0.f;
      }
      c1 = sum4(c1) / (float)H;
      c2 = sum4(c2) / (float)H;
      // pass 2 unpacks h3 and recomputes xhat again: opaque copies keep the compiler from holding
      // pass 1's unpacked / normalised values live (it spilled them) in between
      opaque(mean);
      opaque(rstd);
      pin(hpk);
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) {
        sched_fence();
        const f32x4 gm = *reinterpret_cast<const f32x4*>(gmv + 32 * (ob >> 1) + 8 * g + 4 * (ob & 1));
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 xh = ln_xhat2(f2(op_el(hpk, ob, e), op_el(hpk, ob, e + 1)), mean, rstd);
          const f32x2 o = ln_bwd_out2(f2(acc[ob][e], acc[ob][e + 1]), f2(gm[e], gm[e + 1]), c1, c2, xh, rstd);
          acc[ob][e] = o[0];
          acc[ob][e + 1] = o[1];
        }
      }
    }
    E16_STAMP(4);
    // ---- chain rule; every layer's (G_L, a_L) goes to the dW waves
    Op op;
    pack_op(op, acc);  // G3
    pin(op);
    cbarrier();
    Op a2;
    {
      Op a3;
      bias_init(acc, pv + 0 * H, lane);
      gemm_fwd(acc, a1, lds, 1 * IMG_B, fresh(lane));
      cbarrier();
      relu_op(a2, acc);
      pin(a2);
      bias_init(acc, pv + 1 * H, lane);
      gemm_fwd(acc, a2, lds, 2 * IMG_B, fresh(lane));
      cbarrier();
      relu_op(a3, acc);
      pin(a3);
      E16_STAMP(5);
      produce_wait(lds, 3, m);
      E16_STAMP(6);
      produce_write(lds, 3, m, op, a3, fresh(lane));
      E16_STAMP(7);
      gemm_bwd(acc, op, lds, 3 * IMG_B, fresh(lane));
      cbarrier();
      relu_select(op, acc, a3);  // G2
    }
    pin(op);
    E16_STAMP(8);
    produce_wait(lds, 2, m);
    E16_STAMP(9);
    produce_write(lds, 2, m, op, a2, fresh(lane));
    E16_STAMP(10);
    gemm_bwd(acc, op, lds, 2 * IMG_B, fresh(lane));
    cbarrier();
    relu_select(op, acc, a2);  // G1
    pin(op);
    E16_STAMP(11);
    produce_wait(lds, 1, m);
    E16_STAMP(12);
    produce_write(lds, 1, m, op, a1, fresh(lane));
    E16_STAMP(13);
    gemm_bwd(acc, op, lds, 1 * IMG_B, fresh(lane));
    cbarrier();
    relu_select(op, acc, a1);  // G0
    pin(op);
    E16_STAMP(14);
    store_op(reinterpret_cast<bf16*>(a.g0) + (size_t)row * H, op, lane, valid);
    gemm_bwd(acc, op, lds, 0 * IMG_B, fresh(lane));
    cbarrier();
    // de = G0 W_e + (g + g2) (mlp_bwd_res_kernel's add_grad_w order): the incoming rows re-read (L2)
    {
      int did2 = did, rr2 = rr;
      opaque(did2);
      opaque(rr2);
      uint4 gr[4], g2r[4];
      load_raw(g2r, G2 + (size_t)did2 * H, fresh(lane));
      if (HAS_G) load_raw(gr, Gi + (size_t)rr2 * H, fresh(lane));
      uint4 o[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint32_t wv[4];
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          const int ob = 2 * s + hb;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 t = f2(acc[ob][e], acc[ob][e + 1]);
            const f32x2 y = f2(raw_el(g2r, ob, e), raw_el(g2r, ob, e + 1));
            const f32x2 v = HAS_G ? t + (f2(raw_el(gr, ob, e), raw_el(gr, ob, e + 1)) + y) : t + y;
            wv[2 * hb + e / 2] = pack2(v[0], v[1]);
          }
        }
        o[s] = __builtin_bit_cast(uint4, u32x4{wv[0], wv[1], wv[2], wv[3]});
      }
      store_raw(reinterpret_cast<bf16*>(a.de) + (size_t)row * H, o, lane, valid);
    }
    E16_STAMP(15);
#ifdef AGN_E16_STAMPS
    ++ntile;
#endif
  }
  // the wave's LayerNorm partials -> LDS [cw][2][H] (the ring is free once every wave is done)
  __syncthreads();
  const int r = lane0 & 15, g = lane0 >> 4;
  float* lp = reinterpret_cast<float*>(lds + OFF_RING) + cw * 2 * H;
#pragma unroll
  for (int sp = 0; sp < 2; ++sp) {  // chunk 2 sp + (r & 1), value r >> 1
    const int f = 32 * (2 * sp + (r & 1)) + 8 * g + (r >> 1);
    lp[f] = run[sp];
    lp[H + f] = run[2 + sp];
  }
}

// ------------------------------------------------------------------------------ dW wave
// Transposed reads of an item image for a 32x32x16 operand (k = the item's 16 rows): lane l of
// 16-lane group G' takes rows 8(G'>>1) + q (+4) of columns 32 blk + 16(G'&1) + 4p.. (4q + p = l & 15)
AGN_DEV int dw_base(int lane, int hi) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  return rimg(8 * (G >> 1) + q + 4 * hi, 2 * (G & 1) + (p >> 1), p & 1);
}

template <int L>
AGN_DEV void consume(const char* lds, f32x16 (&dw)[2], float& dbs, int d, int lane, int* consumed) {
  const char* sb = lds + OFF_RING + (L - 1) * ITEM_B;
  const int ob = d >> 1, ib = 2 * (d & 1);
  const int b0 = dw_base(lane, 0), b1 = dw_base(lane, 1);
  const bf16x8 gf = frag2(tr64(sb + (b0 ^ (64 * ob))), tr64(sb + (b1 ^ (64 * ob))));
  const bf16x8 x0 = frag2(tr64(sb + 4096 + (b0 ^ (64 * ib))), tr64(sb + 4096 + (b1 ^ (64 * ib))));
  const bf16x8 x1 = frag2(tr64(sb + 4096 + (b0 ^ (64 * (ib + 1)))), tr64(sb + 4096 + (b1 ^ (64 * (ib + 1)))));
  lgkm_drain();
  if (lane == 0) __hip_atomic_fetch_add(&consumed[L - 1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  dw[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf, x0, dw[0], 0, 0, 0);
  dw[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf, x1, dw[1], 0, 0, 0);
  if ((d & 1) == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dbs += (float)gf[j];
  }
}

AGN_DEV void dw_wave(const agn_edge_bwd_args& a, char* lds, int d, int lane) {
#ifdef AGN_E16_NORING
  __syncthreads();
  return;  // diagnostic build only (see produce_write)
#endif
  int* filled = reinterpret_cast<int*>(lds + OFF_FLAG);
  int* consumed = filled + 4;
  const int ntiles = (a.rows + 15) / 16;
  const int nrounds = (ntiles + CW - 1) / CW;
  const Walk rw(nrounds, 0, 1);
  int total = 0;
  for (int rd = rw.first; rd < rw.end; rd += rw.step) total += min(CW, ntiles - rd * CW);
  total = __builtin_amdgcn_readfirstlane(total);
  f32x16 dw3[2], dw2[2], dw1[2];
  float db3 = 0.f, db2 = 0.f, db1 = 0.f;
#pragma unroll
  for (int x = 0; x < 2; ++x) dw3[x] = dw2[x] = dw1[x] = f32x16{};
  // the dW waves outrank their SIMD's chain waves: their two MFMAs per item issue between the
  // chain's instead of queueing behind a whole 32-MFMA chain step (which holds the slot the next
  // chain wave is waiting for)
  __builtin_amdgcn_s_setprio(2);
  int m3 = 0, m2 = 0, m1 = 0, idle = 0;
#ifdef AGN_E16_STAMPS
  unsigned long long waited = 0;
  const unsigned long long tstart = __builtin_amdgcn_s_memtime();
#endif
  while (m3 < total || m2 < total || m1 < total) {
    bool any = false;
    if (m3 < total && __hip_atomic_load(&filled[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > m3) {
      consume<3>(lds, dw3, db3, d, lane, consumed);
      ++m3;
      any = true;
    }
    if (m2 < total && __hip_atomic_load(&filled[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > m2) {
      consume<2>(lds, dw2, db2, d, lane, consumed);
      ++m2;
      any = true;
    }
    if (m1 < total && __hip_atomic_load(&filled[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > m1) {
      consume<1>(lds, dw1, db1, d, lane, consumed);
      ++m1;
      any = true;
    }
    if (any) {
      idle = 0;
    } else {
#ifdef AGN_E16_STAMPS
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_sleep(1);
      waited += __builtin_amdgcn_s_memtime() - t0;
#else
      __builtin_amdgcn_s_sleep(1);
#endif
      if (++idle >= (1 << 24)) {  // protocol error: record it and stop (the launch's dW are wrong)
        if (lane == 0) __hip_atomic_fetch_or(&g_e16_fault, AGN_FAULT_RING_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
#ifdef AGN_E16_STAMPS
  if (a.stamps && (blockIdx.x == 0 || blockIdx.x == 128) && lane == 0) {
    unsigned long long* sp = a.stamps + ((blockIdx.x == 0 ? 0 : 16) + CW + d) * 8 * 16;
    sp[0] = waited;
    sp[1] = __builtin_amdgcn_s_memtime() - tstart;
    sp[2] = (unsigned long long)total;
  }
#endif
  // partial slabs (natural feature order): dW_L of workgroup b at dw_partial[(L-1) nblk + b][o][i]
  const size_t slab = (size_t)H * H;
  const int ob = d >> 1, ib = 2 * (d & 1);
  // (32-bit lane offsets from a uniform slab base: 64-bit per-store addresses spilled)
  const int lo = (32 * ob + 4 * (lane >> 5)) * H + 32 * ib + (lane & 31);
  auto put = [&](int L, const f32x16 (&w)[2], float dbs) {
    float* Pw = a.dw_partial + ((size_t)(L - 1) * a.nblk + blockIdx.x) * slab;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int k = 0; k < 16; ++k) Pw[lo + ((k & 3) + 8 * (k >> 2)) * H + 32 * x] = w[x][k];
    if ((d & 1) == 0) {
      const float t = dbs + __shfl_xor(dbs, 32, 64);  // rows 0-7 and 8-15 of every item
      if (lane < 32) a.db_partial[((size_t)(L - 1) * a.nblk + blockIdx.x) * H + 32 * ob + lane] = t;
    }
  };
  put(3, dw3, db3);
  put(2, dw2, db2);
  put(1, dw1, db1);
  __syncthreads();  // (pairs with the chain waves' barrier before their LayerNorm partials)
}

template <bool HAS_G>
__global__ __launch_bounds__(NTHR) void edge16_bwd_kernel(const agn_edge_bwd_args a) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_B];
  load_images(lds, a.wpk, threadIdx.x, NTHR);
  float* pv = reinterpret_cast<float*>(lds + OFF_PV);
  for (int i = threadIdx.x; i < 4 * H; i += NTHR) {
    const int l = i / H, f = i - l * H;
    pv[i] = l < 3 ? (a.bias[l + 1] ? a.bias[l + 1][f] : 0.f) : a.ln_g[f];
  }
  if (threadIdx.x < 8) reinterpret_cast<int*>(lds + OFF_FLAG)[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifndef AGN_E16_ONLY
  if (wave < CW) chain_wave<HAS_G>(a, lds, wave, lane);
  else dw_wave(a, lds, wave - CW, lane);
#elif AGN_E16_ONLY == 1
  if (wave < CW) chain_wave<HAS_G>(a, lds, wave, lane);
#else
  if (wave >= CW) dw_wave(a, lds, wave - CW, lane);
#endif
  __syncthreads();
  // LayerNorm parameter partials of the eight chain waves, summed in wave order
  const float* lnp = reinterpret_cast<const float*>(lds + OFF_RING);  // [CW][2][H]
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

int agn_edge_backward_blocks(int rows) {
  if (g_cus == 0) {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) g_cus = pr.multiProcessorCount;
    if (g_cus <= 0) g_cus = 256;
  }
  const int rounds = ((rows + 15) / 16 + CW - 1) / CW;
  if (rounds >= g_cus) return g_cus;
  const int n = (rounds + 7) / 8 * 8;
  return n < 8 ? 8 : n;
}

// this code object's fault word (agn_fault_status ORs it into the reported value)
// (agn_fault_status_async, edge_bwd.hip)
int agn_e16_fault_status_async(int* host_pinned, void* stream) {
  const hipError_t e = hipMemcpyFromSymbolAsync(host_pinned, HIP_SYMBOL(g_e16_fault), sizeof(int), 0,
                                                hipMemcpyDeviceToHost, (hipStream_t)stream);
  return e == hipSuccess ? 0 : (int)e;
}

int agn_e16_fault_status(int* value, int reset) {
  if (!value) return AGN_E_ARG;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(value, HIP_SYMBOL(g_e16_fault), sizeof(int));
  if (e == hipSuccess && reset) {
    const int zero = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_e16_fault), &zero, sizeof(int));
  }
  return e == hipSuccess ? 0 : (int)e;
}

int agn_edge_backward(const agn_edge_bwd_args* a, void* stream) {
  if (!a || a->rows < 1 || a->nblk < 1 || !a->e || !a->proj || !a->src || !a->dst || !a->g2 || !a->ln_g ||
      !a->de || !a->g0 || !a->dw_partial || !a->db_partial || !a->ln_partial || a->dpd)
    return AGN_E_ARG;
  for (int l = 0; l < 4; ++l)
    if (!a->wpk[l]) return AGN_E_ARG;
  if (a->g) hipLaunchKernelGGL(edge16_bwd_kernel<true>, dim3(a->nblk), dim3(NTHR), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL(edge16_bwd_kernel<false>, dim3(a->nblk), dim3(NTHR), 0, (hipStream_t)stream, *a);
  return launch_status();
}

}  // extern "C"
