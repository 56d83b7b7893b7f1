// Issue cost of VALU forms for ONE wave per SIMD (the fused edge backward's chain-wave regime) and
// for two waves per SIMD: cycles per instruction from s_memtime around an unrolled block of
// independent instructions (8 independent chains, inline asm so nothing is folded).
// Build: hipcc --offload-arch=gfx950 -O3 valu_cost.hip -o valu_cost ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int KIND>
__global__ void k(float* out, unsigned long long* cyc, int iters, unsigned long long smask) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  float b = 1.0001f, c = 0.5f;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, pb = {b, b}, pc = {c, c};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {  // v_fma_f32: 8 per round
      REP8(asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                        " v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
    } else if constexpr (KIND == 1) {  // v_pk_fma_f32: 8 per round (16 elements)
      REP8(asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5\n"
                        "v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5"
                        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb), "v"(pc));)
    } else if constexpr (KIND == 2) {  // v_pk_mul_f32
      REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n"
                        "v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));)
    } else if constexpr (KIND == 3) {  // v_cvt_pk_bf16_f32
      REP8(asm volatile("v_cvt_pk_bf16_f32 %0, %0, %8\n v_cvt_pk_bf16_f32 %1, %1, %8\n v_cvt_pk_bf16_f32 %2, %2, %8\n v_cvt_pk_bf16_f32 %3, %3, %8\n"
                        "v_cvt_pk_bf16_f32 %4, %4, %8\n v_cvt_pk_bf16_f32 %5, %5, %8\n v_cvt_pk_bf16_f32 %6, %6, %8\n v_cvt_pk_bf16_f32 %7, %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if constexpr (KIND == 4) {  // v_permlane16_swap
      REP8(asm volatile("v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n v_permlane16_swap_b32 %4, %5\n v_permlane16_swap_b32 %6, %7\n"
                        "v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n v_permlane16_swap_b32 %4, %5\n v_permlane16_swap_b32 %6, %7"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 5) {  // v_add_f32 with DPP row_ror:8 (the butterfly's partner add)
      REP8(asm volatile("v_add_f32_dpp %0, %8, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %1, %8, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                        "v_add_f32_dpp %2, %8, %2 row_ror:8 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %3, %8, %3 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                        "v_add_f32_dpp %4, %8, %4 row_ror:8 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %5, %8, %5 row_ror:8 row_mask:0xf bank_mask:0xf\n"
                        "v_add_f32_dpp %6, %8, %6 row_ror:8 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %7, %8, %7 row_ror:8 row_mask:0xf bank_mask:0xf"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if constexpr (KIND == 6) {  // v_cndmask_b32 (vcc select)
      REP8(asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                        "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");)
    } else if constexpr (KIND == 7) {  // v_pk_add_f32
      REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                        "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                        : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));)
    } else if constexpr (KIND == 8) {  // v_permlane32_swap
      REP8(asm volatile("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n"
                        "v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 10) {  // v_cndmask_b32_e64 with an SGPR-pair mask (the compiler's form)
      REP8(asm volatile("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
                        "v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "s"(smask));)
    } else if constexpr (KIND == 11) {  // v_mov_b32_dpp quad_perm identity with a bank mask (lane merge)
      REP8(asm volatile("v_mov_b32_dpp %0, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n v_mov_b32_dpp %1, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n"
                        "v_mov_b32_dpp %2, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n v_mov_b32_dpp %3, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n"
                        "v_mov_b32_dpp %4, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n v_mov_b32_dpp %5, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n"
                        "v_mov_b32_dpp %6, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc\n v_mov_b32_dpp %7, %8 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xc"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if constexpr (KIND == 12) {  // v_mov_b32 (register copies)
      REP8(asm volatile("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                        "v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if constexpr (KIND == 9) {  // v_pk_max_i16 / v_and (integer)
      REP8(asm volatile("v_pk_max_i16 %0, %0, 0\n v_pk_max_i16 %1, %1, 0\n v_pk_max_i16 %2, %2, 0\n v_pk_max_i16 %3, %3, 0\n"
                        "v_and_b32 %4, %4, %8\n v_and_b32 %5, %5, %8\n v_and_b32 %6, %6, %8\n v_and_b32 %7, %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0[0] + p1[1] + p2[0] + p3[1];
}

template <int KIND>
void run(const char* name, int threads) {
  const int blocks = 256, iters = 2000;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * threads * sizeof(float));
  hipMalloc(&cyc, blocks * (threads / 64) * sizeof(unsigned long long));
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 10, 0x5555555555555555ull);
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 0x5555555555555555ull);
  hipDeviceSynchronize();
  const int n = blocks * (threads / 64);
  unsigned long long* h = new unsigned long long[n];
  hipMemcpy(h, cyc, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < n; ++i) s += h[i];
  s /= n;
  printf("%-22s waves/SIMD %d: %.2f cycles per instruction per wave\n", name, threads / 256, s / (iters * 64.0));
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int t : {256, 512}) {
    run<0>("v_fma_f32", t);
    run<1>("v_pk_fma_f32", t);
    run<2>("v_pk_mul_f32", t);
    run<7>("v_pk_add_f32", t);
    run<3>("v_cvt_pk_bf16_f32", t);
    run<4>("v_permlane16_swap", t);
    run<8>("v_permlane32_swap", t);
    run<5>("v_add_f32_dpp", t);
    run<6>("v_cndmask_b32", t);
    run<9>("v_pk_max_i16/v_and", t);
    run<10>("v_cndmask_b32_e64 sgpr", t);
    run<11>("v_mov_b32_dpp bankmask", t);
    run<12>("v_mov_b32", t);
  }
  return 0;
}
