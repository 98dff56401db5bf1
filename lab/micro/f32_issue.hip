// Microbenchmark (development only): issue cost of the fp32 forms an elimination bulk update can use on gfx950 —
// v_fmac_f32, v_fmac_f32_dpp row_newbcast (k_ipm128x's form, also with its leading s_nop 1), v_pk_fma_f32 with the
// row multiplier broadcast from the low half (op_sel_hi), and v_mov_b32_dpp + 4 v_pk_fma_f32 (the packed bulk of
// one register row of 8 column chunks). W waves per SIMD (256-thread blocks, W blocks per CU), s_memtime per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void kern(float* out, unsigned long long* cyc, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float v[8];
  f2 p[8];
  for (int i = 0; i < 8; ++i) {
    v[i] = a + i;
    p[i] = f2{a + i, b - i};
  }
  f2 bb = {a, b};
  float m = 0.f;
  f2 mm = {0.f, 0.f};
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if constexpr (MODE == 0)
        asm volatile(
            "v_fmac_f32 %0, %8, %9\n\tv_fmac_f32 %1, %8, %9\n\tv_fmac_f32 %2, %8, %9\n\tv_fmac_f32 %3, %8, %9\n\t"
            "v_fmac_f32 %4, %8, %9\n\tv_fmac_f32 %5, %8, %9\n\tv_fmac_f32 %6, %8, %9\n\tv_fmac_f32 %7, %8, %9"
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
            : "v"(a), "v"(b));
      if constexpr (MODE == 1)
        asm volatile(
            "v_fmac_f32_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %1, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %3, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %4, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %5, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %6, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %7, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf"
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
            : "v"(a), "v"(b));
      if constexpr (MODE == 2)
        asm volatile(
            "s_nop 1\n\tv_fmac_f32_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %1, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %3, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %4, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %5, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %6, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "s_nop 1\n\tv_fmac_f32_dpp %7, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf"
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
            : "v"(a), "v"(b));
      if constexpr (MODE == 3)  // 8 packed FMAs = 16 FMAs per lane
        asm volatile(
            "v_pk_fma_f32 %0, %8, %9, %0 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %1, %8, %9, %1 op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %2, %8, %9, %2 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %3, %8, %9, %3 op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %4, %8, %9, %4 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %5, %8, %9, %5 op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %6, %8, %9, %6 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %7, %8, %9, %7 op_sel_hi:[0,1,1]"
            : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7])
            : "v"(bb), "v"(bb));
      if constexpr (MODE == 4)  // one register row of 8 column chunks: row multiplier by DPP, then 4 packed FMAs
        asm volatile(
            "v_mov_b64_dpp %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_pk_fma_f32 %0, %8, %10, %0 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %1, %8, %10, %1 op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %2, %8, %10, %2 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %3, %8, %10, %3 op_sel_hi:[0,1,1]\n\t"
            "v_mov_b64_dpp %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
            "v_pk_fma_f32 %4, %8, %10, %4 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %5, %8, %10, %5 op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %6, %8, %10, %6 op_sel_hi:[0,1,1]\n\tv_pk_fma_f32 %7, %8, %10, %7 op_sel_hi:[0,1,1]"
            : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7]),
              "=&v"(mm)
            : "v"(bb), "v"(bb));
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  float s = m + mm.x;
  for (int i = 0; i < 8; ++i) s += v[i] + p[i].x + p[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) atomicMax(&cyc[MODE], t1 - t0);
}

int main(int argc, char** argv) {
  float* out;
  unsigned long long* cyc;
  const int W = argc > 1 ? atoi(argv[1]) : 1;
  hipMalloc(&out, (size_t)256 * 256 * 8 * sizeof(float));
  hipMalloc(&cyc, 64);
  const int iters = 2048;
  const dim3 grid(256 * W);
  unsigned long long h[5];
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(cyc, 0, 64);
    hipLaunchKernelGGL(kern<0>, grid, dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<1>, grid, dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<2>, grid, dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<3>, grid, dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<4>, grid, dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 40, hipMemcpyDeviceToHost);
  }
  const double n = (double)iters * 16;
  // cycles per instruction of one wave with W waves per SIMD; SIMD throughput in FMA lanes per cycle
  printf("{\"waves_per_simd\": %d, \"v_fmac_f32\": %.2f, \"v_fmac_f32_dpp\": %.2f, \"s_nop1+v_fmac_f32_dpp\": %.2f, "
         "\"v_pk_fma_f32\": %.2f, \"mov_dpp+4pk_per_8chunks\": %.2f, "
         "\"simd_fma_per_clk\": {\"fmac\": %.1f, \"fmac_dpp\": %.1f, \"nop_fmac_dpp\": %.1f, \"pk\": %.1f, "
         "\"mov+pk\": %.1f}}\n",
         W, h[0] / n / 8, h[1] / n / 8, h[2] / n / 8, h[3] / n / 8, h[4] / n / 10, W * 64 * 8 * n / h[0],
         W * 64 * 8 * n / h[1], W * 64 * 8 * n / h[2], W * 64 * 16 * n / h[3], W * 64 * 16 * n / h[4]);
  return 0;
}
