// Microbenchmark (development only): cycles per v_mfma_f64_16x16x4_f64 and whether fp64 VALU FMAs co-execute
// with it on gfx950. One wave per SIMD (256 threads per block, 1 block per CU), s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void kern(double* out, unsigned long long* cyc, int iters) {
  d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0, acc4 = acc0, acc5 = acc0, acc6 = acc0, acc7 = acc0;
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  int ia = threadIdx.x, i0 = 0, i1 = 0, i2 = 0, i3 = 0, i4 = 0, i5 = 0, i6 = 0, i7 = 0;
  double v0 = a, v1 = b, v2 = a + b, v3 = a - b, v4 = a, v5 = b, v6 = a, v7 = b;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0 || MODE == 2) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
    }
    if (MODE == 6) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
      acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc4, 0, 0, 0);
      acc5 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc5, 0, 0, 0);
      acc6 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc6, 0, 0, 0);
      acc7 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc7, 0, 0, 0);
    }
    if (MODE == 7) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
    }
    if (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        asm volatile(
            "v_fmac_f64_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %1, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %3, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %4, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %5, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %6, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %7, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf"
            : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
            : "v"(a), "v"(b));
      }
    }
    if (MODE == 4) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        asm volatile(
            "v_fmac_f64 %0, %8, %9\n\t"
            "v_fmac_f64 %1, %8, %9\n\t"
            "v_fmac_f64 %2, %8, %9\n\t"
            "v_fmac_f64 %3, %8, %9\n\t"
            "v_fmac_f64 %4, %8, %9\n\t"
            "v_fmac_f64 %5, %8, %9\n\t"
            "v_fmac_f64 %6, %8, %9\n\t"
            "v_fmac_f64 %7, %8, %9"
            : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)
            : "v"(a), "v"(b));
      }
    }
    if (MODE == 5) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        asm volatile(
            "v_mov_b32_dpp %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %1, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %3, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %5, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %6, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_mov_b32_dpp %7, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf"
            : "=v"(i0), "=v"(i1), "=v"(i2), "=v"(i3), "=v"(i4), "=v"(i5), "=v"(i6), "=v"(i7)
            : "v"(ia));
        ia += i0 ^ i1 ^ i2 ^ i3 ^ i4 ^ i5 ^ i6 ^ i7;
      }
    }
    if (MODE == 1 || MODE == 2) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        v0 = fma(v0, b, a); v1 = fma(v1, b, a); v2 = fma(v2, b, a); v3 = fma(v3, b, a);
        v4 = fma(v4, b, a); v5 = fma(v5, b, a); v6 = fma(v6, b, a); v7 = fma(v7, b, a);
      }
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 256 + threadIdx.x] = acc0[0] + acc1[1] + acc2[2] + acc3[3] + acc4[0] + acc5[1] + acc6[2] + acc7[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + ia;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[MODE] = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 8); hipMalloc(&cyc, 64);
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern<0>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<1>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<2>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<3>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<4>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<5>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<6>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL(kern<7>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
  }
  unsigned long long h[8];
  hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
  printf("{\"mfma_f64_8chains_cycles_per_mfma\": %.2f, \"mfma_f64_1chain_latency\": %.2f}\n", (double)h[6] / iters / 8,
         (double)h[7] / iters);
  printf("{\"dpp_f64_fmac_cycles\": %.2f, \"asm_f64_fmac_cycles\": %.2f, \"mov_b32_dpp_cycles_plus_xor\": %.2f}\n",
         (double)h[3] / iters / 128, (double)h[4] / iters / 128, (double)h[5] / iters / 128);
  printf("{\"mfma_f64_16x16x4_cycles\": %.2f, \"valu_f64_fma_cycles\": %.2f, \"both_cycles_per_iter\": %.1f, "
         "\"mfma_only_per_iter\": %.1f, \"valu_only_per_iter\": %.1f}\n",
         (double)h[0] / iters / 4, (double)h[1] / iters / 128, (double)h[2] / iters, (double)h[0] / iters,
         (double)h[1] / iters);
  return 0;
}
