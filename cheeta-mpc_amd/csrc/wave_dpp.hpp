#pragma once
// wave_dpp.hpp — wave64 all-reductions on DPP and the gfx950 permlane swaps (no LDS traffic, ~6 dependent steps):
//   quad_perm xor 1, quad_perm xor 2, row_ror 4, row_ror 8 inside each 16-lane row, then v_permlane16_swap
//   (row pairs) and v_permlane32_swap (wave halves). 64-bit values move as two 32-bit DPP movs.
#include <hip/hip_runtime.h>

namespace cmpc {
namespace wdpp {

template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  int2 v = __builtin_bit_cast(int2, x);
  v.x = __builtin_amdgcn_update_dpp(v.x, v.x, CTRL, 0xf, 0xf, false);
  v.y = __builtin_amdgcn_update_dpp(v.y, v.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, v);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, x), __builtin_bit_cast(int, x),
                                                               CTRL, 0xf, 0xf, false));
}
// partner values across row pairs / wave halves: {x of the lane 16 (32) apart in the pair, ...}
__device__ __forceinline__ void swap16(double x, double& p0, double& p1) {
  const int2 v = __builtin_bit_cast(int2, x);
  const auto a = __builtin_amdgcn_permlane16_swap(v.x, v.x, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(v.y, v.y, false, false);
  p0 = __builtin_bit_cast(double, int2{(int)a[0], (int)b[0]});
  p1 = __builtin_bit_cast(double, int2{(int)a[1], (int)b[1]});
}
__device__ __forceinline__ void swap32(double x, double& p0, double& p1) {
  const int2 v = __builtin_bit_cast(int2, x);
  const auto a = __builtin_amdgcn_permlane32_swap(v.x, v.x, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(v.y, v.y, false, false);
  p0 = __builtin_bit_cast(double, int2{(int)a[0], (int)b[0]});
  p1 = __builtin_bit_cast(double, int2{(int)a[1], (int)b[1]});
}
__device__ __forceinline__ void swap16(float x, float& p0, float& p1) {
  const auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, x), __builtin_bit_cast(int, x), false, false);
  p0 = __builtin_bit_cast(float, (int)a[0]);
  p1 = __builtin_bit_cast(float, (int)a[1]);
}
__device__ __forceinline__ void swap32(float x, float& p0, float& p1) {
  const auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, x), __builtin_bit_cast(int, x), false, false);
  p0 = __builtin_bit_cast(float, (int)a[0]);
  p1 = __builtin_bit_cast(float, (int)a[1]);
}

template <typename T, typename Op>
__device__ __forceinline__ T reduce(T x, Op op) {
  x = op(x, dpp<0xB1>(x));   // quad_perm [1,0,3,2]
  x = op(x, dpp<0x4E>(x));   // quad_perm [2,3,0,1]
  x = op(x, dpp<0x124>(x));  // row_ror:4
  x = op(x, dpp<0x128>(x));  // row_ror:8
  T p0, p1;
  swap16(x, p0, p1);  // row 2k <-> row 2k+1
  x = op(p0, p1);
  swap32(x, p0, p1);  // lanes 0-31 <-> 32-63
  return op(p0, p1);
}

}  // namespace wdpp

template <typename T>
__device__ __forceinline__ T wave_max_dpp(T x) {
  return wdpp::reduce(x, [](T a, T b) { return a > b ? a : b; });
}
template <typename T>
__device__ __forceinline__ T wave_min_dpp(T x) {
  return wdpp::reduce(x, [](T a, T b) { return a < b ? a : b; });
}
template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T x) {
  return wdpp::reduce(x, [](T a, T b) { return a + b; });
}

}  // namespace cmpc
