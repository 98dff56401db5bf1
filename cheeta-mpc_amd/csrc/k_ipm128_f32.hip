// k_ipm128_f32.hip — the 64 < n <= 128 size class in float (k_ipm_impl.hpp: row-per-lane register IPM, RPL = 2).
#include "k_ipm_impl.hpp"

namespace cmpc {

int launch_ipm128(const IpmArgs<float>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm_reg<float, 128, 1>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
