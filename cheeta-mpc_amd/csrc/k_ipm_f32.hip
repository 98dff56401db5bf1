// k_ipm_f32.hip — float instantiations of the batched IPM (k_ipm_impl.hpp); split per precision so the two
// heavily unrolled variants compile in parallel.
#include "k_ipm_impl.hpp"

namespace cmpc {

template <>
int launch_ipm<float>(const IpmArgs<float>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL((k_ipm_reg<float, 64>), dim3(B), dim3(64), 0, stream, a);
  if (a.ld >= 128) hipLaunchKernelGGL((k_ipm_reg<float, 128>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
