// k_ipm_f32.hip — float instantiations of the batched IPM (k_ipm_impl.hpp); split per precision so the two
// heavily unrolled variants compile in parallel.
#include <cstdlib>

#include "k_ipm_impl.hpp"

#ifndef CMPC_IPM64_WPE_DEFAULT
#define CMPC_IPM64_WPE_DEFAULT 2
#endif

namespace cmpc {

template <>
int launch_ipm<float>(const IpmArgs<float>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  static const int wpe = [] {
    const char* e = getenv("CMPC_IPM_WPE");  // tuning knob: waves per SIMD the n<=64 class is compiled for
    return e ? atoi(e) : CMPC_IPM64_WPE_DEFAULT;
  }();
  if (wpe == 1) hipLaunchKernelGGL((k_ipm_reg<float, 64, 1>), dim3(B), dim3(64), 0, stream, a);
  else hipLaunchKernelGGL((k_ipm_reg<float, 64, 2>), dim3(B), dim3(64), 0, stream, a);
  if (a.ld >= 128) hipLaunchKernelGGL((k_ipm_reg<float, 128, 1>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
