// k_ipm128x_f32.hip — float instantiation of the four-wave explicit-inverse IPM for 64 < n <= 128 (k_ipm128x.hpp).
#include "k_ipm128x.hpp"

// workgroups per CU of the fused fp32 128 class (lab A/B: -DCMPC_SOLVE128F_MINB=3 gives 168 VGPRs, no scratch)
#ifndef CMPC_SOLVE128F_MINB
#define CMPC_SOLVE128F_MINB 4
#endif

namespace cmpc {

int launch_ipm128(const IpmArgs<float>& a, int B, hipStream_t stream) {
  // four workgroups per CU (128 VGPRs; a few spill outside the elimination): 1.89 ms vs 2.05 ms at three
  hipLaunchKernelGGL((k_ipm128x<float, 4>), dim3(B), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_solve128(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!a.qlist[1] || !a.qcount || a.ld < 128) return -1;  // list-driven only
  hipLaunchKernelGGL((k_solve128<float, CMPC_SOLVE128F_MINB>), dim3(B), dim3(256), 0, stream, a, c);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
