// k_ipm_f32.hip — float instantiation of the n <= 64 IPM (k_ipm64.hpp).
#include "k_ipm64.hpp"

namespace cmpc {

int launch_ipm64(const IpmArgs<float>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm64<float, 3>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_solve64(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL((k_solve64<float, 3>), dim3(B), dim3(64), 0, stream, a, c);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


}  // namespace cmpc
