// k_ipm72_f64.hip — float instantiation of the bordered one-wave IPM for 64 < n <= 72 (k_ipm72.hpp).
#include "k_ipm72.hpp"

namespace cmpc {

int launch_ipm72(const IpmArgs<float>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!a.qlist[1] || !a.qcount || a.ld < 128) return -1;  // list-driven only
  hipLaunchKernelGGL((k_ipm72<float, 3>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
