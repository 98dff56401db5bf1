// k_ipm128x_f64.hip — double instantiation of the four-wave explicit-inverse IPM for 64 < n <= 128 (k_ipm128x.hpp).
#include "k_ipm128x.hpp"

namespace cmpc {

int launch_ipm128(const IpmArgs<double>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm128x<double, 2>), dim3(B), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_solve128(const IpmArgs<double>& a, const CondenseArgs<double>& c, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!a.qlist[1] || !a.qcount || a.ld < 128) return -1;  // list-driven only
  hipLaunchKernelGGL((k_solve128<double, 2>), dim3(B), dim3(256), 0, stream, a, c);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
