// k_ipm_f64.hip — double instantiation of the n <= 64 IPM (k_ipm64.hpp) and the batched-IPM dispatcher.
#include "k_ipm64.hpp"

namespace cmpc {

int launch_ipm64(const IpmArgs<double>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm64<double, 2>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_solve64(const IpmArgs<double>& a, const CondenseArgs<double>& c, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL((k_solve64<double, 2>), dim3(B), dim3(64), 0, stream, a, c);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


// every QP is served by the size class of its condensed size (the other class's blocks exit at once)
template <typename T>
int launch_ipm(const IpmArgs<T>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  int r = launch_ipm64(a, B, stream);
  if (r == 0 && a.ld >= 128) r = launch_ipm128(a, B, stream);
  if (r == 0 && a.ld >= 256) r = launch_ipm256(a, B, stream);
  return r;
}
template int launch_ipm<double>(const IpmArgs<double>&, int, hipStream_t);
template int launch_ipm<float>(const IpmArgs<float>&, int, hipStream_t);

}  // namespace cmpc
