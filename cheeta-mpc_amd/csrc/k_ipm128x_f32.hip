// k_ipm128x_f32.hip — float instantiation of the four-wave explicit-inverse IPM for 64 < n <= 128 (k_ipm128x.hpp).
#include "k_ipm128x.hpp"

namespace cmpc {

int launch_ipm128(const IpmArgs<float>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm128x<float, 3>), dim3(B), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
