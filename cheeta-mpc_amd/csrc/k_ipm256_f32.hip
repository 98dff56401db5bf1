// k_ipm256_f32.hip — the 128 < n <= 256 size class in float (k_ipm256.hpp: one 8-wave workgroup per QP).
#include "k_ipm256.hpp"

namespace cmpc {

int launch_ipm256(const IpmArgs<float>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm_tiled<float, 16>), dim3(B), dim3(512), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
