// k_ipm256_f64.hip — double instantiations of the workgroup-tiled IPM (k_ipm256.hpp): the 128 < n <= 256 class
// (8 waves per QP) and, in fp64, the 64 < n <= 128 class (4 waves per QP).
#include "k_ipm256.hpp"

namespace cmpc {

int launch_ipm256(const IpmArgs<double>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm_tiled<double, 16>), dim3(B), dim3(512), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_ipm128(const IpmArgs<double>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm_tiled<double, 8>), dim3(B), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
