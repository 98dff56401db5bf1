// k_ipm256_f64.hip — double instantiation of the workgroup-tiled IPM (k_ipm256.hpp) for the 128 < n <= 256 class
// (8 waves per QP). The fp64 64 < n <= 128 class runs on k_ipm128x (k_ipm128x_f64.hip).
#include "k_ipm256.hpp"

namespace cmpc {

int launch_ipm256(const IpmArgs<double>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm_tiled<double, 16>), dim3(B), dim3(512), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
