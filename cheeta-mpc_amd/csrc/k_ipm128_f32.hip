// k_ipm128_f32.hip — the 64 < n <= 128 size class in float (k_ipm_impl.hpp: one wave per QP, lower rows l and l + 64 per lane).
#include <cstdlib>

#include "k_ipm_impl.hpp"

namespace cmpc {

int launch_ipm128x_f32(const IpmArgs<float>& a, int B, hipStream_t stream);

int launch_ipm128(const IpmArgs<float>& a, int B, hipStream_t stream) {
  static const bool old = getenv("CMPC_F32_OLD128") != nullptr;  // A/B switch (experiment)
  if (!old) return launch_ipm128x_f32(a, B, stream);
  hipLaunchKernelGGL((k_ipm128<float, 1>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
