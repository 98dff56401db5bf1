// k_ipm_f32.hip — float instantiation of the n <= 64 IPM (k_ipm64.hpp).
#include <cstdlib>

#include "k_ipm64.hpp"

namespace cmpc {

int launch_ipm64(const IpmArgs<float>& a, int B, hipStream_t stream) {
  hipLaunchKernelGGL((k_ipm64<float, 3>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_solve64q(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, int qpw, hipStream_t stream) {
  static const unsigned spin_max = [] {  // bound of a wave's wait for a work item (~1.5 s at the default)
    const char* e = std::getenv("CMPC_ITEMS_SPIN");
    return e ? (unsigned)std::strtoul(e, nullptr, 10) : (1u << 24);
  }();
  if (B <= 0) return 0;
  if (qpw < 1 || qpw > kSolve64qMaxQpw) return -1;
  hipLaunchKernelGGL((k_solve64q<float>), dim3((B + qpw - 1) / qpw), dim3(512), 0, stream, a, c, B, qpw, spin_max);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_solve64(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL((k_solve64<float, 3>), dim3(B), dim3(64), 0, stream, a, c);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


}  // namespace cmpc
