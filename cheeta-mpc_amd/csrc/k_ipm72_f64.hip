// k_ipm72_f64.hip — double instantiation of the bordered one-wave IPM for 64 < n <= 72 (k_ipm72.hpp).
#include "k_ipm72.hpp"

namespace cmpc {

int launch_ipm72(const IpmArgs<double>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!a.qlist[1] || !a.qcount || a.ld < 128) return -1;  // list-driven only
  hipLaunchKernelGGL((k_ipm72<double, 2>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc

#ifdef CMPC_IPM72_STAMPS
extern "C" int cmpc_ipm72_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cmpc::ipm72_stamp_acc), sizeof(unsigned long long) * 16) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cmpc::ipm72_stamp_acc), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif
