// k_ric_f64.hip — double instantiations of the stage-wise hot path (k_ric.hpp).
#include "k_ric.hpp"

namespace cmpc {

template <>
int launch_ric<double>(const RicArgs<double>& a, int tpl, int grid, hipStream_t stream) {
  if (grid <= 0) return 0;
  if (a.N > CMPC_RIC_MAXN || (tpl == 1 && a.N > 16 && !a.qlist)) return -1;
  if (tpl == 1 && a.N <= 10)
    hipLaunchKernelGGL((k_ric<double, 1, 10, 2>), dim3(grid), dim3(64), 0, stream, a);
  else if (tpl == 1)
    hipLaunchKernelGGL((k_ric<double, 1, CMPC_RIC_MAXN, 2>), dim3(grid), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL((k_ric<double, 2, CMPC_RIC_MAXN, 1>), dim3(grid), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
