// k_ric_f32.hip — float instantiations of the stage-wise hot path (k_ric.hpp).
// Instantiations by the largest QP a launch can see (nmax = 3 x force triples): the LDS factor store holds
// sum_k m_k (m_k + 1) / 2 + 12 m_k <= 18.5 nmax values.
#include "k_ric.hpp"

namespace cmpc {

template <>
int launch_ric<float>(const RicArgs<float>& a, int nmax, int grid, hipStream_t stream) {
  if (grid <= 0) return 0;
  if (a.N > CMPC_RIC_MAXN) return -1;
  if (a.N <= 10)
    hipLaunchKernelGGL((k_ric<float, 1, 10, 2220, 2>), dim3(grid), dim3(64), 0, stream, a);
  else if (nmax <= 128)
    hipLaunchKernelGGL((k_ric<float, 1, CMPC_RIC_MAXN, 2368, 2>), dim3(grid), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL((k_ric<float, 2, CMPC_RIC_MAXN, 4662, 1>), dim3(grid), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
