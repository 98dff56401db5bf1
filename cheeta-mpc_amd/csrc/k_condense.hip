// k_condense.hip — stage 1 of the hot path for the workgroup size classes: one workgroup (WAVES wavefronts) per
// QP, the condensing itself in srbd_condense.hpp (shared with the fused 128-class kernel k_solve128).
#include "srbd_condense.hpp"

namespace cmpc {

template <typename T, int NMAX, int WAVES, bool FEET, int HN = MAXN>
__global__ __launch_bounds__(64 * WAVES) void k_srbd_condense(CondenseArgs<T> a) {
  int q = blockIdx.x;
  if (a.qlist) {  // class list: this class's QPs first, the surplus workgroups exit
    if (q >= *a.qcount) return;
    q = a.qlist[q];
    if ((unsigned)q >= gridDim.x) return;  // grid = batch
  }
  if (a.n_lo > 0 && a.nvar[q] <= a.n_lo) return;  // finished (or rejected) by a smaller class
  if (a.skip && a.skip[q]) {                       // converged SQP (CondenseArgs::skip)
    if (threadIdx.x == 0) {  // a rejected / failed QP keeps its status; a solved one keeps its residuals
      if (a.status[q] == CMPC_SUCCESS) a.status[q] = CMPC_STATUS_SKIPPED;
      a.nvar[q] = 0;
    }
    return;
  }
  (void)srbd_condense_qp<T, NMAX, WAVES, false, FEET, HN>(a, q, nullptr);
}

template <typename T>
int launch_srbd_condense(const CondenseArgs<T>& a, int npad, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (npad > a.ld) return -1;
  const bool feet = a.dbar != nullptr;  // foothold columns (cmpc_nlp_solve_batch): the FEET instantiations
  switch (npad) {
    case 72:  // foothold QPs with n <= 72 for k_ipm72 (N <= CMPC_C64_MAXN, h72 set): two waves, four workgroups per CU
      if (!feet || !a.h72) return -1;  // the caller checks N <= CMPC_C64_MAXN
      hipLaunchKernelGGL((k_srbd_condense<T, 80, 2, true, CMPC_C64_MAXN + 1>), dim3(B), dim3(128), 0, stream, a);
      break;
    case 64:
      if (feet) hipLaunchKernelGGL((k_srbd_condense<T, 64, 4, true>), dim3(B), dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((k_srbd_condense<T, 64, 4, false>), dim3(B), dim3(256), 0, stream, a);
      break;
    case 128:
      if (feet) hipLaunchKernelGGL((k_srbd_condense<T, 128, 4, true>), dim3(B), dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((k_srbd_condense<T, 128, 4, false>), dim3(B), dim3(256), 0, stream, a);
      break;
    case 256:  // 17 lower 16x16 tiles per wave; one thread per Bqp column in waves 0-3
      if (feet) hipLaunchKernelGGL((k_srbd_condense<T, 256, 8, true>), dim3(B), dim3(512), 0, stream, a);
      else hipLaunchKernelGGL((k_srbd_condense<T, 256, 8, false>), dim3(B), dim3(512), 0, stream, a);
      break;
    default:
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template int launch_srbd_condense<double>(const CondenseArgs<double>&, int, int, hipStream_t);
template int launch_srbd_condense<float>(const CondenseArgs<float>&, int, int, hipStream_t);

}  // namespace cmpc

#ifdef CMPC_COND_STAMPS
extern "C" int cmpc_cond_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cmpc::cond_stamp_acc), sizeof(unsigned long long) * 16) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cmpc::cond_stamp_acc), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif
