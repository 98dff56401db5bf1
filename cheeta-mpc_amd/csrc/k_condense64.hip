// k_condense64.hip — stage 1 of the hot path for QPs whose condensed size is n <= 64 (every trot QP at N <= 10):
// SRBD linearisation, horizon propagation, dense condensing and friction-pyramid stacking. One wavefront per QP.
//
// Reference semantics (paths relative to the reference repo), identical to k_condense.hip:
//   dynamics  CentroidalMPC.cpp:85-92 forward Euler, lever arm linearised at r = p_{i,k} - c^ref_k, p the
//             stance foot position of stance_point (cmpc_device.hpp: :93 pinning, node 0 = current foot :165-167)
//   horizon   CentroidalMPC.cpp:159-176 multiple shooting -> condensed X = Aqp x0 + Bqp U
//   cost      CentroidalMPC.cpp:203-231 -> H = Bqp' Qbar Bqp + Rbar, g = Bqp' Qbar (Aqp x0 - Xref) + rbar (A.3)
//   f^des     CentroidalMPC.cpp:326-335 (m*9.81/n_stance, "mpc table invalid" when a step has no stance leg)
//   pyramid   CentroidalMPC.cpp:179-201; swing legs (0 <= F f <= 0) eliminated (A.4)
//
// MI355X mapping:
//   - lane c owns column c of Bqp (one stance force component) and propagates its 13-state image through the SRBD
//     transition with the A_k sparsity (13 FMAs per step); lanes 0..12 propagate the free response Aqp x0 and
//     publish Q_k (x_hat_k - xref_k) through LDS;
//   - each step the block row Bqp_k (13 x 64, padded to 16 rows) is staged in LDS twice (plain and Q_k-scaled) and
//     H += Bqp_k' Q_k Bqp_k runs on the matrix cores over the lower 16 x 16 tiles whose columns are already active
//     (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32), so the MFMA work follows the block-triangular Bqp;
//   - the f64 MFMA accumulator layout (lane 16g + col, register q <-> row g + 4q, column col) IS the 4 x 16-cyclic
//     tile of k_ipm64, so tile (I, J) register q is H register 4(4I + q) + J; for f32 the A-operand rows are
//     permuted so that the f32 layout (row 4g + q) lands on the same rows;
//   - upper tiles are the lower tiles transposed once through LDS; Rbar (force tracking + force-rate coupling) and
//     the identity padding are added per lane in the epilogue;
//   - H leaves as 64 coalesced 512-B rows per QP in the order k_ipm64 reads it (h_index).
// QPs with n > 64 are left to the bigger classes (k_condense.hip): their status is not written here, only nvar = n as
// a hint, so that k_srbd_condense can drop every QP this kernel finished without re-reading its contact table.
#include "condense64.hpp"

namespace cmpc {

template <typename T>
__global__ __launch_bounds__(64) void k_condense64(CondenseArgs<T> a) {
  if (a.skip && a.skip[blockIdx.x]) {  // converged SQP (CondenseArgs::skip)
    if (threadIdx.x == 0) {  // a rejected / failed QP keeps its status; a solved one keeps its residuals
      if (a.status[blockIdx.x] == CMPC_SUCCESS) a.status[blockIdx.x] = CMPC_STATUS_SKIPPED;
      a.nvar[blockIdx.x] = 0;
    }
    return;
  }
  __shared__ c64::C64Lds<T> S;
  T K[64], g, mu;
  (void)condense64_qp<T>(a, (int)blockIdx.x, S, K, g, mu);
}

template <typename T>
int launch_condense64(const CondenseArgs<T>& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL((k_condense64<T>), dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template int launch_condense64<double>(const CondenseArgs<double>&, int, hipStream_t);
template int launch_condense64<float>(const CondenseArgs<float>&, int, hipStream_t);

}  // namespace cmpc
