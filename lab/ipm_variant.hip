// ipm_variant.hip — one lab variant of the batched IPM kernel (development harness, not part of libcmpc.so).
// Compiled once per variant with -DLAB_HDR=<header> -DLAB_FN=<launcher name> [-DLAB_STAMPS] [-DLAB_WPE=n]
// [-DLAB_PREP2D] ...
#include "cmpc_kernels.hpp"

#define LAB_STR2(x) #x
#define LAB_STR(x) LAB_STR2(x)
#define LAB_CAT2(a, b) a##b
#define LAB_CAT(a, b) LAB_CAT2(a, b)
#ifdef LAB_PRODUCT
// the product kernel also lives in libcmpc.so (the lab's reference): give this copy its own name
#define k_ipm64 LAB_CAT(k_ipm64_, LAB_FN)
#define k_ipm128x LAB_CAT(k_ipm128x_, LAB_FN)
#endif
#include LAB_STR(LAB_HDR)

#ifndef LAB_WPE
#define LAB_WPE 2
#endif

extern "C" int LAB_FN(const cmpc::IpmArgs<double>* a, int B, hipStream_t s, unsigned long long* stamps) {
#if defined(LAB_PRODUCT) && defined(LAB_K128)  // the 64 < n <= 128 class (csrc/k_ipm128x.hpp), 4 waves per QP
  cmpc::IpmArgs<double> b = *a;
  b.stamps = stamps;
  hipLaunchKernelGGL((cmpc::LAB_CAT(k_ipm128x_, LAB_FN)<double, 2>), dim3(B), dim3(256), 0, s, b);
#elif defined(LAB_PRODUCT)  // the product kernel (csrc/k_ipm64.hpp); stamps through IpmArgs when built with CMPC_IPM_STAMPS
  cmpc::IpmArgs<double> b = *a;
  b.stamps = stamps;
  hipLaunchKernelGGL((cmpc::LAB_CAT(k_ipm64_, LAB_FN)<double, LAB_WPE>), dim3(B), dim3(64), 0, s, b);
#else
  hipLaunchKernelGGL((k_ipm_reg<double, 64, LAB_WPE>), dim3(B), dim3(64), 0, s, *a, stamps);
#endif
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// optional input re-layout (not timed): returns args pointing at a variant-owned copy
extern "C" int LAB_CAT(LAB_FN, _prep)(const cmpc::IpmArgs<double>* a, int B, hipStream_t s, cmpc::IpmArgs<double>* out) {
  *out = *a;
#if defined(LAB_PREP2D) && !defined(LAB_PRODUCT)
  static double* H2 = nullptr;
  if (!H2 && hipMalloc((void**)&H2, (size_t)B * a->ld * a->ld * sizeof(double)) != hipSuccess) return -2;
  hipLaunchKernelGGL(k_prep2d<double>, dim3(B), dim3(64), 0, s, a->H, H2, a->nvar, a->ld);
  out->H = H2;
#endif
#ifdef LAB_PRODUCT  // the product packs H in tile order already (launch_pack_qp -> h_index)
  out->stamps = nullptr;
#endif
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
