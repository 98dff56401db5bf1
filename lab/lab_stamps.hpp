#pragma once
// lab_stamps.hpp — in-kernel s_memtime stamps for the lab (development harness only; never in libcmpc.so).
// Each segment's cycles are added into a scalar sum; lane 0 stores the 8 sums + the total once at the end.
#include <hip/hip_runtime.h>

__device__ __forceinline__ unsigned long long lab_memtime() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

#ifdef LAB_STAMPS
#define STAMP_DECL                          \
  unsigned long long st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  const unsigned long long st_t0_ = lab_memtime();          \
  unsigned long long st_prev_ = st_t0_
#define STAMP(k)                                  \
  do {                                            \
    const unsigned long long t_ = lab_memtime();  \
    st_acc_[k] += t_ - st_prev_;                  \
    st_prev_ = t_;                                \
  } while (0)
#define STAMP_STORE(ptr, q)                                                   \
  do {                                                                        \
    const unsigned long long t_ = lab_memtime();                              \
    if ((ptr) && threadIdx.x == 0) {                                          \
      for (int k_ = 0; k_ < 8; ++k_) (ptr)[(size_t)(q) * 9 + k_] = st_acc_[k_]; \
      (ptr)[(size_t)(q) * 9 + 8] = t_ - st_t0_;                               \
    }                                                                         \
  } while (0)
#else
#define STAMP_DECL (void)0
#define STAMP(k) (void)0
#define STAMP_STORE(ptr, q) (void)(ptr)
#endif
