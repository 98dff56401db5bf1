// step_ratio.hpp — fraction-to-boundary candidate selection shared by every IPM kernel.
// The step length is the smallest v / (-d) over a thread's candidates (slack or multiplier v > 0, direction d < 0).
// The candidates are compared by cross-multiplication and divided once at the end (one IEEE division per thread
// instead of one per candidate). The comparison runs in double for both precisions: in fp32 the products v * den and
// num * (-d) overflow to inf or flush to 0 for slacks / steps near 1e+-20, which would skip a binding candidate.
// Host-compilable (tests/cpp/test_step_ratio.cpp checks the extreme-value cases on the CPU).
#pragma once

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace cmpc {

template <typename T>
struct MinRatio {
  double num = 1e300;  // "no candidate": the ratio stays >= 1, so the step is the full step
  double den = 1.0;
  __host__ __device__ inline void cand(T v, T d) {
    const double dv = (double)v, dd = (double)d;
    if (dd < 0.0 && dv * den < num * (-dd)) {
      num = dv;
      den = -dd;
    }
  }
  // min(v / -d) in T (fp32: values above FLT_MAX become inf, which the caller clips to 1)
  __host__ __device__ inline T value() const { return (T)(num / den); }
};

}  // namespace cmpc
