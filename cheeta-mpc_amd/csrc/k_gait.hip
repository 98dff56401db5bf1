// k_gait.hip — per-QP contact tables from gait templates on the device: the batched analogue of
// GaitSchedule::getModeSchedule / tileModeSequenceTemplate (ocs2_legged_robot/src/gait/GaitSchedule.cpp:78-127)
// followed by modeNumber2StanceLeg (include/ocs2_legged_robot/gait/MotionPhaseDefinition.h:69-124) at the start of
// every horizon interval. Semantics in include/cmpc/cmpc.h; restated in oracle/cmpc_oracle.c:oracle_gait_contact.
//
// One thread per (QP, step): a handful of scalar ops plus a <= 16-entry scan of the template in LDS; the output is
// 4 contact bytes per thread, written as one 32-bit word (coalesced). The step time is formed without contraction
// (__dmul_rn / __dadd_rn) so the table is bit-identical to the oracle's.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <new>

#include "cmpc/cmpc.h"

struct cmpc_gait_table {
  int n;
  int leg_map[4];
  cmpc_gait* d_gaits;  // device copy
};

namespace cmpc {
namespace {

struct GaitArgs {
  const cmpc_gait* gaits;
  int n_gaits;
  int leg_map[4];
  const int* gait_id;
  const double* t_start;
  double t0, dt;
  int N, B;
  uint8_t* contact;
};

constexpr int MODE_STANCE = 15;  // MotionPhaseDefinition.h:63

__global__ __launch_bounds__(256) void k_gait_contact(GaitArgs a) {
  __shared__ cmpc_gait s_g[4];  // the first templates cached (the common case: a handful of gaits)
  const int tid = threadIdx.x;
  const int ncache = a.n_gaits < 4 ? a.n_gaits : 4;
  for (int i = tid; i < ncache * (int)(sizeof(cmpc_gait) / 4); i += blockDim.x)
    reinterpret_cast<int*>(s_g)[i] = reinterpret_cast<const int*>(a.gaits)[i];
  __syncthreads();
  const long e = (long)blockIdx.x * blockDim.x + tid;
  if (e >= (long)a.B * a.N) return;
  const int q = (int)(e / a.N), k = (int)(e % a.N);
  const int id = a.gait_id[q];
  uint32_t word = 0;
  if (id >= 0 && id < a.n_gaits) {
    const cmpc_gait& g = id < 4 ? s_g[id] : a.gaits[id];
    const double t = __dadd_rn(a.t0, __dmul_rn((double)k, a.dt));
    const double ts = a.t_start[q];
    int mode = MODE_STANCE;
    if (!(t < ts)) {
      const int M = g.n_modes;
      const double t0g = g.switching_time[0];
      const double period = g.switching_time[M] - t0g;
      const double tau = __dadd_rn(fmod(t - ts, period), t0g);
      int i = 0;
      for (int j = 1; j < M; ++j) i = (g.switching_time[j] <= tau) ? j : i;
      mode = g.mode[i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t st = (uint32_t)(mode >> (3 - j)) & 1u;  // {LF, RF, LH, RH} = bits 3..0
      word |= st << (8 * a.leg_map[j]);
    }
  }
  reinterpret_cast<uint32_t*>(a.contact)[e] = word;
}

struct Builtin {
  const char* name;
  int n;
  int mode[CMPC_GAIT_MAX_MODES];
  double t[CMPC_GAIT_MAX_MODES + 1];
};
// ModeNumber values (MotionPhaseDefinition.h:48-63)
enum { FLY = 0, RH = 1, LH = 2, LH_RH = 3, RF = 4, RF_RH = 5, RF_LH = 6, RF_LH_RH = 7, LF = 8, LF_RH = 9, LF_LH = 10,
       LF_LH_RH = 11, LF_RF = 12, LF_RF_RH = 13, LF_RF_LH = 14, STANCE = 15 };
// ocs2_legged_robot/config/command/gait.info (pinned by tests/golden/gait_templates.json)
const Builtin kBuiltins[] = {
    {"stance", 1, {STANCE}, {0.0, 0.5}},
    {"trot", 2, {LF_RH, RF_LH}, {0.0, 0.35, 0.70}},
    {"standing_trot", 4, {LF_RH, STANCE, RF_LH, STANCE}, {0.00, 0.30, 0.35, 0.65, 0.70}},
    {"flying_trot", 4, {LF_RH, FLY, RF_LH, FLY}, {0.00, 0.27, 0.30, 0.57, 0.60}},
    {"pace", 4, {LF_LH, FLY, RF_RH, FLY}, {0.0, 0.28, 0.30, 0.58, 0.60}},
    {"standing_pace", 4, {LF_LH, STANCE, RF_RH, STANCE}, {0.0, 0.30, 0.35, 0.65, 0.70}},
    {"dynamic_walk", 6, {LF_RF_RH, RF_RH, RF_LH_RH, LF_RF_LH, LF_LH, LF_LH_RH}, {0.0, 0.2, 0.3, 0.5, 0.7, 0.8, 1.0}},
    {"static_walk", 4, {LF_RF_RH, RF_LH_RH, LF_RF_LH, LF_LH_RH}, {0.0, 0.3, 0.6, 0.9, 1.2}},
    {"amble", 4, {RF_LH, LF_LH, LF_RH, RF_RH}, {0.0, 0.15, 0.40, 0.55, 0.80}},
    {"lindyhop", 12, {LF_RH, STANCE, RF_LH, STANCE, LF_LH, RF_RH, LF_LH, STANCE, RF_RH, LF_LH, RF_RH, STANCE},
     {0.00, 0.35, 0.45, 0.80, 0.90, 1.125, 1.35, 1.70, 1.80, 2.025, 2.25, 2.60, 2.70}},
    {"skipping", 8, {LF_RH, FLY, LF_RH, FLY, RF_LH, FLY, RF_LH, FLY},
     {0.00, 0.27, 0.30, 0.57, 0.60, 0.87, 0.90, 1.17, 1.20}},
    {"pawup", 1, {RF_LH_RH}, {0.0, 2.0}},
};

bool gait_ok(const cmpc_gait& g) {
  if (g.n_modes < 1 || g.n_modes > CMPC_GAIT_MAX_MODES) return false;
  for (int i = 0; i < g.n_modes; ++i) {
    if (g.mode[i] < 0 || g.mode[i] > 15) return false;
    if (!(g.switching_time[i + 1] > g.switching_time[i])) return false;
  }
  return std::isfinite(g.switching_time[0]) && std::isfinite(g.switching_time[g.n_modes]);
}

}  // namespace
}  // namespace cmpc

using namespace cmpc;

extern "C" {

int cmpc_gait_builtin(const char* name, cmpc_gait* out) {
  if (!name || !out) return CMPC_ERR_ARG;
  for (const Builtin& b : kBuiltins) {
    if (std::strcmp(b.name, name) != 0) continue;
    std::memset(out, 0, sizeof(*out));
    out->n_modes = b.n;
    for (int i = 0; i < b.n; ++i) out->mode[i] = b.mode[i];
    for (int i = 0; i <= b.n; ++i) out->switching_time[i] = b.t[i];
    return CMPC_OK;
  }
  return CMPC_ERR_ARG;
}

int cmpc_gait_table_create(const cmpc_gait* gaits, int n, const int* leg_map, cmpc_gait_table** out) {
  if (!out || !gaits || n < 1 || n > CMPC_GAIT_MAX_TEMPLATES) return CMPC_ERR_ARG;
  *out = nullptr;
  for (int i = 0; i < n; ++i)
    if (!gait_ok(gaits[i])) return CMPC_ERR_ARG;
  static const int kDefaultMap[4] = {0, 1, 3, 2};
  const int* lm = leg_map ? leg_map : kDefaultMap;
  int seen = 0;
  for (int j = 0; j < 4; ++j) {
    if (lm[j] < 0 || lm[j] > 3 || (seen >> lm[j]) & 1) return CMPC_ERR_ARG;
    seen |= 1 << lm[j];
  }
  cmpc_gait_table* t = new (std::nothrow) cmpc_gait_table();
  if (!t) return CMPC_ERR_ARG;
  t->n = n;
  for (int j = 0; j < 4; ++j) t->leg_map[j] = lm[j];
  if (hipMalloc((void**)&t->d_gaits, sizeof(cmpc_gait) * n) != hipSuccess ||
      hipMemcpy(t->d_gaits, gaits, sizeof(cmpc_gait) * n, hipMemcpyHostToDevice) != hipSuccess) {
    if (t->d_gaits) (void)hipFree(t->d_gaits);
    delete t;
    return CMPC_ERR_HIP;
  }
  *out = t;
  return CMPC_OK;
}

int cmpc_gait_table_destroy(cmpc_gait_table* t) {
  if (!t) return CMPC_ERR_ARG;
  if (t->d_gaits) (void)hipFree(t->d_gaits);
  delete t;
  return CMPC_OK;
}

int cmpc_gait_contact_batch(const cmpc_gait_table* t, int B, const int* d_gait_id, const double* d_t_start, double t0,
                            double dt, int N, uint8_t* d_contact, void* stream) {
  if (!t || B < 0 || N < 1 || !(dt > 0.0) || !std::isfinite(t0) || !d_gait_id || !d_t_start || !d_contact)
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  GaitArgs a;
  a.gaits = t->d_gaits;
  a.n_gaits = t->n;
  for (int j = 0; j < 4; ++j) a.leg_map[j] = t->leg_map[j];
  a.gait_id = d_gait_id;
  a.t_start = d_t_start;
  a.t0 = t0;
  a.dt = dt;
  a.N = N;
  a.B = B;
  a.contact = d_contact;
  const long total = (long)B * N;
  hipLaunchKernelGGL(k_gait_contact, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? CMPC_OK : CMPC_ERR_HIP;
}

}  // extern "C"
