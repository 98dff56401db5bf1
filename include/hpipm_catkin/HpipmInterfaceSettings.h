/*
 * HpipmInterfaceSettings.h — hpipm_interface::Settings (reference
 * ocs2_sqp/hpipm_catkin/include/hpipm_catkin/HpipmInterfaceSettings.h:44-57), same fields and defaults.
 *
 * What the MI355X engine does with them (cheeta-mpc_amd/host/HpipmInterface.cpp -> cmpc_ocp_create / set_settings):
 * the OCP path runs HPIPM's interior point method on the device (k_ocp_ipm), so iter_max, alpha_min, mu0 and the four
 * tolerances act as in HPIPM; reg_prim is the factorisation's primal regularisation (the returned trajectory is the
 * unregularised problem's). pred_corr must be 1 (the Mehrotra corrector HPIPM's default runs; 0 is refused), ric_alg
 * 0 or 1 (both give the same Newton steps here: one factorisation form), hpipmMode is accepted and stored (the
 * device's tolerances, not the mode's presets, decide); warm_start != 0 is HPIPM's primal warm start: the mirror keeps
 * the last solution of the same size and the device solve starts x, u from it (slacks and multipliers by the
 * cold-start rule); at the default warm_start = 0 every solve cold-starts, as HPIPM's does.
 * The centroidal engine's interior point method (cmpc_settings) honours every field.
 */
#pragma once

#include <ostream>

#include "hpipm_catkin/ocs2_types.h"

namespace ocs2 {
namespace hpipm_interface {

struct Settings {
  hpipm_mode hpipmMode = hpipm_mode::SPEED;
  int iter_max = 30;
  double alpha_min = 1e-12;
  double mu0 = 1e1;
  double tol_stat = 1e-6;  // res_g_max
  double tol_eq = 1e-8;    // res_b_max
  double tol_ineq = 1e-8;  // res_d_max
  double tol_comp = 1e-8;  // res_m_max
  double reg_prim = 1e-12;
  int warm_start = 0;
  int pred_corr = 1;
  int ric_alg = 0;  // square root Riccati recursion
};

/* the reference's printout (HpipmInterfaceSettings.cpp) */
std::ostream& operator<<(std::ostream& stream, const Settings& settings);

}  // namespace hpipm_interface
}  // namespace ocs2
