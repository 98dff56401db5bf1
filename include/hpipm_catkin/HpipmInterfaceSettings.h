/*
 * HpipmInterfaceSettings.h — hpipm_interface::Settings (reference
 * ocs2_sqp/hpipm_catkin/include/hpipm_catkin/HpipmInterfaceSettings.h:44-57), same fields and defaults.
 *
 * What the MI355X engine does with them (cheeta-mpc_amd/host/HpipmInterface.cpp): the OCP path is a direct
 * equality-constrained solve, not an interior point method, so only reg_prim acts (added to the input Hessians, as
 * HPIPM's primal regularisation); hpipmMode, iter_max, alpha_min, mu0, the tolerances, warm_start, pred_corr and
 * ric_alg are stored and printed but cannot change the result of a problem without inequalities. The centroidal
 * engine's interior point method (cmpc_settings) honours every field.
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
