// dmodel.h — device-side (float) model constants for the SO-ARM101 kernels.
// Built on the host from sim_model_desc (include/soarm_sim.h) by
// soarm_sim.hip:build_dmodel; lives in device global memory and is read with
// wave-uniform (scalar) loads.  Derived constants that MuJoCo recomputes every
// step but that depend only on the model (frictionloss-row impedance, K/B of
// each solref, rotation matrices of fixed quaternions) are folded here.
#pragma once
#include <stdint.h>

#include "../../include/soarm_sim.h"

namespace soarm {

constexpr int MAXB = SIM_MAXBODY, MAXJ = SIM_MAXJNT, MAXD = SIM_MAXDOF, MAXQ = SIM_MAXQ;
constexpr int MAXG = SIM_MAXGEOM, MAXP = SIM_MAXPAIR, MAXU = SIM_MAXU;

struct DModel {
  int nq, nv, nu, ngeom, npair, nact, obs_site, obs_nq;
  int obs_qadr[SIM_MAXOBSQ];
  int iterations, disable_contact, eulerdamp, nhullvert;
  float timestep, impratio, tolerance, _pad0;
  float gravity[4];

  // bodies
  float body_pos[MAXB][3], body_quat[MAXB][4];
  float body_ipos[MAXB][3], body_imat[MAXB][9];  // inertia frame rotation
  float body_mass[MAXB], body_inertia[MAXB][3], body_invweight0[MAXB][2];

  // joints (arm hinges in dof order, then free joints)
  float jnt_pos[MAXJ][3], jnt_axis[MAXJ][3], jnt_range[MAXJ][2];
  float jnt_solimp[MAXJ][5], jnt_KB[MAXJ][2], jnt_margin[MAXJ];
  int jnt_limited[MAXJ];
  float qpos0[MAXQ];

  // dofs
  float dof_armature[MAXD], dof_damping[MAXD], dof_frictionloss[MAXD], dof_invweight0[MAXD];
  float dof_fricR[MAXD], dof_fricB[MAXD];  // frictionloss row: R and B (pos = 0 -> imp = solimp[0])

  // collidable geoms
  int geom_type[MAXG], geom_bodyid[MAXG], geom_hulladr[MAXG], geom_hullnum[MAXG];
  float geom_pos[MAXG][3], geom_mat[MAXG][9], geom_size[MAXG][3];
  float geom_center[MAXG][3], geom_half[MAXG][3], geom_rbound[MAXG];
  float geom_friction[MAXG];

  // candidate pairs (mixed per-pair contact parameters)
  int pair_geom1[MAXP], pair_geom2[MAXP];
  float pair_solimp[MAXP][5], pair_KB[MAXP][2], pair_margin[MAXP], pair_tran[MAXP];
  float pair_friction[MAXP];
  int pair_slot[MAXP];  // first contact slot of the pair in the collide output
  int nslot;            // total contact slots (sum of per-pair capacities)
  int free_diag;        // every free body has ipos = 0 and iquat = 1: its 6x6 M block is diagonal

  // sites
  int site_bodyid[SIM_MAXSITE];
  float site_pos[SIM_MAXSITE][3];

  // actuators (actuator a drives dof a; checked on the host)
  int act_ctrllimited[MAXU], act_forcelimited[MAXU];
  float act_gear[MAXU], act_gain[MAXU], act_bias[MAXU][3];
  float act_ctrlrange[MAXU][2], act_forcerange[MAXU][2];

  // hull data (device pointers)
  const float4* hull_vert;  // xyz, w unused
  const int32_t* hull_adr;  // CSR offsets per global vertex (+1)
  const int32_t* hull_adj;  // local neighbour ids
  const int32_t* hull_seed; // per mesh geom: HULL_NSEED local start vertices for hill climbing
};

// Hill-climbing seeds: the argmax vertex of each hull for HULL_NSEED directions
// on a Fibonacci sphere.  Climbing starts at the best seed for the query
// direction, so a support query walks a few edges instead of crossing the hull.
constexpr int HULL_NSEED = 32;
inline void fibonacci_dir(int k, double d[3]) {
  const double z = 1.0 - (2.0 * k + 1.0) / HULL_NSEED;
  const double r = __builtin_sqrt(1.0 - z * z);
  const double phi = k * 2.399963229728653;  // pi * (3 - sqrt 5)
  d[0] = r * __builtin_cos(phi), d[1] = r * __builtin_sin(phi), d[2] = z;
}

}  // namespace soarm
