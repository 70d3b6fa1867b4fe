// dmodel.h — device-side (float) model constants for the SO-ARM101 kernels.
// Built on the host from sim_model_desc (include/soarm_sim.h) by
// soarm_sim.hip:build_dmodel; lives in device global memory and is read with
// wave-uniform (scalar) loads.  Derived constants that MuJoCo recomputes every
// step but that depend only on the model (frictionloss-row impedance, K/B of
// each solref, rotation matrices of fixed quaternions) are folded here.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/soarm_sim.h"

namespace soarm {

constexpr int MAXB = SIM_MAXBODY, MAXJ = SIM_MAXJNT, MAXD = SIM_MAXDOF, MAXQ = SIM_MAXQ;
constexpr int MAXG = SIM_MAXGEOM, MAXP = SIM_MAXPAIR, MAXU = SIM_MAXU;

struct DModel {
  int nq, nv, nu, ngeom, npair, nact, obs_site, obs_nq;
  int obs_qadr[SIM_MAXOBSQ];
  int iterations, disable_contact, eulerdamp, nhullvert;
  int ccd, _pad_ccd[3];  // SIM_CCD_* (convex-convex narrowphase)
  float timestep, impratio, tolerance, pgs_scale;  // pgs_scale = 1 / (meaninertia * max(1, nv))
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
  float geom_cbody[MAXG][3];  // the collision-box centre in the body frame: pos + mat centre (midphase)
  float geom_friction[MAXG];

  // candidate pairs (mixed per-pair contact parameters)
  int pair_geom1[MAXP], pair_geom2[MAXP];
  float pair_solimp[MAXP][5], pair_KB[MAXP][2], pair_margin[MAXP], pair_tran[MAXP];
  float pair_friction[MAXP];
  int pair_slot[MAXP];  // first contact slot of the pair in the collide output
  int pair_body1[MAXP], pair_body2[MAXP];  // geom_bodyid of the pair's geoms
  int pair_cap[MAXP];                      // contact slots of the pair (1 or PAIR_MAXCON)
  // multi-contact pairs (cap > 1, at most 16): index q into the collide output's count word,
  // which holds (contacts - 1) in bits 2q, 2q+1 (-1: single-contact pair, a set mask bit is
  // its one contact); the count word follows the presence words in pmask
  int pair_cq[MAXP];
  // the same per 32-pair word of the contact mask, for the contact list walk (wave-uniform words:
  // scalar loads, where pair_cq[p] / pair_body[p] of a lane's own pair p are per-lane gathers):
  // multi-contact pairs (cq = pair_cqbase[w] + the multi-contact pairs below p in word w, since cq
  // is assigned in pair order), pairs touching an arm body, pairs touching a free body
  uint32_t pair_mw_multi[(MAXP + 31) / 32], pair_mw_arm[(MAXP + 31) / 32], pair_mw_free[(MAXP + 31) / 32];
  int pair_cqbase[(MAXP + 31) / 32];
  // k_collide's dispatch order (blockIdx.y -> pair): the pairs whose narrowphase is a convex-convex
  // solver or box-box clipping first (the launch's longest waves), plane pairs last
  int pair_order[MAXP];
  int ncq;
  int nslot;            // total contact slots (sum of per-pair capacities)
  int free_diag;        // every free body has ipos = 0 and iquat = 1: its 6x6 M block is diagonal
  // the contacts at qpos0, mj_resetData's pose: a soft reset (mj_checkPos/Vel/Acc) re-runs
  // mj_forward there, collision included, so k_substep hands a reset env these instead of the
  // collide output of the state it discarded.  Made once on the host with the kernels' own collide
  // code (soarm_cpu.hip cpu_qpos0_contacts): the pair-mask words then the count word, and per
  // contact its slot and 7-float record (dist, pos, normal), in pair order
  uint32_t c0_w[(MAXP + 31) / 32 + 1];
  int c0_n;
  int c0_slot[SIM_MAXCON];
  float c0_rec[SIM_MAXCON][7];

  // sites
  int site_bodyid[SIM_MAXSITE];
  float site_pos[SIM_MAXSITE][3];
  float site_quat[SIM_MAXSITE][4];  // unit (w, x, y, z): site frame in its body frame

  // actuators (actuator a drives dof a; checked on the host)
  int act_ctrllimited[MAXU], act_forcelimited[MAXU];
  float act_gear[MAXU], act_gain[MAXU], act_bias[MAXU][3];
  float act_ctrlrange[MAXU][2], act_forcerange[MAXU][2];

  // hull data (device pointers)
  const float4* hull_vert;   // xyz; w = bits (adjacency start << 8 | degree) of the vertex
  const int32_t* hull_adr;   // CSR offsets per global vertex (+1)
  const int32_t* hull_adj;   // local neighbour ids
  const uint16_t* hull_lut;  // per mesh geom: HULL_LUT_CELLS start vertices (cube-map of directions)
  int geom_lutadr[MAXG];     // first LUT entry of each mesh geom (-1: not a mesh)
  // hill-climbing records, 160 B per vertex (HULL_LUTREC uint4): [0] x, y, z (float bits),
  // degree | overflow offset << 8; [1] the first 8 neighbour ids (local, uint16, padded with
  // the vertex itself); [2..9] those neighbours' x, y, z and local id.  Neighbours past 8 live
  // in hull_ovf.  hull_lutrec holds, per LUT cell, a copy of its start vertex's record, so a
  // query whose start already holds the maximum (the usual case) finishes in one round trip
  // and each climbing step costs one more (the record moved to carries its neighbours'
  // coordinates: round 6, where a step had loaded the vertex and then its neighbours).
  const uint4* hull_rec;
  const uint4* hull_lutrec;
  const uint16_t* hull_ovf;
  // support-bound table (see HULL_SB_K): per mesh geom, the hull's support value at every grid
  // point of a cube map of directions, rounded up; geom_sbadr = first float of the geom's table
  const float* hull_sb;
  int geom_sbadr[MAXG];
};

// words per env of the collide output's pair mask: presence bits, then the count word
__host__ __device__ inline int pmask_words(const DModel& m) { return ((m.npair + 31) >> 5) + (m.ncq > 0 ? 1 : 0); }

// Support-point start table: a cube map of HULL_LUT_K x HULL_LUT_K cells per
// face; each cell holds the hull's argmax vertex for the cell-centre
// direction.  Hill climbing starts there, so a query usually ends at the start
// (verified from the neighbour coordinates the cell carries).  96 x 96: the
// collide kernel is latency-bound on support round trips, and a finer map
// (115 MB of cell records for the 13 arm hulls) lands the start on the answer
// more often: collide 0.287 (16) -> 0.251 (48) -> 0.231 (96) ms per env-step.
#ifndef SOARM_HULL_LUT_K
#define SOARM_HULL_LUT_K 96
#endif
constexpr int HULL_LUT_K = SOARM_HULL_LUT_K;
// uint4 per climbing record (hull_rec, hull_lutrec): the vertex's two record words, then its
// first 8 neighbours as (x, y, z, local id) -- a climbing step needs no second round trip
constexpr int HULL_LUTREC = 10;
constexpr int HULL_LUT_CELLS = 6 * HULL_LUT_K * HULL_LUT_K;

// Support-bound table: h(p) = max_v v.p at the (HULL_SB_K + 1)^2 grid points p = (+-1, u, v)
// (axis order as lut_dir) of every cube face.  The support function is convex and positively
// homogeneous, so for l = m q (q on a face, inside a grid cell's triangle with barycentric
// weights b_k >= 0 on corners p_k) h(l) = m h(q) <= m sum_k b_k h(p_k): an upper bound on the
// hull's support from 3 table values, no vertex data touched.  Slack ~ R (cell angle)^2.
constexpr int HULL_SB_K = 32;
constexpr int HULL_SB_FACE = (HULL_SB_K + 1) * (HULL_SB_K + 1);

// cube-map cell of a (not necessarily unit) direction; same mapping on host and device
inline __host__ __device__ int lut_cell(float l0, float l1, float l2) {
  const float a0 = fabsf(l0), a1 = fabsf(l1), a2 = fabsf(l2);
  int face;
  float u, v, m;
  if (a0 >= a1 && a0 >= a2) {
    face = l0 >= 0.f ? 0 : 1, m = a0, u = l1, v = l2;
  } else if (a1 >= a2) {
    face = l1 >= 0.f ? 2 : 3, m = a1, u = l0, v = l2;
  } else {
    face = l2 >= 0.f ? 4 : 5, m = a2, u = l0, v = l1;
  }
  if (!(m > 0.f)) return 0;
  const float s = 0.5f * HULL_LUT_K / m;
  int i = (int)((u + m) * s), j = (int)((v + m) * s);
  i = i < 0 ? 0 : (i >= HULL_LUT_K ? HULL_LUT_K - 1 : i);
  j = j < 0 ? 0 : (j >= HULL_LUT_K ? HULL_LUT_K - 1 : j);
  return (face * HULL_LUT_K + i) * HULL_LUT_K + j;
}

// centre direction of a cube-map cell (inverse of lut_cell)
inline void lut_dir(int cell, double d[3]) {
  const int face = cell / (HULL_LUT_K * HULL_LUT_K), i = (cell / HULL_LUT_K) % HULL_LUT_K, j = cell % HULL_LUT_K;
  const double u = -1.0 + (2.0 * i + 1.0) / HULL_LUT_K, v = -1.0 + (2.0 * j + 1.0) / HULL_LUT_K;
  const double sg = (face & 1) ? -1.0 : 1.0;
  switch (face >> 1) {
    case 0: d[0] = sg, d[1] = u, d[2] = v; break;
    case 1: d[0] = u, d[1] = sg, d[2] = v; break;
    default: d[0] = u, d[1] = v, d[2] = sg; break;
  }
}

}  // namespace soarm
