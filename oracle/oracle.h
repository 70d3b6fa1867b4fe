/*
 * oracle.h — float64 CPU restatement of the reference hot path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker; never linked into the product.
 *
 * What it restates:
 *   SOARM101Env.reset   SOARM101/SOARM101_Env.py:77-106  (mj_resetData + init + mj_forward)
 *   SOARM101Env.step    SOARM101/SOARM101_Env.py:108-142 (ctrl[:5] = a; 10 x mj_step; obs)
 *   mj_step  [ext: MuJoCo engine_forward.c / engine_core_smooth.c /
 *             engine_core_constraint.c / engine_solver.c]: kinematics, comPos,
 *             CRBA, LDL', comVel, passive, RNE, actuation, collision (MPR +
 *             box-box + plane), constraint rows (dof frictionloss, joint
 *             limits, pyramidal contacts), PGS dual solve, Euler with
 *             implicit damping.
 *
 * Parity status: the reference's own engine (MuJoCo) is absent from this
 * image and running reference code is denied, so this oracle
 * is "parity unpinned" against mj_step; it is pinned by the analytic
 * known-answer tests in tests/test_oracle.py and by the survey's FK anchors.
 */
#ifndef SOARM_ORACLE_H
#define SOARM_ORACLE_H

#include "../include/soarm_sim.h"

#define ORC_MAXEFC (2 * SIM_MAXDOF + 4 * SIM_MAXCON)
#define ORC_NSEED 32 /* hill-climbing seeds per hull: argmax vertex of 32 Fibonacci directions */

typedef struct orc_model {
  const sim_model_desc* m;
  const float* hull_vert;
  const int32_t* hull_adr;
  const int32_t* hull_adj;
  const int32_t* hull_seed; /* [ngeom][ORC_NSEED] hill-climb start candidates, or NULL */
  /* per-env domain randomisation (1,0/neg,1 = nominal) */
  double mass_scale;
  double friction; /* <0: use geom_friction */
  double damping_scale;
  int pgs_warm; /* experiment (tools/pgs_warm_exp.py): 0 = mj_solPGS's warm start from qacc_warmstart,
                   1 = the previous substep's forces for rows that persist (same dof / limit / pair
                   contact slot and edge), the implied force for new rows */
} orc_model;

typedef struct orc_contact {
  double dist;
  double pos[3];
  double frame[9]; /* normal (geom1->geom2), tangent1, tangent2 */
  double mu;       /* friction[0] after mixing */
  double friction[5];
  int geom1, geom2, pair;
} orc_contact;

typedef struct orc_data {
  /* state */
  double qpos[SIM_MAXQ], qvel[SIM_MAXDOF], ctrl[SIM_MAXU], qacc_warmstart[SIM_MAXDOF];
  double qacc[SIM_MAXDOF];
  int status;
  /* position-dependent */
  double xpos[SIM_MAXBODY][3], xquat[SIM_MAXBODY][4], xmat[SIM_MAXBODY][9];
  double xipos[SIM_MAXBODY][3], ximat[SIM_MAXBODY][9];
  double xanchor[SIM_MAXJNT][3], xaxis[SIM_MAXJNT][3];
  double geom_xpos[SIM_MAXGEOM][3], geom_xmat[SIM_MAXGEOM][9];
  double site_xpos[SIM_MAXSITE][3], site_xmat[SIM_MAXSITE][9];
  double subtree_com[SIM_MAXBODY][3];
  double cinert[SIM_MAXBODY][10], crb[SIM_MAXBODY][10], cdof[SIM_MAXDOF][6];
  double M[SIM_MAXDOF][SIM_MAXDOF];
  double L[SIM_MAXDOF][SIM_MAXDOF], Dinv[SIM_MAXDOF]; /* M = L D L', L unit lower */
  /* velocity-dependent */
  double cvel[SIM_MAXBODY][6], cdof_dot[SIM_MAXDOF][6];
  double qfrc_bias[SIM_MAXDOF], qfrc_passive[SIM_MAXDOF], qfrc_actuator[SIM_MAXDOF];
  double qfrc_smooth[SIM_MAXDOF], qacc_smooth[SIM_MAXDOF], qfrc_constraint[SIM_MAXDOF];
  double qfrc_applied[SIM_MAXDOF]; /* user input (mjData.qfrc_applied), zeroed by a reset */
  double actuator_force[SIM_MAXU];
  /* contacts & constraints */
  int ncon;
  orc_contact contact[SIM_MAXCON];
  int nefc;
  int efc_type[ORC_MAXEFC]; /* 0 friction dof, 1 limit, 2 contact pyramid edge */
  int efc_id[ORC_MAXEFC];
  double efc_J[ORC_MAXEFC][SIM_MAXDOF];
  double efc_pos[ORC_MAXEFC], efc_vel[ORC_MAXEFC], efc_aref[ORC_MAXEFC];
  double efc_R[ORC_MAXEFC], efc_diag[ORC_MAXEFC], efc_fl[ORC_MAXEFC];
  double efc_force[ORC_MAXEFC];
  int solver_iter;
  /* previous substep's rows (pgs_warm = 1): key per row and its force */
  int prev_n;
  int prev_key[ORC_MAXEFC];
  double prev_f[ORC_MAXEFC];
  /* flop counter (SURVEY.md §8d binding procedure) */
  double flops;
  double cflops; /* the collision share of flops */
} orc_data;

enum { ORC_EFC_FRICTION = 0, ORC_EFC_LIMIT = 1, ORC_EFC_CONTACT = 2 };

#ifdef __cplusplus
extern "C" {
#endif
/* single-env pipeline */
void orc_reset_data(const orc_model* om, orc_data* d);
void orc_kinematics(const orc_model* om, orc_data* d);
void orc_com_pos(const orc_model* om, orc_data* d);
void orc_crb(const orc_model* om, orc_data* d);
void orc_factor(const orc_model* om, orc_data* d);
void orc_solve_m(const orc_model* om, const orc_data* d, double* x, const double* b);
void orc_com_vel(const orc_model* om, orc_data* d);
void orc_rne(const orc_model* om, orc_data* d);
void orc_passive_actuation(const orc_model* om, orc_data* d);
void orc_collision(const orc_model* om, orc_data* d);
void orc_make_constraint(const orc_model* om, orc_data* d);
void orc_solve_pgs(const orc_model* om, orc_data* d);
/* MuJoCo's default primal Newton solver; tol <= 0 iterates to the exact optimum */
void orc_solve_newton(const orc_model* om, orc_data* d, double tol);
void orc_newton_stats(double* out /*[3] calls, iterations, line searches*/, int reset);
void orc_solver_stats(double* out /*[3] PGS calls, sweeps, rows*/, int reset);
void orc_forward(const orc_model* om, orc_data* d);
void orc_step(const orc_model* om, orc_data* d);
void orc_jac(const orc_model* om, const orc_data* d, const double p[3], int body, double* jacp,
             double* jacr);

/* collision primitives (oracle_collision.c) */
void orc_hull_seeds(const sim_model_desc* m, const float* hv, int32_t* seeds /*[ngeom][ORC_NSEED]*/);
int orc_hull_support(const orc_model* om, int g, const double l[3]);
int orc_hull_support_ex(const orc_model* om, int g, const double l[3], int use_graph);
int orc_hull_support_flat(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                          const int32_t* hadj, int g, const double* dirs, int n, int use_graph,
                          int32_t* out);
void orc_geom_frames(const sim_model_desc* m, const double* qpos, double* xpos, double* xmat);
void orc_collision_stats(double* out /*[8 + 2*SIM_MAXPAIR]*/, int reset);
int orc_collide_pair(const orc_model* om, const orc_data* d, int g1, int g2, orc_contact* out,
                     int maxout);

/* ---- flat ctypes entry points (batch; row-major per env) ---- */
void orc_batch_reset(const sim_model_desc* m, int n, double* qpos, double* qvel, double* warm,
                     double* ctrl, const double* init_qpos, const double* init_qvel,
                     const double* extra_qpos, double* obs);
/* params: NULL or [n][3] (mass_scale, friction(<0 nominal), damping_scale) */
void orc_batch_step(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                    const int32_t* hadj, int n, double* qpos, double* qvel, double* warm,
                    double* ctrl, const double* action, int nsub, double* obs, int32_t* status,
                    double* ncon_sum, const double* params, int nthreads, double* flops,
                    double* applied /* [n][nv] qfrc_applied in/out (zeroed by a soft reset) or NULL */);
/* qfrc_bias (mj_forward: comVel + RNE with qvel, flg_acc = 0) at n states: bias [n][nv] */
void orc_batch_bias(const sim_model_desc* m, int n, const double* qpos, const double* qvel,
                    const double* params, double* bias);
/* full diagnostic forward at a state: writes M[nv*nv], bias[nv], qacc[nv],
   ncon, contacts [ncon][14] = dist,pos3,frame9,geom1? (dist,pos,normal,g1,g2) */
int orc_debug_forward(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                      const int32_t* hadj, const double* qpos, const double* qvel,
                      const double* ctrl, const double* warm, double* M, double* bias,
                      double* qacc, double* contacts, double* site_xpos, double* geom_xpos,
                      double* efc_force, int* nefc);
int orc_collide_geoms(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                      const int32_t* hadj, const double* qpos, int g1, int g2, double* out,
                      int maxout);
void orc_ik_dls(const sim_model_desc* m, int n, const double* target, const double* target_quat, double* q,
                int32_t* ok, int32_t* iters, double tol, double rot_weight, double reg_thresh,
                double reg_strength, double max_update, double progress_thresh, int max_steps, int site,
                int ndof);
#ifdef __cplusplus
}
#endif

#endif
