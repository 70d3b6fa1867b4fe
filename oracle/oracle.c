/*
 * oracle.c — float64 restatement of mj_step for the SO-ARM101 hot path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Each function cites the MuJoCo
 * stage it restates [ext] and the reference call site that drives it.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MINVAL 1e-15
#define MAXVAL 1e10
#define MINIMP 0.0001
#define MAXIMP 0.9999

/* ------------------------------------------------------------ small algebra */
static void quat_mul(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void quat_normalize(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
    return;
  }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void quat2mat(double R[9], const double q[4]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z);
  R[1] = 2 * (x * y - w * z);
  R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);
  R[4] = 1 - 2 * (x * x + z * z);
  R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);
  R[7] = 2 * (y * z + w * x);
  R[8] = 1 - 2 * (x * x + y * y);
}
static void axisangle_quat(double q[4], const double ax[3], double a) {
  double s = sin(0.5 * a);
  q[0] = cos(0.5 * a);
  q[1] = ax[0] * s;
  q[2] = ax[1] * s;
  q[3] = ax[2] * s;
}
static void mat_vec(double r[3], const double R[9], const double v[3]) {
  double t[3] = {R[0] * v[0] + R[1] * v[1] + R[2] * v[2], R[3] * v[0] + R[4] * v[1] + R[5] * v[2],
                 R[6] * v[0] + R[7] * v[1] + R[8] * v[2]};
  memcpy(r, t, sizeof(t));
}
static void mat_mul(double r[9], const double A[9], const double B[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(r, t, sizeof(t));
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof(t));
}
static double dot3(const double a[3], const double b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static double dot6(const double a[6], const double b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* spatial algebra in MuJoCo's com-based convention: motion = [ang; lin] */
static void cross_motion(double r[6], const double v[6], const double m[6]) {
  double t[6];
  t[0] = -v[2] * m[1] + v[1] * m[2];
  t[1] = v[2] * m[0] - v[0] * m[2];
  t[2] = -v[1] * m[0] + v[0] * m[1];
  t[3] = -v[2] * m[4] + v[1] * m[5];
  t[4] = v[2] * m[3] - v[0] * m[5];
  t[5] = -v[1] * m[3] + v[0] * m[4];
  t[3] += -v[5] * m[1] + v[4] * m[2];
  t[4] += v[5] * m[0] - v[3] * m[2];
  t[5] += -v[4] * m[0] + v[3] * m[1];
  memcpy(r, t, sizeof(t));
}
static void cross_force(double r[6], const double v[6], const double f[6]) {
  double t[6];
  t[0] = -v[2] * f[1] + v[1] * f[2];
  t[1] = v[2] * f[0] - v[0] * f[2];
  t[2] = -v[1] * f[0] + v[0] * f[1];
  t[3] = -v[2] * f[4] + v[1] * f[5];
  t[4] = v[2] * f[3] - v[0] * f[5];
  t[5] = -v[1] * f[3] + v[0] * f[4];
  t[0] += -v[5] * f[4] + v[4] * f[5];
  t[1] += v[5] * f[3] - v[3] * f[5];
  t[2] += -v[4] * f[3] + v[3] * f[4];
  memcpy(r, t, sizeof(t));
}
/* cinert = [Ixx Iyy Izz Ixy Ixz Iyz, m*c (3), m] about the root's subtree com */
static void mul_inert_vec(double r[6], const double i[10], const double v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}

static int body_has_free(const sim_model_desc* m, int b) {
  return m->body_jntnum[b] > 0 && m->jnt_type[m->body_jntadr[b]] == SIM_JNT_FREE;
}

/* ----------------------------------------------------- mj_resetData [ext] */
void orc_reset_data(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  memset(d, 0, sizeof(*d));
  for (int i = 0; i < m->nq; i++) d->qpos[i] = m->qpos0[i];
}

/* ----------------------------------------------------- mj_kinematics [ext] */
void orc_kinematics(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  d->xquat[0][0] = 1;
  d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  memset(d->xpos[0], 0, sizeof(d->xpos[0]));
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parentid[b];
    double pos[3], quat[4];
    if (body_has_free(m, b)) {
      int j = m->body_jntadr[b], qa = m->jnt_qposadr[j];
      for (int k = 0; k < 3; k++) pos[k] = d->qpos[qa + k];
      for (int k = 0; k < 4; k++) quat[k] = d->qpos[qa + 3 + k];
      quat_normalize(quat);
      memcpy(d->xanchor[j], pos, sizeof(pos));
      d->xaxis[j][0] = d->xaxis[j][1] = 0;
      d->xaxis[j][2] = 1;
    } else {
      mat_vec(pos, d->xmat[p], m->body_pos[b]);
      for (int k = 0; k < 3; k++) pos[k] += d->xpos[p][k];
      quat_mul(quat, d->xquat[p], m->body_quat[b]);
      for (int jj = 0; jj < m->body_jntnum[b]; jj++) {
        int j = m->body_jntadr[b] + jj, qa = m->jnt_qposadr[j];
        double R[9];
        quat2mat(R, quat);
        mat_vec(d->xanchor[j], R, m->jnt_pos[j]);
        for (int k = 0; k < 3; k++) d->xanchor[j][k] += pos[k];
        mat_vec(d->xaxis[j], R, m->jnt_axis[j]);
        if (m->jnt_type[j] == SIM_JNT_HINGE) {
          double ql[4], t[3];
          axisangle_quat(ql, m->jnt_axis[j], d->qpos[qa] - m->qpos0[qa]);
          quat_mul(quat, quat, ql);
          quat2mat(R, quat);
          mat_vec(t, R, m->jnt_pos[j]);
          for (int k = 0; k < 3; k++) pos[k] = d->xanchor[j][k] - t[k];
        } else if (m->jnt_type[j] == SIM_JNT_SLIDE) {
          for (int k = 0; k < 3; k++) pos[k] += d->xaxis[j][k] * (d->qpos[qa] - m->qpos0[qa]);
        }
      }
    }
    quat_normalize(quat);
    memcpy(d->xpos[b], pos, sizeof(pos));
    memcpy(d->xquat[b], quat, sizeof(quat));
    quat2mat(d->xmat[b], quat);
  }
  for (int b = 0; b < m->nbody; b++) {
    double t[3], Ri[9];
    mat_vec(t, d->xmat[b], m->body_ipos[b]);
    for (int k = 0; k < 3; k++) d->xipos[b][k] = d->xpos[b][k] + t[k];
    quat2mat(Ri, m->body_iquat[b]);
    mat_mul(d->ximat[b], d->xmat[b], Ri);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double t[3], Rg[9];
    mat_vec(t, d->xmat[b], m->geom_pos[g]);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = d->xpos[b][k] + t[k];
    quat2mat(Rg, m->geom_quat[g]);
    mat_mul(d->geom_xmat[g], d->xmat[b], Rg);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double t[3], Rs[9];
    mat_vec(t, d->xmat[b], m->site_pos[s]);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + t[k];
    quat2mat(Rs, m->site_quat[s]);
    mat_mul(d->site_xmat[s], d->xmat[b], Rs);
  }
  d->flops += 120.0 * (m->nbody - 1) + 45.0 * m->ngeom + 45.0 * m->nsite;
}

/* -------------------------------------------------------- mj_comPos [ext] */
void orc_com_pos(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  double mass[SIM_MAXBODY];
  for (int b = 0; b < m->nbody; b++) {
    mass[b] = m->body_mass[b] * om->mass_scale;
    for (int k = 0; k < 3; k++) d->subtree_com[b][k] = mass[b] * d->xipos[b][k];
  }
  double smass[SIM_MAXBODY];
  memcpy(smass, mass, sizeof(smass));
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p == b) continue;
    for (int k = 0; k < 3; k++) d->subtree_com[p][k] += d->subtree_com[b][k];
    smass[p] += smass[b];
  }
  for (int b = 0; b < m->nbody; b++) {
    if (smass[b] < MINVAL)
      memcpy(d->subtree_com[b], d->xipos[b], sizeof(d->subtree_com[b]));
    else
      for (int k = 0; k < 3; k++) d->subtree_com[b][k] /= smass[b];
  }
  for (int b = 1; b < m->nbody; b++) {
    const double* ref = d->subtree_com[m->body_rootid[b]];
    const double* R = d->ximat[b];
    double in[3] = {m->body_inertia[b][0] * om->mass_scale, m->body_inertia[b][1] * om->mass_scale,
                    m->body_inertia[b][2] * om->mass_scale};
    double I[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        I[3 * i + j] = R[3 * i] * in[0] * R[3 * j] + R[3 * i + 1] * in[1] * R[3 * j + 1] +
                       R[3 * i + 2] * in[2] * R[3 * j + 2];
    double c[3] = {d->xipos[b][0] - ref[0], d->xipos[b][1] - ref[1], d->xipos[b][2] - ref[2]};
    double cc = dot3(c, c);
    double* ci = d->cinert[b];
    ci[0] = I[0] + mass[b] * (cc - c[0] * c[0]);
    ci[1] = I[4] + mass[b] * (cc - c[1] * c[1]);
    ci[2] = I[8] + mass[b] * (cc - c[2] * c[2]);
    ci[3] = I[1] - mass[b] * c[0] * c[1];
    ci[4] = I[2] - mass[b] * c[0] * c[2];
    ci[5] = I[5] - mass[b] * c[1] * c[2];
    ci[6] = mass[b] * c[0];
    ci[7] = mass[b] * c[1];
    ci[8] = mass[b] * c[2];
    ci[9] = mass[b];
  }
  /* cdof */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    const double* ref = d->subtree_com[m->body_rootid[b]];
    double off[3] = {ref[0] - d->xanchor[j][0], ref[1] - d->xanchor[j][1],
                     ref[2] - d->xanchor[j][2]};
    if (m->jnt_type[j] == SIM_JNT_HINGE) {
      double* c = d->cdof[da];
      memcpy(c, d->xaxis[j], 3 * sizeof(double));
      cross3(c + 3, d->xaxis[j], off);
    } else if (m->jnt_type[j] == SIM_JNT_SLIDE) {
      double* c = d->cdof[da];
      c[0] = c[1] = c[2] = 0;
      memcpy(c + 3, d->xaxis[j], 3 * sizeof(double));
    } else if (m->jnt_type[j] == SIM_JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        double* c = d->cdof[da + k];
        memset(c, 0, 6 * sizeof(double));
        c[3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        double* c = d->cdof[da + 3 + k];
        double ax[3] = {d->xmat[b][k], d->xmat[b][3 + k], d->xmat[b][6 + k]};
        memcpy(c, ax, sizeof(ax));
        cross3(c + 3, ax, off);
      }
    }
  }
  d->flops += 70.0 * (m->nbody - 1) + 9.0 * m->nv;
}

/* ------------------------------------------------- mj_crb + mj_makeM [ext] */
void orc_crb(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  memcpy(d->crb, d->cinert, sizeof(d->crb));
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[p][k] += d->crb[b][k];
  }
  memset(d->M, 0, sizeof(d->M));
  for (int i = 0; i < m->nv; i++) {
    double buf[6];
    mul_inert_vec(buf, d->crb[m->dof_bodyid[i]], d->cdof[i]);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      d->M[i][j] = dot6(d->cdof[j], buf);
      d->M[j][i] = d->M[i][j];
      d->flops += 11;
    }
    d->M[i][i] += m->dof_armature[i];
    d->flops += 30;
  }
}

/* dense LDL' of M (restates mj_factorM's result; MuJoCo uses the tree-sparse
   L'DL form, which yields the same solves up to rounding) */
static void ldl(int n, double A[SIM_MAXDOF][SIM_MAXDOF], double L[SIM_MAXDOF][SIM_MAXDOF],
                double* Dinv) {
  double D[SIM_MAXDOF];
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < i; j++) {
      double s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k] * D[k];
      L[i][j] = s / D[j];
    }
    double s = A[i][i];
    for (int k = 0; k < i; k++) s -= L[i][k] * L[i][k] * D[k];
    D[i] = s;
    Dinv[i] = 1.0 / s;
    L[i][i] = 1;
    for (int j = i + 1; j < n; j++) L[i][j] = 0;
  }
}
static void ldl_solve(int n, const double L[SIM_MAXDOF][SIM_MAXDOF], const double* Dinv, double* x,
                      const double* b) {
  double y[SIM_MAXDOF];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s;
  }
  for (int i = 0; i < n; i++) y[i] *= Dinv[i];
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k][i] * x[k];
    x[i] = s;
  }
}
void orc_factor(const orc_model* om, orc_data* d) {
  ldl(om->m->nv, d->M, d->L, d->Dinv);
  d->flops += (double)om->m->nv * om->m->nv * om->m->nv / 3.0;
}
void orc_solve_m(const orc_model* om, const orc_data* d, double* x, const double* b) {
  ldl_solve(om->m->nv, d->L, d->Dinv, x, b);
}

/* -------------------------------------------------------- mj_comVel [ext] */
void orc_com_vel(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  memset(d->cvel[0], 0, sizeof(d->cvel[0]));
  for (int b = 1; b < m->nbody; b++) {
    double cvel[6];
    memcpy(cvel, d->cvel[m->body_parentid[b]], sizeof(cvel));
    for (int jj = 0; jj < m->body_jntnum[b]; jj++) {
      int j = m->body_jntadr[b] + jj, da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == SIM_JNT_FREE) {
        for (int k = 0; k < 3; k++) {
          memset(d->cdof_dot[da + k], 0, 6 * sizeof(double));
          for (int e = 0; e < 6; e++) cvel[e] += d->cdof[da + k][e] * d->qvel[da + k];
        }
        for (int k = 3; k < 6; k++) cross_motion(d->cdof_dot[da + k], cvel, d->cdof[da + k]);
        for (int k = 3; k < 6; k++)
          for (int e = 0; e < 6; e++) cvel[e] += d->cdof[da + k][e] * d->qvel[da + k];
      } else {
        cross_motion(d->cdof_dot[da], cvel, d->cdof[da]);
        for (int e = 0; e < 6; e++) cvel[e] += d->cdof[da][e] * d->qvel[da];
      }
    }
    memcpy(d->cvel[b], cvel, sizeof(cvel));
  }
  d->flops += 30.0 * m->nv;
}

/* --------------------------------------------------- mj_rne(flg_acc=0) [ext] */
void orc_rne(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  double cacc[SIM_MAXBODY][6], cfrc[SIM_MAXBODY][6];
  memset(cacc[0], 0, sizeof(cacc[0]));
  for (int k = 0; k < 3; k++) cacc[0][3 + k] = -m->gravity[k];
  for (int b = 1; b < m->nbody; b++) {
    memcpy(cacc[b], cacc[m->body_parentid[b]], sizeof(cacc[b]));
    int da = m->body_dofadr[b];
    for (int k = 0; k < m->body_dofnum[b]; k++)
      for (int e = 0; e < 6; e++) cacc[b][e] += d->cdof_dot[da + k][e] * d->qvel[da + k];
    double t1[6], t2[6], t3[6];
    mul_inert_vec(t1, d->cinert[b], cacc[b]);
    mul_inert_vec(t2, d->cinert[b], d->cvel[b]);
    cross_force(t3, d->cvel[b], t2);
    for (int e = 0; e < 6; e++) cfrc[b][e] = t1[e] + t3[e];
  }
  memset(cfrc[0], 0, sizeof(cfrc[0]));
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p > 0)
      for (int e = 0; e < 6; e++) cfrc[p][e] += cfrc[b][e];
  }
  for (int i = 0; i < m->nv; i++) d->qfrc_bias[i] = dot6(d->cdof[i], cfrc[m->dof_bodyid[i]]);
  d->flops += 100.0 * (m->nbody - 1) + 12.0 * m->nv;
}

/* ------------------------------------- mj_passive + mj_fwdActuation [ext] */
void orc_passive_actuation(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  for (int i = 0; i < m->nv; i++) {
    d->qfrc_passive[i] = -m->dof_damping[i] * om->damping_scale * d->qvel[i];
    d->qfrc_actuator[i] = 0;
  }
  for (int a = 0; a < m->nu; a++) {
    int j = m->actuator_trnid[a], da = m->jnt_dofadr[j], qa = m->jnt_qposadr[j];
    double g = m->actuator_gear[a];
    double ctrl = d->ctrl[a];
    if (m->actuator_ctrllimited[a]) {
      if (ctrl < m->actuator_ctrlrange[a][0]) ctrl = m->actuator_ctrlrange[a][0];
      if (ctrl > m->actuator_ctrlrange[a][1]) ctrl = m->actuator_ctrlrange[a][1];
    }
    double len = g * d->qpos[qa], vel = g * d->qvel[da];
    double f = m->actuator_gainprm[a] * ctrl + m->actuator_biasprm[a][0] +
               m->actuator_biasprm[a][1] * len + m->actuator_biasprm[a][2] * vel;
    if (m->actuator_forcelimited[a]) {
      if (f < m->actuator_forcerange[a][0]) f = m->actuator_forcerange[a][0];
      if (f > m->actuator_forcerange[a][1]) f = m->actuator_forcerange[a][1];
    }
    d->actuator_force[a] = f;
    d->qfrc_actuator[da] += g * f;
  }
  d->flops += 2.0 * m->nv + 10.0 * m->nu;
}

/* --------------------------------------------------------- Jacobians [ext mj_jac] */
void orc_jac(const orc_model* om, const orc_data* d, const double p[3], int body, double* jacp,
             double* jacr) {
  const sim_model_desc* m = om->m;
  int nv = m->nv;
  if (jacp) memset(jacp, 0, 3 * nv * sizeof(double));
  if (jacr) memset(jacr, 0, 3 * nv * sizeof(double));
  if (body <= 0) return;
  const double* ref = d->subtree_com[m->body_rootid[body]];
  double off[3] = {p[0] - ref[0], p[1] - ref[1], p[2] - ref[2]};
  /* walk the dof chain up from the body's last dof */
  int b = body;
  while (b > 0 && m->body_dofnum[b] == 0) b = m->body_parentid[b];
  if (b <= 0) return;
  for (int i = m->body_dofadr[b] + m->body_dofnum[b] - 1; i >= 0; i = m->dof_parentid[i]) {
    const double* c = d->cdof[i];
    double t[3];
    cross3(t, c, off);
    for (int k = 0; k < 3; k++) {
      if (jacp) jacp[k * nv + i] = c[3 + k] + t[k];
      if (jacr) jacr[k * nv + i] = c[k];
    }
  }
}

/* ------------------------------------------ constraint rows [ext mj_makeConstraint,
   mj_diagApprox, mj_makeImpedance] */
static void impedance(const double* solimp, double pos, double margin, double* imp) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], pw = solimp[4];
  if (dmin < MINIMP) dmin = MINIMP;
  if (dmin > MAXIMP) dmin = MAXIMP;
  if (dmax < MINIMP) dmax = MINIMP;
  if (dmax > MAXIMP) dmax = MAXIMP;
  if (dmin == dmax || width <= MINVAL) {
    *imp = 0.5 * (dmin + dmax);
    return;
  }
  double x = fabs((pos - margin) / width);
  if (x >= 1) {
    *imp = dmax;
    return;
  }
  if (x <= 0) {
    *imp = dmin;
    return;
  }
  double y;
  if (pw == 1)
    y = x;
  else if (x <= mid)
    y = pow(x, pw) / pow(mid, pw - 1);
  else
    y = 1 - pow(1 - x, pw) / pow(1 - mid, pw - 1);
  *imp = dmin + y * (dmax - dmin);
}

static void add_row_params(const orc_model* om, orc_data* d, int r, const double* solref,
                           const double* solimp, double margin) {
  const sim_model_desc* m = om->m;
  double imp;
  impedance(solimp, d->efc_pos[r], margin, &imp);
  double R = (1 - imp) * d->efc_diag[r] / imp;
  d->efc_R[r] = R < MINVAL ? MINVAL : R;
  double dmax = solimp[1];
  if (dmax < MINIMP) dmax = MINIMP;
  if (dmax > MAXIMP) dmax = MAXIMP;
  double K, B;
  if (solref[0] > 0) {
    double tc = solref[0] > 2 * m->timestep ? solref[0] : 2 * m->timestep; /* refsafe */
    double dr = solref[1];
    K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
    B = 2.0 / (dmax * tc);
  } else {
    K = -solref[0] / (dmax * dmax);
    B = -solref[1] / dmax;
  }
  d->efc_aref[r] = -B * d->efc_vel[r] - K * imp * (d->efc_pos[r] - margin);
}

void orc_make_constraint(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  int nv = m->nv, r = 0;
  /* dof frictionloss rows */
  for (int i = 0; i < nv; i++) {
    if (m->dof_frictionloss[i] <= 0) continue;
    memset(d->efc_J[r], 0, sizeof(d->efc_J[r]));
    d->efc_J[r][i] = 1;
    d->efc_type[r] = ORC_EFC_FRICTION;
    d->efc_id[r] = i;
    d->efc_pos[r] = 0;
    d->efc_fl[r] = m->dof_frictionloss[i];
    d->efc_diag[r] = m->dof_invweight0[i];
    d->efc_vel[r] = d->qvel[i];
    add_row_params(om, d, r, m->dof_solref[i], m->dof_solimp[i], 0);
    r++;
  }
  /* joint limit rows */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j]) continue;
    if (m->jnt_type[j] != SIM_JNT_HINGE && m->jnt_type[j] != SIM_JNT_SLIDE) continue;
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side < 0 ? d->qpos[qa] - m->jnt_range[j][0] : m->jnt_range[j][1] - d->qpos[qa];
      if (dist >= m->jnt_margin[j]) continue;
      memset(d->efc_J[r], 0, sizeof(d->efc_J[r]));
      d->efc_J[r][da] = -side;
      d->efc_type[r] = ORC_EFC_LIMIT;
      d->efc_id[r] = j;
      d->efc_pos[r] = dist;
      d->efc_fl[r] = 0;
      d->efc_diag[r] = m->dof_invweight0[da];
      d->efc_vel[r] = -side * d->qvel[da];
      add_row_params(om, d, r, m->jnt_solref[j], m->jnt_solimp[j], m->jnt_margin[j]);
      r++;
    }
  }
  /* contacts: 4 pyramid edges each (condim 3) */
  for (int c = 0; c < d->ncon; c++) {
    const orc_contact* con = &d->contact[c];
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    double j1[3 * SIM_MAXDOF], j2[3 * SIM_MAXDOF], jd[3][SIM_MAXDOF];
    orc_jac(om, d, con->pos, b1, j1, NULL);
    orc_jac(om, d, con->pos, b2, j2, NULL);
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < nv; i++) {
        double diff[3] = {j2[0 * nv + i] - j1[0 * nv + i], j2[1 * nv + i] - j1[1 * nv + i],
                          j2[2 * nv + i] - j1[2 * nv + i]};
        jd[k][i] = dot3(con->frame + 3 * k, diff);
      }
    double tran = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    /* geom solref/solimp mixing: equal solmix -> average */
    double solref[2], solimp[5];
    for (int k = 0; k < 2; k++)
      solref[k] = 0.5 * (m->geom_solref[con->geom1][k] + m->geom_solref[con->geom2][k]);
    for (int k = 0; k < 5; k++)
      solimp[k] = 0.5 * (m->geom_solimp[con->geom1][k] + m->geom_solimp[con->geom2][k]);
    double margin = m->geom_margin[con->geom1] > m->geom_margin[con->geom2]
                        ? m->geom_margin[con->geom1]
                        : m->geom_margin[con->geom2];
    int r0 = r;
    for (int e = 0; e < 4; e++) {
      int k = 1 + e / 2;
      double sgn = (e & 1) ? -1.0 : 1.0;
      double mu = con->friction[e / 2];
      for (int i = 0; i < nv; i++) d->efc_J[r][i] = jd[0][i] + sgn * mu * jd[k][i];
      for (int i = nv; i < SIM_MAXDOF; i++) d->efc_J[r][i] = 0;
      d->efc_type[r] = ORC_EFC_CONTACT;
      d->efc_id[r] = c;
      d->efc_pos[r] = con->dist;
      d->efc_fl[r] = 0;
      d->efc_diag[r] = tran + mu * mu * tran;
      double v = 0;
      for (int i = 0; i < nv; i++) v += d->efc_J[r][i] * d->qvel[i];
      d->efc_vel[r] = v;
      add_row_params(om, d, r, solref, solimp, margin);
      r++;
    }
    double Rpy = 2 * con->mu * con->mu * d->efc_R[r0] / m->impratio;
    for (int e = 0; e < 4; e++) d->efc_R[r0 + e] = Rpy;
    d->flops += 60.0 * nv + 200;
  }
  d->nefc = r;
  d->flops += 30.0 * r;
}

/* solver statistics (single-threaded use): calls, sweeps, rows */
static double orc_stats[3];
void orc_solver_stats(double* out, int reset) {
  for (int k = 0; k < 3; k++) {
    out[k] = orc_stats[k];
    if (reset) orc_stats[k] = 0;
  }
}

/* stopping-test scale of MuJoCo's solvers: 1 / (mjStatistic.meaninertia * max(1, nv)) */
static double solver_scale(const sim_model_desc* m) {
  const double mi = m->meaninertia > MINVAL ? m->meaninertia : 1.0;
  return 1.0 / (mi * (m->nv > 1 ? m->nv : 1));
}

/* identity of a constraint row across substeps (experiment harness, pgs_warm = 1) */
static int row_key(const orc_data* d, int r) {
  const int id = d->efc_id[r];
  if (d->efc_type[r] == ORC_EFC_FRICTION) return 1000000 + id;
  if (d->efc_type[r] == ORC_EFC_LIMIT) {
    double s = 0;
    for (int i = 0; i < SIM_MAXDOF; i++) s += d->efc_J[r][i];
    return 2000000 + 2 * id + (s > 0 ? 0 : 1);
  }
  int k = 0; /* k-th contact of its pair */
  for (int c = 0; c < id; c++) k += d->contact[c].pair == d->contact[id].pair;
  int e = 0; /* edge within the contact */
  for (int q = r - 1; q >= 0 && d->efc_type[q] == ORC_EFC_CONTACT && d->efc_id[q] == id; q--) e++;
  return d->contact[id].pair * 64 + k * 4 + e;
}

/* ------------------------------------------------ PGS dual solver [ext mj_solPGS] */
static double project(int type, double f, double fl) {
  if (type == ORC_EFC_FRICTION) return f < -fl ? -fl : (f > fl ? fl : f);
  return f < 0 ? 0 : f;
}

void orc_solve_pgs(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  int nv = m->nv, ne = d->nefc;
  double W[ORC_MAXEFC][SIM_MAXDOF]; /* M^-1 J_i' */
  double ARd[ORC_MAXEFC];
  for (int r = 0; r < ne; r++) {
    orc_solve_m(om, d, W[r], d->efc_J[r]);
    double s = 0;
    for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * W[r][i];
    ARd[r] = s + d->efc_R[r];
  }
  d->flops += ne * (2.0 * nv * nv + 2.0 * nv);
  /* warm start from qacc_warmstart through the primal's implied forces */
  double f[ORC_MAXEFC], v[SIM_MAXDOF];
  for (int r = 0; r < ne; r++) {
    double jar = -d->efc_aref[r];
    for (int i = 0; i < nv; i++) jar += d->efc_J[r][i] * d->qacc_warmstart[i];
    double D = 1.0 / d->efc_R[r];
    if (d->efc_type[r] == ORC_EFC_FRICTION) {
      double fl = d->efc_fl[r];
      if (jar <= -fl * d->efc_R[r])
        f[r] = fl;
      else if (jar >= fl * d->efc_R[r])
        f[r] = -fl;
      else
        f[r] = -D * jar;
    } else {
      f[r] = jar < 0 ? -D * jar : 0;
    }
  }
  if (om->pgs_warm == 1) /* experiment: persisting rows restart from their previous force */
    for (int r = 0; r < ne; r++) {
      const int key = row_key(d, r);
      for (int q = 0; q < d->prev_n; q++)
        if (d->prev_key[q] == key) {
          f[r] = project(d->efc_type[r], d->prev_f[q], d->efc_fl[r]);
          break;
        }
    }
  /* keep the warm start only if its dual cost beats f = 0 */
  memcpy(v, d->qacc_smooth, nv * sizeof(double));
  for (int r = 0; r < ne; r++)
    for (int i = 0; i < nv; i++) v[i] += W[r][i] * f[r];
  double cost = 0;
  for (int r = 0; r < ne; r++) {
    double Jv = 0;
    for (int i = 0; i < nv; i++) Jv += d->efc_J[r][i] * v[i];
    /* (AR f + b)_r = J_r v - aref_r + R_r f_r ; cost = 0.5 f'(AR f + b) + 0.5 f'b */
    double Jqs = 0;
    for (int i = 0; i < nv; i++) Jqs += d->efc_J[r][i] * d->qacc_smooth[i];
    double b = Jqs - d->efc_aref[r];
    cost += 0.5 * f[r] * (Jv - d->efc_aref[r] + d->efc_R[r] * f[r]) + 0.5 * f[r] * b;
  }
  if (cost > 0) {
    for (int r = 0; r < ne; r++) f[r] = 0;
    memcpy(v, d->qacc_smooth, nv * sizeof(double));
  }
  /* Gauss-Seidel sweeps with projection; mj_solPGS stops when the sweep's cost improvement,
     scaled by 1 / (meaninertia * max(1, nv)) (a model constant, M at qpos0), is below tolerance */
  const double scale = solver_scale(m);
  int it;
  for (it = 0; it < m->iterations; it++) {
    double improvement = 0;
    for (int r = 0; r < ne; r++) {
      double res = -d->efc_aref[r] + d->efc_R[r] * f[r];
      for (int i = 0; i < nv; i++) res += d->efc_J[r][i] * v[i];
      double fn = project(d->efc_type[r], f[r] - res / ARd[r], d->efc_fl[r]);
      double df = fn - f[r];
      if (df != 0) {
        for (int i = 0; i < nv; i++) v[i] += W[r][i] * df;
        f[r] = fn;
        improvement -= df * res + 0.5 * ARd[r] * df * df;
      }
    }
    d->flops += ne * 4.0 * nv;
    if (improvement * scale < m->tolerance) {
      it++;
      break;
    }
  }
  d->solver_iter = it;
  if (om->pgs_warm == 1) {
    d->prev_n = ne;
    for (int r = 0; r < ne; r++) d->prev_key[r] = row_key(d, r), d->prev_f[r] = f[r];
  }
  orc_stats[0] += 1;
  orc_stats[1] += it;
  orc_stats[2] += ne;
  memcpy(d->qacc, v, nv * sizeof(double));
  memcpy(d->efc_force, f, ne * sizeof(double));
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int r = 0; r < ne; r++) s += d->efc_J[r][i] * f[r];
    d->qfrc_constraint[i] = s;
  }
}

/* ---------------------------------------- primal Newton solver [ext mj_solNewton]
 * The reference scene has no <option> (SOARM101/SO101/scene_with_table_v.xml:1-32), so the
 * reference's mj_step (SOARM101_Env.py:131-132) solves the constraint problem with MuJoCo's
 * default solver: primal Newton, iterations 100, tolerance 1e-8.  Restated from MuJoCo's
 * published algorithm (engine_solver.c / mj_constraintUpdate):
 *   minimise  c(a) = 1/2 (a - a0)' M (a - a0) + sum_r s_r(J_r a - aref_r),  a0 = qacc_smooth,
 *   s_r(x) = x^2 / (2 R_r)                          limits, pyramid edges: x < 0 (else 0)
 *          = Huber: x^2/(2R) for |x| < R fl, fl |x| - R fl^2 / 2 beyond   frictionloss rows
 *   force f_r = -s_r'(x);  gradient g = M (a - a0) - J' f;  Hessian H = M + J_q' D J_q over the
 *   rows in their quadratic zone (D = 1/R);  direction p = -H^-1 g;  line search: exact
 *   minimiser of the convex piecewise-quadratic c(a + alpha p) (MuJoCo's 1-D Newton search
 *   with gtol = tolerance * ls_tolerance(0.01) * |p| * meaninertia * nv finds the same point
 *   to within that tolerance);  stop when scale * (c_old - c) < tol or scale * |g| < tol,
 *   scale = 1 / (meaninertia * max(1, nv)).
 *   Warm start: qacc_warmstart if its cost beats qacc_smooth's (mj_fwdConstraint).
 * The problem is strictly convex (R > 0), so the optimum is unique: with tol <= 0 the loop
 * runs until the step stops changing the cost (the exact optimum to double precision) — the
 * reference point the PGS kernels are measured against.
 * ------------------------------------------------------------------------------- */
static double row_force(const orc_data* d, int r, double x, int* quad) {
  const double R = d->efc_R[r];
  if (d->efc_type[r] == ORC_EFC_FRICTION) {
    const double fl = d->efc_fl[r];
    if (x <= -R * fl) {
      *quad = 0;
      return fl;
    }
    if (x >= R * fl) {
      *quad = 0;
      return -fl;
    }
    *quad = 1;
    return -x / R;
  }
  *quad = x < 0;
  return x < 0 ? -x / R : 0.0;
}
static double row_cost(const orc_data* d, int r, double x) {
  const double R = d->efc_R[r];
  if (d->efc_type[r] == ORC_EFC_FRICTION) {
    const double fl = d->efc_fl[r];
    if (x <= -R * fl) return -fl * x - 0.5 * R * fl * fl;
    if (x >= R * fl) return fl * x - 0.5 * R * fl * fl;
    return 0.5 * x * x / R;
  }
  return x < 0 ? 0.5 * x * x / R : 0.0;
}
/* c(a); jar [nefc] = J a - aref */
static double primal_cost(const sim_model_desc* m, const orc_data* d, const double* a, double* jar) {
  const int nv = m->nv;
  double da[SIM_MAXDOF], c = 0;
  for (int i = 0; i < nv; i++) da[i] = a[i] - d->qacc_smooth[i];
  for (int i = 0; i < nv; i++)
    for (int k = 0; k < nv; k++) c += 0.5 * da[i] * d->M[i][k] * da[k];
  for (int r = 0; r < d->nefc; r++) {
    double x = -d->efc_aref[r];
    for (int i = 0; i < nv; i++) x += d->efc_J[r][i] * a[i];
    jar[r] = x;
    c += row_cost(d, r, x);
  }
  return c;
}
/* derivative of c(a + alpha p) at alpha: g0 + alpha pMp - sum_r f_r(jar_r + alpha jv_r) jv_r */
static double ls_deriv(const orc_data* d, double g0, double pMp, const double* jar, const double* jv,
                       double alpha, double* curv) {
  double g = g0 + alpha * pMp, h = pMp;
  for (int r = 0; r < d->nefc; r++) {
    int q;
    const double f = row_force(d, r, jar[r] + alpha * jv[r], &q);
    g -= f * jv[r];
    if (q) h += jv[r] * jv[r] / d->efc_R[r];
  }
  if (curv) *curv = h;
  return g;
}
static int cmp_double(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}
/* exact minimiser of the convex piecewise quadratic c(a + alpha p), alpha >= 0 */
static double line_search(const orc_data* d, double g0, double pMp, const double* jar, const double* jv) {
  if (ls_deriv(d, g0, pMp, jar, jv, 0.0, NULL) >= 0) return 0.0;
  double bp[2 * ORC_MAXEFC];
  int nb = 0;
  for (int r = 0; r < d->nefc; r++) {
    if (jv[r] == 0) continue;
    const double R = d->efc_R[r];
    double xs[2];
    int nx = 0;
    if (d->efc_type[r] == ORC_EFC_FRICTION) {
      xs[nx++] = -R * d->efc_fl[r];
      xs[nx++] = R * d->efc_fl[r];
    } else {
      xs[nx++] = 0.0;
    }
    for (int k = 0; k < nx; k++) {
      const double al = (xs[k] - jar[r]) / jv[r];
      if (al > 0) bp[nb++] = al;
    }
  }
  qsort(bp, nb, sizeof(double), cmp_double);
  double lo = 0.0, glo = ls_deriv(d, g0, pMp, jar, jv, 0.0, NULL);
  for (int k = 0; k < nb; k++) {
    const double hi = bp[k];
    if (hi <= lo) continue;
    const double ghi = ls_deriv(d, g0, pMp, jar, jv, hi, NULL);
    if (ghi >= 0) /* the derivative is linear on [lo, hi]: its root */
      return lo + (hi - lo) * (-glo) / (ghi - glo);
    lo = hi, glo = ghi;
  }
  double h;
  ls_deriv(d, g0, pMp, jar, jv, lo + 1.0, &h); /* curvature of the last (unbounded) piece */
  return lo - glo / h;
}
/* dense Cholesky solve (H SPD), n <= SIM_MAXDOF */
static int chol_solve_n(int n, double A[SIM_MAXDOF][SIM_MAXDOF], double* x, const double* b) {
  double L[SIM_MAXDOF][SIM_MAXDOF];
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      double s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (s <= 0) return -1;
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  double y[SIM_MAXDOF];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return 0;
}

static double newton_stats[3]; /* calls, iterations, line-search steps taken */
void orc_newton_stats(double* out, int reset) {
  for (int k = 0; k < 3; k++) {
    out[k] = newton_stats[k];
    if (reset) newton_stats[k] = 0;
  }
}

void orc_solve_newton(const orc_model* om, orc_data* d, double tol) {
  const sim_model_desc* m = om->m;
  const int nv = m->nv, ne = d->nefc;
  const double scale = solver_scale(m);
  double a[SIM_MAXDOF], jar[ORC_MAXEFC], jv[ORC_MAXEFC];
  /* warm start (mj_fwdConstraint): qacc_warmstart unless qacc_smooth costs less */
  double cw = primal_cost(m, d, d->qacc_warmstart, jar);
  double cs = primal_cost(m, d, d->qacc_smooth, jar);
  memcpy(a, cw < cs ? d->qacc_warmstart : d->qacc_smooth, nv * sizeof(double));
  double cost = primal_cost(m, d, a, jar);
  int it = 0;
  for (; it < m->iterations; it++) {
    /* gradient and Hessian at a */
    double g[SIM_MAXDOF], H[SIM_MAXDOF][SIM_MAXDOF], da[SIM_MAXDOF];
    for (int i = 0; i < nv; i++) da[i] = a[i] - d->qacc_smooth[i];
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int k = 0; k < nv; k++) {
        s += d->M[i][k] * da[k];
        H[i][k] = d->M[i][k];
      }
      g[i] = s;
    }
    for (int r = 0; r < ne; r++) {
      int q;
      const double f = row_force(d, r, jar[r], &q);
      for (int i = 0; i < nv; i++) g[i] -= d->efc_J[r][i] * f;
      if (q) {
        const double D = 1.0 / d->efc_R[r];
        for (int i = 0; i < nv; i++)
          for (int k = 0; k < nv; k++) H[i][k] += D * d->efc_J[r][i] * d->efc_J[r][k];
      }
    }
    double gn = 0;
    for (int i = 0; i < nv; i++) gn += g[i] * g[i];
    if (tol > 0 && scale * sqrt(gn) < tol) break;
    if (gn == 0) break;
    double p[SIM_MAXDOF], mg[SIM_MAXDOF];
    for (int i = 0; i < nv; i++) mg[i] = -g[i];
    if (chol_solve_n(nv, H, p, mg)) break;
    /* exact line search along p */
    double Mp[SIM_MAXDOF], pMp = 0, g0 = 0;
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int k = 0; k < nv; k++) s += d->M[i][k] * p[k];
      Mp[i] = s;
    }
    for (int i = 0; i < nv; i++) pMp += p[i] * Mp[i], g0 += da[i] * Mp[i];
    for (int r = 0; r < ne; r++) {
      double s = 0;
      for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * p[i];
      jv[r] = s;
    }
    const double alpha = line_search(d, g0, pMp, jar, jv);
    if (!(alpha > 0)) break;
    double an[SIM_MAXDOF], jn[ORC_MAXEFC];
    for (int i = 0; i < nv; i++) an[i] = a[i] + alpha * p[i];
    const double cn = primal_cost(m, d, an, jn);
    newton_stats[2] += 1;
    if (!(cn <= cost)) break; /* rounding-level: no further progress */
    const double improvement = scale * (cost - cn);
    memcpy(a, an, nv * sizeof(double));
    memcpy(jar, jn, ne * sizeof(double));
    cost = cn;
    if (tol > 0 ? improvement < tol : improvement == 0) {
      it++;
      break;
    }
  }
  newton_stats[0] += 1;
  newton_stats[1] += it;
  d->solver_iter = it;
  d->flops += it * (2.0 * ne * nv * nv + (double)nv * nv * nv / 3.0);
  memcpy(d->qacc, a, nv * sizeof(double));
  for (int i = 0; i < nv; i++) d->qfrc_constraint[i] = 0;
  for (int r = 0; r < ne; r++) {
    int q;
    d->efc_force[r] = row_force(d, r, jar[r], &q);
    for (int i = 0; i < nv; i++) d->qfrc_constraint[i] += d->efc_J[r][i] * d->efc_force[r];
  }
}

/* --------------------------------------------------------- mj_forward [ext] */
void orc_forward(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  int nv = m->nv;
  orc_kinematics(om, d);
  orc_com_pos(om, d);
  orc_crb(om, d);
  orc_factor(om, d);
  if (m->disable_contact)
    d->ncon = 0;
  else
    orc_collision(om, d);
  orc_com_vel(om, d);
  orc_passive_actuation(om, d);
  orc_rne(om, d);
  for (int i = 0; i < nv; i++)
    d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i] + d->qfrc_applied[i];
  orc_solve_m(om, d, d->qacc_smooth, d->qfrc_smooth);
  orc_make_constraint(om, d);
  if (d->nefc) {
    if (m->solver == SIM_SOL_NEWTON)
      orc_solve_newton(om, d, m->tolerance); /* tolerance <= 0: to the exact optimum */
    else
      orc_solve_pgs(om, d);
  } else {
    memcpy(d->qacc, d->qacc_smooth, nv * sizeof(double));
    memset(d->qfrc_constraint, 0, sizeof(d->qfrc_constraint));
  }
  d->flops += 2.0 * nv * nv + 3.0 * nv;
}

static int bad(double x) { return !(x == x) || fabs(x) > MAXVAL; }

static void soft_reset(const orc_model* om, orc_data* d, int bit) {
  int st = d->status | bit;
  double fl = d->flops, cf = d->cflops;
  orc_reset_data(om, d);
  d->status = st;
  d->flops = fl;
  d->cflops = cf;
}

/* integrate positions: hinge/slide q += h v; free: pos += h v, quat *= exp(h w_local / 2) */
static void integrate_pos(const sim_model_desc* m, double* qpos, const double* qvel, double h) {
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == SIM_JNT_FREE) {
      for (int k = 0; k < 3; k++) qpos[qa + k] += h * qvel[da + k];
      double w[3] = {qvel[da + 3], qvel[da + 4], qvel[da + 5]};
      double n = sqrt(dot3(w, w));
      double* q = qpos + qa + 3;
      quat_normalize(q);
      if (n > MINVAL) {
        double ax[3] = {w[0] / n, w[1] / n, w[2] / n}, qr[4];
        axisangle_quat(qr, ax, n * h);
        quat_mul(q, q, qr);
      }
    } else {
      qpos[qa] += h * qvel[da];
    }
  }
}

/* ------------------------------------------------ mj_step (Euler) [ext] */
void orc_step(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  int nv = m->nv;
  for (int i = 0; i < m->nq; i++)
    if (bad(d->qpos[i])) {
      soft_reset(om, d, SIM_ST_BADQPOS);
      break;
    }
  for (int i = 0; i < nv; i++)
    if (bad(d->qvel[i])) {
      soft_reset(om, d, SIM_ST_BADQVEL);
      break;
    }
  orc_forward(om, d);
  for (int i = 0; i < nv; i++)
    if (bad(d->qacc[i])) {
      soft_reset(om, d, SIM_ST_BADQACC);
      orc_forward(om, d);
      break;
    }
  double h = m->timestep, qacc[SIM_MAXDOF];
  int damp = 0;
  if (!m->disable_eulerdamp)
    for (int i = 0; i < nv; i++)
      if (m->dof_damping[i] * om->damping_scale > 0) damp = 1;
  if (damp) {
    double H[SIM_MAXDOF][SIM_MAXDOF], LH[SIM_MAXDOF][SIM_MAXDOF], Hd[SIM_MAXDOF], rhs[SIM_MAXDOF];
    memcpy(H, d->M, sizeof(H));
    for (int i = 0; i < nv; i++) {
      H[i][i] += h * m->dof_damping[i] * om->damping_scale;
      rhs[i] = d->qfrc_smooth[i] + d->qfrc_constraint[i];
    }
    ldl(nv, H, LH, Hd);
    ldl_solve(nv, LH, Hd, qacc, rhs);
    d->flops += (double)nv * nv * nv / 3.0 + 2.0 * nv * nv;
  } else {
    memcpy(qacc, d->qacc, nv * sizeof(double));
  }
  for (int i = 0; i < nv; i++) d->qvel[i] += h * qacc[i];
  integrate_pos(m, d->qpos, d->qvel, h);
  memcpy(d->qacc_warmstart, d->qacc, nv * sizeof(double));
  d->flops += 4.0 * nv;
}

/* ================================================================ batch API */
static void make_om(orc_model* om, const sim_model_desc* m, const float* hv, const int32_t* hadr,
                    const int32_t* hadj, const double* params) {
  om->m = m;
  om->hull_vert = hv;
  om->hull_adr = hadr;
  om->hull_adj = hadj;
  om->hull_seed = NULL; /* callers with hulls set the seeds they computed once per call */
  om->mass_scale = params ? params[0] : 1.0;
  om->friction = params ? params[1] : -1.0;
  om->damping_scale = params ? params[2] : 1.0;
  om->pgs_warm = 0;
}

static void write_obs(const sim_model_desc* m, const orc_data* d, double* obs) {
  for (int k = 0; k < 3; k++) obs[k] = d->site_xpos[m->obs_site][k];
  for (int k = 0; k < m->obs_nq; k++) obs[3 + k] = d->qpos[m->obs_qadr[k]];
}

static int dof_of_qadr(const sim_model_desc* m, int qa) {
  for (int j = 0; j < m->njnt; j++)
    if (m->jnt_qposadr[j] == qa) return m->jnt_dofadr[j];
  return -1;
}

/* SOARM101Env.reset (SOARM101_Env.py:77-106): mj_resetData, overwrite
   qpos/qvel of the observed joints, mj_forward, _get_state.
   Arrays are row-major per env: qpos [n][nq], init_qpos [n][obs_nq], obs [n][3+obs_nq]. */
void orc_batch_reset(const sim_model_desc* m, int n, double* qpos, double* qvel, double* warm,
                     double* ctrl, const double* init_qpos, const double* init_qvel,
                     const double* extra_qpos, double* obs) {
  orc_model om;
  make_om(&om, m, NULL, NULL, NULL, NULL);
  for (int e = 0; e < n; e++) {
    orc_data d;
    orc_reset_data(&om, &d);
    if (extra_qpos)
      for (int i = 0; i < m->nq; i++) d.qpos[i] = extra_qpos[e * m->nq + i];
    for (int k = 0; k < m->obs_nq; k++) {
      if (init_qpos) d.qpos[m->obs_qadr[k]] = init_qpos[e * m->obs_nq + k];
      int da = dof_of_qadr(m, m->obs_qadr[k]);
      if (init_qvel && da >= 0) d.qvel[da] = init_qvel[e * m->obs_nq + k];
    }
    orc_kinematics(&om, &d);
    for (int i = 0; i < m->nq; i++) qpos[e * m->nq + i] = d.qpos[i];
    for (int i = 0; i < m->nv; i++) {
      qvel[e * m->nv + i] = d.qvel[i];
      warm[e * m->nv + i] = 0;
    }
    for (int i = 0; i < m->nu; i++) ctrl[e * m->nu + i] = 0;
    if (obs) write_obs(m, &d, obs + e * (3 + m->obs_nq));
  }
}

/* SOARM101Env.step (SOARM101_Env.py:108-142) for n envs: ctrl[:nact] = action,
   nsub x mj_step, obs = [site_xpos (from the last substep's forward pass, as
   MuJoCo leaves it), qpos[obs]]. */
void orc_batch_step(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                    const int32_t* hadj, int n, double* qpos, double* qvel, double* warm,
                    double* ctrl, const double* action, int nsub, double* obs, int32_t* status,
                    double* ncon_sum, const double* params, int nthreads, double* flops,
                    double* applied) {
  double fl_total = 0, cf_total = 0;
  int32_t seeds[SIM_MAXGEOM * ORC_NSEED];
  if (hv) orc_hull_seeds(m, hv, seeds);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(+ : fl_total, cf_total)
#endif
  for (int e = 0; e < n; e++) {
    orc_model om;
    make_om(&om, m, hv, hadr, hadj, params ? params + 3 * e : NULL);
    om.hull_seed = hv ? seeds : NULL;
    orc_data d;
    memset(&d, 0, sizeof(d));
    for (int i = 0; i < m->nq; i++) d.qpos[i] = qpos[e * m->nq + i];
    for (int i = 0; i < m->nv; i++) {
      d.qvel[i] = qvel[e * m->nv + i];
      d.qacc_warmstart[i] = warm[e * m->nv + i];
    }
    for (int i = 0; i < m->nu; i++) d.ctrl[i] = ctrl[e * m->nu + i];
    if (action)
      for (int i = 0; i < m->nact; i++) d.ctrl[i] = action[e * m->nact + i];
    d.status = status ? status[e] : 0;
    if (applied)
      for (int i = 0; i < m->nv; i++) d.qfrc_applied[i] = applied[e * m->nv + i];
    double nc = 0;
    for (int s = 0; s < nsub; s++) {
      orc_step(&om, &d);
      nc += d.ncon;
    }
    for (int i = 0; i < m->nq; i++) qpos[e * m->nq + i] = d.qpos[i];
    for (int i = 0; i < m->nv; i++) {
      qvel[e * m->nv + i] = d.qvel[i];
      warm[e * m->nv + i] = d.qacc_warmstart[i];
    }
    for (int i = 0; i < m->nu; i++) ctrl[e * m->nu + i] = d.ctrl[i];
    if (status) status[e] = d.status;
    if (applied)
      for (int i = 0; i < m->nv; i++) applied[e * m->nv + i] = d.qfrc_applied[i];
    if (ncon_sum) ncon_sum[e] += nc;
    if (obs) write_obs(m, &d, obs + e * (3 + m->obs_nq));
    fl_total += d.flops;
    cf_total += d.cflops;
  }
  (void)nthreads;
  if (flops) {
    flops[0] = fl_total; /* total */
    flops[1] = cf_total; /* of which collision */
  }
}

/* Koopman_MPC.py:119 reads d.qfrc_bias as left by mj_forward (Koopman_MPC.py:126) */
void orc_batch_bias(const sim_model_desc* m, int n, const double* qpos, const double* qvel,
                    const double* params, double* bias) {
  for (int e = 0; e < n; e++) {
    orc_model om;
    make_om(&om, m, NULL, NULL, NULL, params ? params + 3 * e : NULL);
    orc_data d;
    orc_reset_data(&om, &d);
    for (int i = 0; i < m->nq; i++) d.qpos[i] = qpos[e * m->nq + i];
    for (int i = 0; i < m->nv; i++) d.qvel[i] = qvel[e * m->nv + i];
    orc_kinematics(&om, &d);
    orc_com_pos(&om, &d);
    orc_crb(&om, &d);
    orc_com_vel(&om, &d);
    orc_rne(&om, &d);
    for (int i = 0; i < m->nv; i++) bias[e * m->nv + i] = d.qfrc_bias[i];
  }
}

int orc_debug_forward(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                      const int32_t* hadj, const double* qpos, const double* qvel,
                      const double* ctrl, const double* warm, double* M, double* bias,
                      double* qacc, double* contacts, double* site_xpos, double* geom_xpos,
                      double* efc_force, int* nefc) {
  int32_t seeds[SIM_MAXGEOM * ORC_NSEED];
  if (hv) orc_hull_seeds(m, hv, seeds);
  orc_model om;
  make_om(&om, m, hv, hadr, hadj, NULL);
  om.hull_seed = hv ? seeds : NULL;
  orc_data d;
  orc_reset_data(&om, &d);
  for (int i = 0; i < m->nq; i++) d.qpos[i] = qpos[i];
  for (int i = 0; i < m->nv; i++) {
    d.qvel[i] = qvel ? qvel[i] : 0;
    d.qacc_warmstart[i] = warm ? warm[i] : 0;
  }
  for (int i = 0; i < m->nu; i++) d.ctrl[i] = ctrl ? ctrl[i] : 0;
  orc_forward(&om, &d);
  int nv = m->nv;
  if (M)
    for (int i = 0; i < nv; i++)
      for (int j = 0; j < nv; j++) M[i * nv + j] = d.M[i][j];
  if (bias)
    for (int i = 0; i < nv; i++) bias[i] = d.qfrc_bias[i];
  if (qacc)
    for (int i = 0; i < nv; i++) qacc[i] = d.qacc[i];
  if (contacts)
    for (int c = 0; c < d.ncon; c++) {
      double* o = contacts + 9 * c;
      o[0] = d.contact[c].dist;
      for (int k = 0; k < 3; k++) o[1 + k] = d.contact[c].pos[k];
      for (int k = 0; k < 3; k++) o[4 + k] = d.contact[c].frame[k];
      o[7] = d.contact[c].geom1;
      o[8] = d.contact[c].geom2;
    }
  if (site_xpos)
    for (int s = 0; s < m->nsite; s++)
      for (int k = 0; k < 3; k++) site_xpos[3 * s + k] = d.site_xpos[s][k];
  if (geom_xpos)
    for (int g = 0; g < m->ngeom; g++)
      for (int k = 0; k < 3; k++) geom_xpos[3 * g + k] = d.geom_xpos[g][k];
  if (efc_force)
    for (int r = 0; r < d.nefc; r++) efc_force[r] = d.efc_force[r];
  if (nefc) *nefc = d.nefc;
  return d.ncon;
}

/* ---------------------------------------------------------------------------
 * dm_control utils.inverse_kinematics.qpos_from_site_pose [ext; restated from its published
 * algorithm], as called at control/TrajectoryGenerator.py:96-107 (tol 1e-6, rot_weight 0.5,
 * regularization_strength 1e-2, regularization_threshold 0.1, max_update_norm 2,
 * progress_thresh 20, max_steps 100; joints = the first `ndof` hinges):
 *   err_pos = target_pos - site_xpos
 *   err_rot = quat2vel(target_quat * conj(site_xquat), 1)       (target_quat given)
 *   err_norm = |err_pos| + rot_weight |err_rot|;  success if err_norm < tol
 *   J = mj_jacSite rows [jacp; jacr] of the joints (3 or 6 rows; rot_weight weighs only the norm)
 *   reg = strength if err_norm > threshold else 0
 *   dq = solve(J'J + reg I, J'err)   (reg > 0)
 *   dq = lstsq(J'J, J'err)           (reg = 0: pseudo-inverse, cutoff eps * largest eigenvalue)
 *   halt if err_norm/|dq| > progress_thresh; clip |dq| <= max_update_norm
 *   mj_integratePos(q, dq, 1); joint limits are NOT enforced.
 * q is [n][nq] row-major in/out; target_quat [n][4] (w, x, y, z) or NULL (position only).
 * ------------------------------------------------------------------------- */
static int chol_solve(int n, double A[8][8], double* x, const double* b) {
  double L[8][8] = {{0}};
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      double s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (s <= 0) return -1;
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  double y[8];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return 0;
}

/* numpy.linalg.lstsq(A, b, rcond=-1) for symmetric PSD A (n <= 8): eigen-decomposition by
   cyclic Jacobi rotations, pseudo-inverse with the cutoff eps * largest eigenvalue */
static void sym_lstsq(int n, double A[8][8], double* x, const double* b) {
  double a[8][8], V[8][8];
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) a[i][j] = A[i][j], V[i][j] = i == j;
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) off += a[p][q] * a[p][q];
    if (off < 1e-300) break;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) {
        if (fabs(a[p][q]) < 1e-300) continue;
        const double th = (a[q][q] - a[p][p]) / (2 * a[p][q]);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
        const double c = 1 / sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; k++) {
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq, a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; k++) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk, a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq, V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  double lmax = 0;
  for (int i = 0; i < n; i++) lmax = fmax(lmax, fabs(a[i][i]));
  const double cut = 2.220446049250313e-16 * n * lmax;
  for (int i = 0; i < n; i++) x[i] = 0;
  for (int e = 0; e < n; e++) {
    if (fabs(a[e][e]) <= cut) continue;
    double c = 0;
    for (int k = 0; k < n; k++) c += V[k][e] * b[k];
    c /= a[e][e];
    for (int k = 0; k < n; k++) x[k] += c * V[k][e];
  }
}

/* MuJoCo mju_quat2Vel(res, quat, dt = 1) */
static void quat2vel(double res[3], const double q[4]) {
  double ax[3] = {q[1], q[2], q[3]};
  const double s = sqrt(dot3(ax, ax));
  if (s < MINVAL) {
    res[0] = res[1] = res[2] = 0;
    return;
  }
  double speed = 2 * atan2(s, q[0]);
  if (speed > M_PI) speed -= 2 * M_PI;
  for (int k = 0; k < 3; k++) res[k] = ax[k] / s * speed;
}

void orc_ik_dls(const sim_model_desc* m, int n, const double* target, const double* target_quat, double* q,
                int32_t* ok, int32_t* iters, double tol, double rot_weight, double reg_thresh,
                double reg_strength, double max_update, double progress_thresh, int max_steps, int site,
                int ndof) {
  orc_model om;
  make_om(&om, m, NULL, NULL, NULL, NULL);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int e = 0; e < n; e++) {
    orc_data d;
    orc_reset_data(&om, &d);
    for (int i = 0; i < m->nq; i++) d.qpos[i] = q[e * m->nq + i];
    const double* tg = target + 3 * e;
    const double* tq = target_quat ? target_quat + 4 * e : NULL;
    const int nr = tq ? 6 : 3;
    int success = 0, it;
    for (it = 0; it < max_steps; it++) {
      orc_kinematics(&om, &d);
      double err[6] = {0};
      for (int k = 0; k < 3; k++) err[k] = tg[k] - d.site_xpos[site][k];
      double en = sqrt(err[0] * err[0] + err[1] * err[1] + err[2] * err[2]);
      if (tq) {
        /* site frame quaternion = body quaternion * site quaternion (mju_mat2Quat of site_xmat, up
           to a sign that quat2vel's > pi branch makes irrelevant) */
        double sq[4], cq[4], eq[4];
        quat_mul(sq, d.xquat[m->site_bodyid[site]], m->site_quat[site]);
        quat_normalize(sq);
        cq[0] = sq[0], cq[1] = -sq[1], cq[2] = -sq[2], cq[3] = -sq[3];
        quat_mul(eq, tq, cq);
        quat2vel(err + 3, eq);
        en += rot_weight * sqrt(err[3] * err[3] + err[4] * err[4] + err[5] * err[5]);
      }
      if (en < tol) {
        success = 1;
        break;
      }
      /* site Jacobian columns of the hinges that are ancestors of the site body */
      double J[6][8] = {{0}};
      int sb = m->site_bodyid[site];
      for (int j = 0; j < ndof; j++) {
        int b = m->jnt_bodyid[j], anc = 0;
        for (int x = sb; x > 0; x = m->body_parentid[x])
          if (x == b) anc = 1;
        if (!anc) continue;
        double r[3] = {d.site_xpos[site][0] - d.xanchor[j][0], d.site_xpos[site][1] - d.xanchor[j][1],
                       d.site_xpos[site][2] - d.xanchor[j][2]};
        double c[3] = {d.xaxis[j][1] * r[2] - d.xaxis[j][2] * r[1],
                       d.xaxis[j][2] * r[0] - d.xaxis[j][0] * r[2],
                       d.xaxis[j][0] * r[1] - d.xaxis[j][1] * r[0]};
        for (int k = 0; k < 3; k++) J[k][j] = c[k], J[3 + k][j] = d.xaxis[j][k];
      }
      double reg = en > reg_thresh ? reg_strength : 0.0;
      double dq[8] = {0};
      if (reg > 0 || tq) {
        double H[8][8], g[8];
        for (int a = 0; a < ndof; a++) {
          g[a] = 0;
          for (int k = 0; k < nr; k++) g[a] += J[k][a] * err[k];
          for (int b = 0; b < ndof; b++) {
            double h = 0;
            for (int k = 0; k < nr; k++) h += J[k][a] * J[k][b];
            H[a][b] = h + (a == b ? reg : 0);
          }
        }
        if (reg > 0)
          chol_solve(ndof, H, dq, g);
        else
          sym_lstsq(ndof, H, dq, g);
      } else {
        double A[8][8], y[3];
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) {
            double s = 0;
            for (int k = 0; k < ndof; k++) s += J[a][k] * J[b][k];
            A[a][b] = s;
          }
        if (chol_solve(3, A, y, err) != 0) break;
        for (int k = 0; k < ndof; k++) dq[k] = J[0][k] * y[0] + J[1][k] * y[1] + J[2][k] * y[2];
      }
      double dn = 0;
      for (int k = 0; k < ndof; k++) dn += dq[k] * dq[k];
      dn = sqrt(dn);
      if (en / dn > progress_thresh) break;
      if (dn > max_update)
        for (int k = 0; k < ndof; k++) dq[k] *= max_update / dn;
      for (int k = 0; k < ndof; k++) d.qpos[m->jnt_qposadr[k]] += dq[k];
    }
    for (int i = 0; i < m->nq; i++) q[e * m->nq + i] = d.qpos[i];
    if (ok) ok[e] = success;
    if (iters) iters[e] = it;
  }
}

/* ---------------------------------------------------------------------------
 * Experiment harness (tools/pgs_warm_exp.py; test infrastructure): n envs for T env-steps of
 * `nsub` substeps with per-step actions [T][n][nact], persistent per-env data, PGS with warm
 * start `mode` (orc_model.pgs_warm).  Per env-step and env: out_sweeps = mean PGS sweeps per
 * substep, out_gap[.][2] = max over the step's substeps of |qacc_PGS - qacc_Newton-exact| on
 * the arm dofs / the free dofs, for the same constraint problem (same rows).
 * ------------------------------------------------------------------------- */
void orc_experiment_pgs(const sim_model_desc* m, const float* hv, const int32_t* hadr, const int32_t* hadj,
                        int n, const double* qpos, const double* qvel, const double* warm, const double* actions,
                        int T, int nsub, int mode, int nthreads, double* out_sweeps, double* out_gap,
                        double* qpos_out) {
  int32_t seeds[SIM_MAXGEOM * ORC_NSEED];
  if (hv) orc_hull_seeds(m, hv, seeds);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
#endif
  for (int e = 0; e < n; e++) {
    orc_model om;
    make_om(&om, m, hv, hadr, hadj, NULL);
    om.hull_seed = hv ? seeds : NULL;
    om.pgs_warm = mode;
    orc_model ex = om;
    sim_model_desc mx = *m;
    mx.solver = SIM_SOL_NEWTON;
    mx.tolerance = 0;
    ex.m = &mx;
    orc_data* d = (orc_data*)calloc(1, sizeof(orc_data));
    orc_data* t = (orc_data*)calloc(1, sizeof(orc_data));
    for (int i = 0; i < m->nq; i++) d->qpos[i] = qpos[e * m->nq + i];
    for (int i = 0; i < m->nv; i++) d->qvel[i] = qvel[e * m->nv + i], d->qacc_warmstart[i] = warm[e * m->nv + i];
    for (int s = 0; s < T; s++) {
      for (int i = 0; i < m->nact; i++) d->ctrl[i] = actions[((size_t)s * n + e) * m->nact + i];
      double sw = 0, ga = 0, gf = 0;
      for (int k = 0; k < nsub; k++) {
        orc_step(&om, d);
        sw += d->solver_iter;
        /* the exact optimum of this substep's problem: rebuild the same rows from the state
           the step started at is not kept, so re-solve from d's rows (kept by orc_step) */
        memcpy(t, d, sizeof(orc_data));
        if (t->nefc) orc_solve_newton(&ex, t, 0.0);
        for (int i = 0; i < m->nv; i++) {
          const double g = fabs(t->qacc[i] - d->qacc[i]);
          if (i < 6) ga = fmax(ga, g); else gf = fmax(gf, g);
        }
      }
      out_sweeps[(size_t)s * n + e] = sw / nsub;
      out_gap[((size_t)s * n + e) * 2] = ga;
      out_gap[((size_t)s * n + e) * 2 + 1] = gf;
    }
    if (qpos_out)
      for (int i = 0; i < m->nq; i++) qpos_out[e * m->nq + i] = d->qpos[i];
    free(d);
    free(t);
  }
}
