// soarm_step.h — the fused per-env physics (smooth dynamics, constraint rows,
// PGS, implicit-damping Euler).  Collision lives in soarm_collide.h.
#pragma once
#include "soarm_kernels.h"

namespace soarm {

template <int NA, int NF>
struct Sim {
  static constexpr int NB = 2 + NA + NF;
  static constexpr int NV = NA + 6 * NF;
  static constexpr int NQ = NA + 7 * NF;
  static constexpr int NLA = NA * (NA + 1) / 2;
  static constexpr int NSLOT = 3 * NA;  // friction, lower limit, upper limit per arm dof

  const DModel* mp;  // laundered once per substep (see relaunder) so uniform loads are not
                     // hoisted across substeps and held live in SGPRs
  float mscale, fric, dscale;

  // state
  float qpos[NQ], qvel[NV], warm[NV], ctrl[NA];
  int status;

  // kinematics
  float xpos[NB][3], xmat[NB][9], xquat[NB][4];
  float anchor[NA][3], axis[NA][3];
  float ee[3];

  // dynamics
  float cinert[NB][10];
  float cdof[NV][6];
  float MA[NLA], LA[NLA], DAi[NA];
  float MF[NF > 0 ? NF : 1][21], LF[NF > 0 ? NF : 1][21], DFi[NF > 0 ? NF : 1][6];
  float cdofdot[NV][6];
  float fsmooth[NV], qacc_s[NV], qacc[NV], fcon[NV];
  // Newton's zone prediction for the frictionloss rows (soarm_newton.h): 2 bits per dof (the pass's
  // zone codes), bit 31 = set; zpred in (from the caller's history), zfin out (the solve's result)
  uint32_t zpred = 0u, zfin = 0u;

  HDI Sim(const DModel* m_, float ms, float fr, float ds) : mp(m_), mscale(ms), fric(fr), dscale(ds) {}
  HDI void relaunder() {  // (through the constant address space: the model stays scalar-loaded)
#if SOARM_DEVICE_PASS
    auto c = (__attribute__((address_space(4))) const DModel*)mp;
    asm volatile("" : "+s"(c));
    mp = (const DModel*)c;
#endif
  }

  // ---------------------------------------------------------------- mj_kinematics
  HDI void kinematics() {
    const DModel& m = *mp;
    xpos[0][0] = xpos[0][1] = xpos[0][2] = 0.f;
    xquat[0][0] = 1.f, xquat[0][1] = xquat[0][2] = xquat[0][3] = 0.f;
#pragma unroll
    for (int b = 1; b < 2 + NA; b++) {
      const int p = b - 1;  // base's parent is the world; chain is serial
      float R[9], t[3], pos[3], q[4];
      if (p == 0) {
        R[0] = R[4] = R[8] = 1.f, R[1] = R[2] = R[3] = R[5] = R[6] = R[7] = 0.f;
      } else {  // the parent's frame, converted from its final quaternion in its own iteration
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = xmat[p][k];
      }
      const float bp[3] = {m.body_pos[b][0], m.body_pos[b][1], m.body_pos[b][2]};
      mv(t, R, bp);
      pos[0] = xpos[p][0] + t[0], pos[1] = xpos[p][1] + t[1], pos[2] = xpos[p][2] + t[2];
      const float bq[4] = {m.body_quat[b][0], m.body_quat[b][1], m.body_quat[b][2], m.body_quat[b][3]};
      qmul(q, xquat[p], bq);
      if (b >= 2) {
        const int j = b - 2;
        const float jp[3] = {m.jnt_pos[j][0], m.jnt_pos[j][1], m.jnt_pos[j][2]};
        const float ja[3] = {m.jnt_axis[j][0], m.jnt_axis[j][1], m.jnt_axis[j][2]};
        q2m(R, q);
        mv(t, R, jp);
        anchor[j][0] = pos[0] + t[0], anchor[j][1] = pos[1] + t[1], anchor[j][2] = pos[2] + t[2];
        mv(axis[j], R, ja);
        float s, c;
        fsincos(0.5f * (qpos[j] - m.qpos0[j]), &s, &c);
        const float ql[4] = {c, ja[0] * s, ja[1] * s, ja[2] * s};
        qmul(q, q, ql);
        q2m(R, q);
        mv(t, R, jp);
        pos[0] = anchor[j][0] - t[0], pos[1] = anchor[j][1] - t[1], pos[2] = anchor[j][2] - t[2];
      }
      qnormalize(q);
#pragma unroll
      for (int k = 0; k < 4; k++) xquat[b][k] = q[k];
#pragma unroll
      for (int k = 0; k < 3; k++) xpos[b][k] = pos[k];
      q2m(xmat[b], q);
    }
#pragma unroll
    for (int f = 0; f < NF; f++) {
      const int b = 2 + NA + f, qa = NA + 7 * f;
      float q[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]};
      qnormalize(q);
#pragma unroll
      for (int k = 0; k < 4; k++) xquat[b][k] = q[k];
#pragma unroll
      for (int k = 0; k < 3; k++) xpos[b][k] = qpos[qa + k];
      q2m(xmat[b], q);
    }
    // observed site (runtime body id -> select over the unrolled bodies)
    const int sb = m.site_bodyid[m.obs_site];
    const float sp[3] = {m.site_pos[m.obs_site][0], m.site_pos[m.obs_site][1], m.site_pos[m.obs_site][2]};
#pragma unroll
    for (int b = 1; b < NB; b++)
      if (b == sb) {
        float t[3];
        mv(t, xmat[b], sp);
        ee[0] = xpos[b][0] + t[0], ee[1] = xpos[b][1] + t[1], ee[2] = xpos[b][2] + t[2];
      }
  }

  // ---------------------------------------------------- mj_comPos + mj_crb/makeM
  HDI void com_crb() {
    const DModel& m = *mp;
#pragma unroll
    for (int b = 1; b < NB; b++) {
      const bool freeb = b >= 2 + NA;
      const float mass = m.body_mass[b] * mscale;
      float ximat[9], xip[3];
      const float imat[9] = {m.body_imat[b][0], m.body_imat[b][1], m.body_imat[b][2],
                             m.body_imat[b][3], m.body_imat[b][4], m.body_imat[b][5],
                             m.body_imat[b][6], m.body_imat[b][7], m.body_imat[b][8]};
      mm(ximat, xmat[b], imat);
      const float ip[3] = {m.body_ipos[b][0], m.body_ipos[b][1], m.body_ipos[b][2]};
      mv(xip, xmat[b], ip);
      // reference point: arm -> world origin (base frame), free body -> its own origin
      float c[3];
      if (freeb)
        c[0] = xip[0], c[1] = xip[1], c[2] = xip[2];
      else
        c[0] = xpos[b][0] + xip[0], c[1] = xpos[b][1] + xip[1], c[2] = xpos[b][2] + xip[2];
      const float in0 = m.body_inertia[b][0] * mscale, in1 = m.body_inertia[b][1] * mscale,
                  in2 = m.body_inertia[b][2] * mscale;
      const float* R = ximat;
      const float Ixx = R[0] * R[0] * in0 + R[1] * R[1] * in1 + R[2] * R[2] * in2;
      const float Iyy = R[3] * R[3] * in0 + R[4] * R[4] * in1 + R[5] * R[5] * in2;
      const float Izz = R[6] * R[6] * in0 + R[7] * R[7] * in1 + R[8] * R[8] * in2;
      const float Ixy = R[0] * R[3] * in0 + R[1] * R[4] * in1 + R[2] * R[5] * in2;
      const float Ixz = R[0] * R[6] * in0 + R[1] * R[7] * in1 + R[2] * R[8] * in2;
      const float Iyz = R[3] * R[6] * in0 + R[4] * R[7] * in1 + R[5] * R[8] * in2;
      const float cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
      float* ci = cinert[b];
      ci[0] = Ixx + mass * (cc - c[0] * c[0]);
      ci[1] = Iyy + mass * (cc - c[1] * c[1]);
      ci[2] = Izz + mass * (cc - c[2] * c[2]);
      ci[3] = Ixy - mass * c[0] * c[1];
      ci[4] = Ixz - mass * c[0] * c[2];
      ci[5] = Iyz - mass * c[1] * c[2];
      ci[6] = mass * c[0], ci[7] = mass * c[1], ci[8] = mass * c[2];
      ci[9] = mass;
    }
    // cdof: hinge = [axis; anchor x axis] (reference at origin)
#pragma unroll
    for (int i = 0; i < NA; i++) {
      cdof[i][0] = axis[i][0], cdof[i][1] = axis[i][1], cdof[i][2] = axis[i][2];
      float l[3];
      cross(l, anchor[i], axis[i]);
      cdof[i][3] = l[0], cdof[i][4] = l[1], cdof[i][5] = l[2];
    }
#pragma unroll
    for (int f = 0; f < NF; f++) {
      const int b = 2 + NA + f, d0 = NA + 6 * f;
#pragma unroll
      for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int e = 0; e < 6; e++) cdof[d0 + k][e] = (e == 3 + k) ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 3; e++) cdof[d0 + 3 + k][e] = xmat[b][3 * e + k];
        cdof[d0 + 3 + k][3] = cdof[d0 + 3 + k][4] = cdof[d0 + 3 + k][5] = 0.f;
      }
    }
    // composite rigid body inertia, arm chain
    float crb[10];
#pragma unroll
    for (int k = 0; k < 10; k++) crb[k] = 0.f;
#pragma unroll
    for (int i = NA - 1; i >= 0; i--) {
#pragma unroll
      for (int k = 0; k < 10; k++) crb[k] += cinert[i + 2][k];
      float buf[6];
      inert_mul(buf, crb, cdof[i]);
#pragma unroll
      for (int j = 0; j <= i; j++) MA[i * (i + 1) / 2 + j] = dot6(cdof[j], buf);
      MA[i * (i + 1) / 2 + i] += m.dof_armature[i];
    }
#pragma unroll
    for (int f = 0; f < NF; f++) {
      const int b = 2 + NA + f, d0 = NA + 6 * f;
#pragma unroll
      for (int i = 0; i < 6; i++) {
        float buf[6];
        inert_mul(buf, cinert[b], cdof[d0 + i]);
#pragma unroll
        for (int j = 0; j <= i; j++) MF[f][i * (i + 1) / 2 + j] = dot6(cdof[d0 + j], buf);
        MF[f][i * (i + 1) / 2 + i] += m.dof_armature[d0 + i];
      }
    }
  }

  HDI void factor() {
    const DModel& m = *mp;
#pragma unroll
    for (int k = 0; k < NLA; k++) LA[k] = MA[k];
    ldl_factor<NA>(LA, DAi);
#pragma unroll
    for (int f = 0; f < NF; f++) {
#pragma unroll
      for (int k = 0; k < 21; k++) LF[f][k] = MF[f][k];
      ldl_factor<6>(LF[f], DFi[f]);
    }
  }

  // x = M^-1 b (block diagonal)
  HDI void solve_m(float x[NV], const float b[NV]) const {
    const DModel& m = *mp;
    ldl_solve<NA>(LA, DAi, x, b);
#pragma unroll
    for (int f = 0; f < NF; f++) ldl_solve<6>(LF[f], DFi[f], x + NA + 6 * f, b + NA + 6 * f);
  }

  // ------------------------------- mj_comVel + mj_rne(flg_acc=0) + passive + actuation
  // RNE_ONLY: fsmooth = -qfrc_bias (gravity + Coriolis/centrifugal), no passive/actuation
  template <bool RNE_ONLY = false>
  HDI void smooth_forces() {
    const DModel& m = *mp;
    // arm chain
    float cv[6] = {0, 0, 0, 0, 0, 0};
    float ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    float cfr[NA][6];
#pragma unroll
    for (int i = 0; i < NA; i++) {
      cross_motion(cdofdot[i], cv, cdof[i]);
#pragma unroll
      for (int e = 0; e < 6; e++) {
        cv[e] += cdof[i][e] * qvel[i];
        ca[e] += cdofdot[i][e] * qvel[i];
      }
      float t1[6], t2[6], t3[6];
      inert_mul(t1, cinert[i + 2], ca);
      inert_mul(t2, cinert[i + 2], cv);
      cross_force(t3, cv, t2);
#pragma unroll
      for (int e = 0; e < 6; e++) cfr[i][e] = t1[e] + t3[e];
    }
    float acc[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = NA - 1; i >= 0; i--) {
#pragma unroll
      for (int e = 0; e < 6; e++) acc[e] += cfr[i][e];
      fsmooth[i] = -dot6(cdof[i], acc);
    }
    // free bodies
#pragma unroll
    for (int f = 0; f < NF; f++) {
      const int b = 2 + NA + f, d0 = NA + 6 * f;
      float v[6] = {0, 0, 0, qvel[d0], qvel[d0 + 1], qvel[d0 + 2]};
      float a[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
#pragma unroll
      for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int e = 0; e < 6; e++) cdofdot[d0 + k][e] = 0.f;
        cross_motion(cdofdot[d0 + 3 + k], v, cdof[d0 + 3 + k]);
      }
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int e = 0; e < 6; e++) v[e] += cdof[d0 + 3 + k][e] * qvel[d0 + 3 + k];
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int e = 0; e < 6; e++) a[e] += cdofdot[d0 + 3 + k][e] * qvel[d0 + 3 + k];
      float t1[6], t2[6], t3[6], fb[6];
      inert_mul(t1, cinert[b], a);
      inert_mul(t2, cinert[b], v);
      cross_force(t3, v, t2);
#pragma unroll
      for (int e = 0; e < 6; e++) fb[e] = t1[e] + t3[e];
#pragma unroll
      for (int k = 0; k < 6; k++) fsmooth[d0 + k] = -dot6(cdof[d0 + k], fb);
    }
    if constexpr (RNE_ONLY) return;
    // passive damping + actuators (actuator a -> dof a)
#pragma unroll
    for (int i = 0; i < NV; i++) fsmooth[i] -= m.dof_damping[i] * dscale * qvel[i];
#pragma unroll
    for (int a = 0; a < NA; a++) {
      if (a >= m.nu) break;
      float c = ctrl[a];
      if (m.act_ctrllimited[a]) c = fminf(fmaxf(c, m.act_ctrlrange[a][0]), m.act_ctrlrange[a][1]);
      const float g = m.act_gear[a];
      float force = m.act_gain[a] * c + m.act_bias[a][0] + m.act_bias[a][1] * g * qpos[a] +
                    m.act_bias[a][2] * g * qvel[a];
      if (m.act_forcelimited[a])
        force = fminf(fmaxf(force, m.act_forcerange[a][0]), m.act_forcerange[a][1]);
      fsmooth[a] += g * force;
    }
  }

  // qfrc_smooth += qfrc_applied ([nv][N] SoA, caller-owned)
  HDI void add_applied(const float* applied, int n, int e) {
#pragma unroll
    for (int i = 0; i < NV; i++) fsmooth[i] += soa(applied, i, n, e);
  }

  // ---------------------------------------------------------- Euler integration
  HDI void integrate() {
    const DModel& m = *mp;
    const float h = m.timestep;
    float qa[NV];
    if (m.eulerdamp) {
      // (M + h D) a = qfrc_smooth + qfrc_constraint  (mj_Euler implicit damping)
      float rhs[NV];
#pragma unroll
      for (int i = 0; i < NV; i++) rhs[i] = fsmooth[i] + fcon[i];
      float H[NLA], Hd[NA];
#pragma unroll
      for (int k = 0; k < NLA; k++) H[k] = MA[k];
#pragma unroll
      for (int i = 0; i < NA; i++) H[i * (i + 1) / 2 + i] += h * m.dof_damping[i] * dscale;
      ldl_factor<NA>(H, Hd);
      ldl_solve<NA>(H, Hd, qa, rhs);
#pragma unroll
      for (int f = 0; f < NF; f++) {
        const int d0 = NA + 6 * f;
        float Hf[21], Hfd[6];
#pragma unroll
        for (int k = 0; k < 21; k++) Hf[k] = MF[f][k];
#pragma unroll
        for (int i = 0; i < 6; i++) Hf[i * (i + 1) / 2 + i] += h * m.dof_damping[d0 + i] * dscale;
        ldl_factor<6>(Hf, Hfd);
        ldl_solve<6>(Hf, Hfd, qa + d0, rhs + d0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; i++) qa[i] = qacc[i];
    }
    advance(qa);
  }
  // qvel += h a; qpos += h qvel (free bodies: quaternion by the angular velocity); warm start = qacc
  HDI void advance(const float (&qa)[NV]) {
    const DModel& m = *mp;
    const float h = m.timestep;
#pragma unroll
    for (int i = 0; i < NV; i++) qvel[i] += h * qa[i];
#pragma unroll
    for (int i = 0; i < NA; i++) qpos[i] += h * qvel[i];
#pragma unroll
    for (int f = 0; f < NF; f++) {
      const int q0 = NA + 7 * f, d0 = NA + 6 * f;
#pragma unroll
      for (int k = 0; k < 3; k++) qpos[q0 + k] += h * qvel[d0 + k];
      float q[4] = {qpos[q0 + 3], qpos[q0 + 4], qpos[q0 + 5], qpos[q0 + 6]};
      qnormalize(q);
      const float w[3] = {qvel[d0 + 3], qvel[d0 + 4], qvel[d0 + 5]};
      const float n2 = dot3(w, w);
      if (n2 > 1e-30f) {
        const float n = sqrtf(n2), inv = 1.f / n;
        float s, c;
        fsincos(0.5f * n * h, &s, &c);
        const float qr[4] = {c, w[0] * inv * s, w[1] * inv * s, w[2] * inv * s};
        qmul(q, q, qr);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) qpos[q0 + 3 + k] = q[k];
    }
#pragma unroll
    for (int i = 0; i < NV; i++) warm[i] = qacc[i];
  }

  // The implicit-damping Euler step in two halves (the RS contact kernel): (M + h D) a = qfrc_smooth
  // + qfrc_constraint = M qacc, so a = qacc - (M + h D)^-1 h D qacc.  damp_factor() factors H = M + h D
  // before the constraint solve (arm block: LDL' into LH / DHi; free bodies: their diagonal blocks,
  // a_i = qacc_i M_ii / (M_ii + h d_i)), integrate_qacc() finishes the step from qacc alone -- no
  // mass matrix, no qfrc_smooth and no factorization after the solve.
  float LH[NLA], DHi[NA], kf[NF > 0 ? NF : 1][6];
  HDI void damp_factor() {
    const DModel& m = *mp;
    const float h = m.timestep;
#pragma unroll
    for (int k = 0; k < NLA; k++) LH[k] = MA[k];
#pragma unroll
    for (int i = 0; i < NA; i++) LH[i * (i + 1) / 2 + i] += h * m.dof_damping[i] * dscale;
    ldl_factor<NA>(LH, DHi);
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const float mi = MF[f][i * (i + 1) / 2 + i];
        kf[f][i] = mi / (mi + h * m.dof_damping[NA + 6 * f + i] * dscale);
      }
  }
  HDI void integrate_qacc() {
    const DModel& m = *mp;
    const float h = m.timestep;
    float qa[NV];
    if (m.eulerdamp) {
      float y[NA], x[NA];
#pragma unroll
      for (int i = 0; i < NA; i++) y[i] = h * m.dof_damping[i] * dscale * qacc[i];
      ldl_solve<NA>(LH, DHi, x, y);
#pragma unroll
      for (int i = 0; i < NA; i++) qa[i] = qacc[i] - x[i];
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int i = 0; i < 6; i++) qa[NA + 6 * f + i] = kf[f][i] * qacc[NA + 6 * f + i];
    } else {
#pragma unroll
      for (int i = 0; i < NV; i++) qa[i] = qacc[i];
    }
    advance(qa);
  }

  // mj_resetData for this env (MuJoCo's auto-reset on a bad state)
  HDI void soft_reset(int bit) {
    const DModel& m = *mp;
    status |= bit;
#pragma unroll
    for (int i = 0; i < NQ; i++) qpos[i] = m.qpos0[i];
#pragma unroll
    for (int i = 0; i < NV; i++) qvel[i] = warm[i] = 0.f;
#pragma unroll
    for (int i = 0; i < NA; i++) ctrl[i] = 0.f;
  }
  // true when it reset the env (the status bits are sticky: a second reset for the same cause
  // leaves them as they were, so callers test this, not a status change)
  HDI bool check_state() {
    const DModel& m = *mp;
    bool bq = false, bv = false;
#pragma unroll
    for (int i = 0; i < NQ; i++) bq |= bad(qpos[i]);
    if (bq) soft_reset(SIM_ST_BADQPOS);
#pragma unroll
    for (int i = 0; i < NV; i++) bv |= bad(qvel[i]);
    if (bv) soft_reset(SIM_ST_BADQVEL);
    return bq || bv;
  }
  HDI bool acc_bad() const {
    const DModel& m = *mp;
    bool b = false;
#pragma unroll
    for (int i = 0; i < NV; i++) b |= bad(qacc[i]);
    return b;
  }
};

}  // namespace soarm
