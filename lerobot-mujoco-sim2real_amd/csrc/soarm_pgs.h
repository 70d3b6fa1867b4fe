// soarm_pgs.h — constraint rows + projected Gauss-Seidel dual solve.
//
// Restates MuJoCo's mj_makeConstraint / mj_makeImpedance / mj_solPGS
//  for the rows the hot path creates: one
// frictionloss row per arm dof (always active), joint-limit rows when a
// hinge is past its range, and 4 pyramidal edges per contact.  Rows are
// visited in MuJoCo's order (friction rows, then limits joint by joint
// lower/upper, then contacts), so the sweep matches the oracle's.
//
// Fixed rows live in per-slot registers (J = +-e_i, so W = M^-1 J' is a
// column of the arm block's inverse).  Contact edges keep J and W in a
// per-lane scratch slab in global memory (L2-resident, [slot][env] SoA).
#pragma once
#include "soarm_collide.h"

namespace soarm {

template <int NA, int NF>
struct ContactRows {
  static constexpr int NV = NA + 6 * NF;
  // scratch layout: for edge r (0..4*MAXCON-1): J[NV], W[NV] then scalars
  float* base;  // = scratch + e
  int stride;   // = n envs
  DEVI float& J(int r, int i) const { return base[((size_t)r * (2 * NV + 4) + i) * stride]; }
  DEVI float& W(int r, int i) const { return base[((size_t)r * (2 * NV + 4) + NV + i) * stride]; }
  DEVI float& S(int r, int k) const { return base[((size_t)r * (2 * NV + 4) + 2 * NV + k) * stride]; }
  // S: 0 aref, 1 R, 2 ARdiag, 3 force
};

template <int NA, int NF, bool CON>
DEVI void solve_constraints(Sim<NA, NF>& S, const ConLds& C, int ncon, const ContactRows<NA, NF>& cr) {
  constexpr int NV = Sim<NA, NF>::NV;
  const DModel& m = *S.mp;
  S.solve_m(S.qacc_s, S.fsmooth);

  // inverse of the arm block, column by column
  float Wa[NA][NA];
#pragma unroll
  for (int i = 0; i < NA; i++) {
    float ei[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) ei[k] = (k == i) ? 1.f : 0.f;
    ldl_solve<NA>(S.LA, S.DAi, Wa[i], ei);
  }

  // ---- fixed slots: [friction_i], then per joint [lower_i, upper_i]
  float f[3 * NA], aref[3 * NA], R[3 * NA], ARd[3 * NA];
  bool act[3 * NA];
#pragma unroll
  for (int i = 0; i < NA; i++) {
    act[i] = m.dof_frictionloss[i] > 0.f;
    R[i] = m.dof_fricR[i];
    aref[i] = -m.dof_fricB[i] * S.qvel[i];
    ARd[i] = Wa[i][i] + R[i];
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const int s = NA + 2 * i + side;
      const float dist = side == 0 ? S.qpos[i] - m.jnt_range[i][0] : m.jnt_range[i][1] - S.qpos[i];
      act[s] = m.jnt_limited[i] && dist < m.jnt_margin[i];
      const float imp = impedance(m.jnt_solimp[i], dist, m.jnt_margin[i]);
      R[s] = fmaxf(MINVALF, (1.f - imp) * m.dof_invweight0[i] / imp);
      const float vel = side == 0 ? S.qvel[i] : -S.qvel[i];
      aref[s] = -m.jnt_KB[i][1] * vel - m.jnt_KB[i][0] * imp * (dist - m.jnt_margin[i]);
      ARd[s] = Wa[i][i] + R[s];
    }
  }
  auto slot_dof = [](int s) { return s < NA ? s : (s - NA) >> 1; };
  auto slot_sgn = [](int s) { return (s < NA || ((s - NA) & 1) == 0) ? 1.f : -1.f; };

  // ---- contact edges -> scratch (J, W, aref, R, ARd)
  int ne = 0;
  if constexpr (CON) {
    ne = 4 * ncon;
    for (int c = 0; c < ncon; c++) {
      const int p = C.pair(c);
      const float cpos[3] = {C.pos(c, 0), C.pos(c, 1), C.pos(c, 2)};
      const float cdist = C.dist(c);
      const int b1 = m.geom_bodyid[m.pair_geom1[p]], b2 = m.geom_bodyid[m.pair_geom2[p]];
      // frame (mju_makeFrame)
      float fr[9] = {C.n(c, 0), C.n(c, 1), C.n(c, 2), 0, 0, 0, 0, 0, 0};
      {
        float y[3];
        if (fabsf(fr[1]) < 0.5f)
          y[0] = 0, y[1] = 1, y[2] = 0;
        else
          y[0] = 0, y[1] = 0, y[2] = 1;
        const float dd = dot3(fr, y);
        y[0] -= dd * fr[0], y[1] -= dd * fr[1], y[2] -= dd * fr[2];
        const float inv = rsqrtf(dot3(y, y));
        fr[3] = y[0] * inv, fr[4] = y[1] * inv, fr[5] = y[2] * inv;
        cross(fr + 6, fr, fr + 3);
      }
      // relative translational Jacobian (body2 - body1) at the contact point, in the contact frame
      float jd[3][NV];
#pragma unroll
      for (int i = 0; i < NV; i++) jd[0][i] = jd[1][i] = jd[2][i] = 0.f;
#pragma unroll
      for (int side = 0; side < 2; side++) {
        const int b = side ? b2 : b1;
        const float sg = side ? 1.f : -1.f;
        // arm dofs: dof i moves bodies >= i+2 of the chain
#pragma unroll
        for (int i = 0; i < NA; i++) {
          if (b >= i + 2 && b < 2 + NA) {
            float l[3];
            cross(l, S.cdof[i], cpos);
            const float jp[3] = {S.cdof[i][3] + l[0], S.cdof[i][4] + l[1], S.cdof[i][5] + l[2]};
#pragma unroll
            for (int k = 0; k < 3; k++) jd[k][i] += sg * dot3(fr + 3 * k, jp);
          }
        }
#pragma unroll
        for (int ff = 0; ff < NF; ff++) {
          const int fb = 2 + NA + ff, d0 = NA + 6 * ff;
          if (b == fb) {
            const float off[3] = {cpos[0] - S.xpos[fb][0], cpos[1] - S.xpos[fb][1],
                                  cpos[2] - S.xpos[fb][2]};
#pragma unroll
            for (int i = 0; i < 6; i++) {
              float l[3];
              cross(l, S.cdof[d0 + i], off);
              const float jp[3] = {S.cdof[d0 + i][3] + l[0], S.cdof[d0 + i][4] + l[1],
                                   S.cdof[d0 + i][5] + l[2]};
#pragma unroll
              for (int k = 0; k < 3; k++) jd[k][d0 + i] += sg * dot3(fr + 3 * k, jp);
            }
          }
        }
      }
      const float mu = S.fric >= 0.f ? S.fric : m.pair_friction[p];
      const float tran = m.pair_tran[p];
      const float margin = m.pair_margin[p];
      const float imp = impedance(m.pair_solimp[p], cdist, margin);
      const float diag = tran + mu * mu * tran;
      const float R0 = fmaxf(MINVALF, (1.f - imp) * diag / imp);
      const float Rpy = 2.f * mu * mu * R0 / m.impratio;
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
        const int r = 4 * c + ed;
        const int k = 1 + (ed >> 1);
        const float sg = (ed & 1) ? -1.f : 1.f;
        float J[NV], W[NV];
        float vel = 0.f;
#pragma unroll
        for (int i = 0; i < NV; i++) {
          J[i] = jd[0][i] + sg * mu * jd[k][i];
          vel += J[i] * S.qvel[i];
        }
        S.solve_m(W, J);
        float jw = 0.f;
#pragma unroll
        for (int i = 0; i < NV; i++) {
          jw += J[i] * W[i];
          cr.J(r, i) = J[i];
          cr.W(r, i) = W[i];
        }
        cr.S(r, 0) = -m.pair_KB[p][1] * vel - m.pair_KB[p][0] * imp * (cdist - margin);
        cr.S(r, 1) = Rpy;
        cr.S(r, 2) = jw + Rpy;
      }
    }
  }

  // ---- warm start from qacc_warmstart (forces implied by the primal), keep if it beats f = 0
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
#pragma unroll
  for (int s = 0; s < 3 * NA; s++) {
    const int i = slot_dof(s);
    const float sg = slot_sgn(s);
    const float jar = sg * S.warm[i] - aref[s];
    float fs;
    if (s < NA) {
      const float fl = m.dof_frictionloss[i];
      fs = (jar <= -fl * R[s]) ? fl : (jar >= fl * R[s]) ? -fl : -jar / R[s];
    } else {
      fs = jar < 0.f ? -jar / R[s] : 0.f;
    }
    f[s] = act[s] ? fs : 0.f;
#pragma unroll
    for (int k = 0; k < NA; k++) v[k] += Wa[i][k] * sg * f[s];
  }
  for (int r = 0; r < ne; r++) {
    float jar = -cr.S(r, 0);
#pragma unroll
    for (int i = 0; i < NV; i++) jar += cr.J(r, i) * S.warm[i];
    const float fs = jar < 0.f ? -jar / cr.S(r, 1) : 0.f;
    cr.S(r, 3) = fs;
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] += cr.W(r, i) * fs;
  }
  {
    float cost = 0.f;
#pragma unroll
    for (int s = 0; s < 3 * NA; s++) {
      const int i = slot_dof(s);
      const float sg = slot_sgn(s);
      cost += 0.5f * f[s] * (sg * v[i] - aref[s] + R[s] * f[s]) + 0.5f * f[s] * (sg * S.qacc_s[i] - aref[s]);
    }
    for (int r = 0; r < ne; r++) {
      float jv = 0.f, jq = 0.f;
#pragma unroll
      for (int i = 0; i < NV; i++) {
        jv += cr.J(r, i) * v[i];
        jq += cr.J(r, i) * S.qacc_s[i];
      }
      const float fr = cr.S(r, 3), ar = cr.S(r, 0);
      cost += 0.5f * fr * (jv - ar + cr.S(r, 1) * fr) + 0.5f * fr * (jq - ar);
    }
    if (cost > 0.f) {
#pragma unroll
      for (int s = 0; s < 3 * NA; s++) f[s] = 0.f;
      for (int r = 0; r < ne; r++) cr.S(r, 3) = 0.f;
#pragma unroll
      for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
    }
  }

  // ---- projected Gauss-Seidel sweeps
  float tr = 0.f;
#pragma unroll
  for (int i = 0; i < NA; i++) tr += S.MA[i * (i + 1) / 2 + i];
#pragma unroll
  for (int ff = 0; ff < NF; ff++)
#pragma unroll
    for (int i = 0; i < 6; i++) tr += S.MF[ff][i * (i + 1) / 2 + i];
  const float scale = 1.f / tr;
  for (int it = 0; it < m.iterations; it++) {
    float improvement = 0.f;
#pragma unroll
    for (int s = 0; s < 3 * NA; s++) {
      if (!act[s]) continue;
      const int i = slot_dof(s);
      const float sg = slot_sgn(s);
      const float res = sg * v[i] - aref[s] + R[s] * f[s];
      float fn = f[s] - res / ARd[s];
      if (s < NA) {
        const float fl = m.dof_frictionloss[i];
        fn = fminf(fmaxf(fn, -fl), fl);
      } else {
        fn = fmaxf(fn, 0.f);
      }
      const float df = fn - f[s];
#pragma unroll
      for (int k = 0; k < NA; k++) v[k] += Wa[i][k] * sg * df;
      f[s] = fn;
      improvement -= df * res + 0.5f * ARd[s] * df * df;
    }
    for (int r = 0; r < ne; r++) {
      float res = -cr.S(r, 0) + cr.S(r, 1) * cr.S(r, 3);
#pragma unroll
      for (int i = 0; i < NV; i++) res += cr.J(r, i) * v[i];
      const float fo = cr.S(r, 3);
      const float fn = fmaxf(fo - res / cr.S(r, 2), 0.f);
      const float df = fn - fo;
      if (df != 0.f) {
#pragma unroll
        for (int i = 0; i < NV; i++) v[i] += cr.W(r, i) * df;
        cr.S(r, 3) = fn;
        improvement -= df * res + 0.5f * cr.S(r, 2) * df * df;
      }
    }
    if (improvement * scale < m.tolerance) break;
  }

#pragma unroll
  for (int i = 0; i < NV; i++) {
    S.qacc[i] = v[i];
    S.fcon[i] = 0.f;
  }
#pragma unroll
  for (int s = 0; s < 3 * NA; s++) S.fcon[slot_dof(s)] += slot_sgn(s) * f[s];
  for (int r = 0; r < ne; r++) {
    const float fr = cr.S(r, 3);
#pragma unroll
    for (int i = 0; i < NV; i++) S.fcon[i] += cr.J(r, i) * fr;
  }
}

}  // namespace soarm
