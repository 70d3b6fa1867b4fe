// soarm_newton.h — MuJoCo's default constraint solver (primal Newton) on the device.
//
// The reference scene has no <option> (SOARM101/SO101/scene_with_table_v.xml:1-32), so the
// reference's mj_step (SOARM101_Env.py:131-132) solves its constraint problem with MuJoCo's
// default solver: primal Newton, iterations 100, tolerance 1e-8 [ext mj_solNewton].  The
// kernels' default is PGS (BASELINE.json north_star); a model compiled with solver="Newton"
// runs this instead, on the same rows (soarm_pgs.h builds them):
//
//   minimise c(a) = 1/2 (a - a0)' M (a - a0) + sum_r s_r(J_r a - aref_r),   a0 = qacc_smooth
//     s_r(x) = x^2 / 2R                    pyramid edges, limits: x < 0 (else 0)
//            = Huber(x; R, frictionloss)   dof frictionloss rows
//   gradient g = M (a - a0) - J' f(a);  Hessian H = M + J_q' D J_q over the rows in their
//   quadratic zone (D = 1/R);  p = -H^-1 g (dense LDL' of the nv x nv H);  exact line search
//   along p (1-D Newton on the piecewise-linear derivative, bracketed);  stop when
//   scale * improvement < tolerance or scale * |g| < tolerance (scale = 1 / (meaninertia nv)).
//   Warm start: qacc_warmstart unless qacc_smooth costs less (mj_fwdConstraint).
//
// The problem is strictly convex (R > 0): its optimum is unique and this converges to it in a
// few iterations from the warm start, so the result equals the reference's to fp32 precision
// (the oracle restatement: oracle/oracle.c orc_solve_newton).  Per row the arithmetic is short
// and independent across rows (no Gauss-Seidel chain): a contact contributes its frame
// Jacobian J_c = [J_n; J_t1; J_t2] once, edges e = J_n + s_e J_t(e) are formed in that 3-D
// space, and its Hessian term is J_c' K J_c with the 3x3 K = sum over quadratic edges of
// D u_e u_e' (u_e = (1, s_e on t(e))).
#pragma once

namespace soarm {

template <int NA, int NF, bool CON>
struct NewtonRows {
  static constexpr int NV = NA + 6 * NF;
  static constexpr int NH = NV * (NV + 1) / 2;
  const DModel& m;
  const RowLds& L;
  const ContactRows<NA, NF>& cr;
  const float *fR, *fa;  // frictionloss rows: R, aref (= -B qvel)
  int nlim, nl, ncon;

  // one pass over every row at a: cost, J' f, (want_h) the rows' Hessian terms added to H, and
  // sig, a signature of the rows' zones (quadratic / linear / inactive): Newton has converged
  // once a full step leaves it unchanged (the cost is one quadratic there)
  template <bool WANT_H>
  DEVI float pass(const float a[NV], float jtf[NV], float H[NH], uint32_t& sig) const {
    float cost = 0.f;
    sig = 0u;
#pragma unroll
    for (int i = 0; i < NV; i++) jtf[i] = 0.f;
    // frictionloss rows (J = e_i)
#pragma unroll
    for (int i = 0; i < NA; i++) {
      const float fl = m.dof_frictionloss[i], R = fR[i];
      const float x = a[i] - fa[i];
      float f, c;
      bool q = false;
      if (x <= -R * fl) {
        f = fl, c = -fl * x - 0.5f * R * fl * fl;
      } else if (x >= R * fl) {
        f = -fl, c = fl * x - 0.5f * R * fl * fl;
      } else {
        f = -x / R, c = 0.5f * x * x / R, q = fl > 0.f;
      }
      cost += c;
      jtf[i] += f;
      sig = sig * 3u + (q ? 1u : (x < 0.f ? 2u : 0u));
      if constexpr (WANT_H)
        if (q) H[i * (i + 1) / 2 + i] += 1.f / R;
    }
    // joint limits (J = sign e_dof)
    for (int l = 0; l < nlim; l++) {
      const int d = (int)L.lm(l, L_DOF);
      const float sg = L.lm(l, L_SGN), R = L.lm(l, L_R);
      float ad = 0.f;
#pragma unroll
      for (int i = 0; i < NA; i++) ad = i == d ? a[i] : ad;
      const float x = sg * ad - L.lm(l, L_AREF);
      sig = sig * 2u + (x < 0.f ? 1u : 0u);
      if (x < 0.f) {
        cost += 0.5f * x * x / R;
        const float f = -x / R;
#pragma unroll
        for (int i = 0; i < NA; i++) {
          jtf[i] += i == d ? sg * f : 0.f;
          if constexpr (WANT_H) H[i * (i + 1) / 2 + i] += i == d ? 1.f / R : 0.f;
        }
      }
    }
    if constexpr (CON) {
      // contacts in LDS records: the frame Jacobian once, the 4 pyramid edges in its 3-D space
      // one contact over the dof range [LO, HI) it can touch (J_c is zero elsewhere): the free
      // body's 6 dofs for the cube's contacts, the arm's for arm-only ones, all of them for an
      // arm-cube contact -- a wave-uniform choice, as the PGS sweeps make it
      auto contact = [&](int c, auto lo_c, auto hi_c) {
        constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
        float jc[3][NV];
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = LO; i < HI; i++) jc[q][i] = L.at(c, 12 * q + i);
        const float mu = L.at(c, F_MU), R = L.at(c, F_R), D = 1.f / R;
        float y[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = LO; i < HI; i++) y[q] = fmaf(jc[q][i], a[i], y[q]);
        float F[3] = {0.f, 0.f, 0.f}, K[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // K: nn n1 n2 11 12 22
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float s = (ed & 1) ? -mu : mu;
          const int t = 1 + (ed >> 1);
          const float x = y[0] + s * y[t] - L.at(c, F_AREF + ed);
          sig = sig * 2u + (x < 0.f ? 1u : 0u);
          if (x < 0.f) {
            cost += 0.5f * x * x * D;
            const float f = -x * D;
            F[0] += f, F[t] += s * f;
            K[0] += D, K[t] += s * D, K[t == 1 ? 3 : 5] += s * s * D;
          }
        }
#pragma unroll
        for (int i = LO; i < HI; i++) jtf[i] += jc[0][i] * F[0] + jc[1][i] * F[1] + jc[2][i] * F[2];
        if constexpr (WANT_H) {  // H += J_c' K J_c
          float kj[3][NV];
#pragma unroll
          for (int i = LO; i < HI; i++) {
            kj[0][i] = K[0] * jc[0][i] + K[1] * jc[1][i] + K[2] * jc[2][i];
            kj[1][i] = K[1] * jc[0][i] + K[3] * jc[1][i] + K[4] * jc[2][i];
            kj[2][i] = K[2] * jc[0][i] + K[4] * jc[1][i] + K[5] * jc[2][i];
          }
#pragma unroll
          for (int i = LO; i < HI; i++)
#pragma unroll
            for (int j = LO; j <= i; j++)
              H[i * (i + 1) / 2 + j] += jc[0][i] * kj[0][j] + jc[1][i] * kj[1][j] + jc[2][i] * kj[2][j];
        }
      };
      for (int c = 0; c < nl; c++) {
        const int fl = (int)L.at(c, F_FLAGS);
        if (NF > 0 && __all(fl == TOUCH_FREE))
          contact(c, std::integral_constant<int, NA>{}, std::integral_constant<int, NV>{});
        else if (__all(!(fl & TOUCH_FREE)))
          contact(c, std::integral_constant<int, 0>{}, std::integral_constant<int, NA>{});
        else
          contact(c, std::integral_constant<int, 0>{}, std::integral_constant<int, NV>{});
      }
      // contacts past the LDS records: per-edge rows in the global slab (rare)
      for (int r = 4 * nl; r < 4 * ncon; r++) {
        float J[NV], x = -cr.S(r, 0);
#pragma unroll
        for (int i = 0; i < NV; i++) J[i] = cr.J(r, i), x = fmaf(J[i], a[i], x);
        sig = sig * 2u + (x < 0.f ? 1u : 0u);
        if (x < 0.f) {
          const float D = 1.f / cr.S(r, 1), f = -x * D;
          cost += 0.5f * x * x * D;
#pragma unroll
          for (int i = 0; i < NV; i++) jtf[i] += J[i] * f;
          if constexpr (WANT_H)
#pragma unroll
            for (int i = 0; i < NV; i++)
#pragma unroll
              for (int j = 0; j <= i; j++) H[i * (i + 1) / 2 + j] += D * J[i] * J[j];
        }
      }
    }
    return cost;
  }

  // line-search data along p: per row the residual at a and its rate along p, in LDS scratch
  // (ext area; contacts: 4 edges each) -- evaluated at every line-search point
  DEVI void ls_setup(const float a[NV], const float p[NV]) const {
    if constexpr (CON) {
      for (int c = 0; c < nl; c++) {
        float ya[3] = {0.f, 0.f, 0.f}, yp[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = 0; i < NV; i++) {
            const float j = L.at(c, 12 * q + i);
            ya[q] = fmaf(j, a[i], ya[q]), yp[q] = fmaf(j, p[i], yp[q]);
          }
        const float mu = L.at(c, F_MU);
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float s = (ed & 1) ? -mu : mu;
          const int t = 1 + (ed >> 1);
          L.ex(XS_LIST + 8 * c + ed) = ya[0] + s * ya[t] - L.at(c, F_AREF + ed);
          L.ex(XS_LIST + 8 * c + 4 + ed) = yp[0] + s * yp[t];
        }
      }
      for (int r = 4 * nl; r < 4 * ncon; r++) {
        float x = -cr.S(r, 0), v = 0.f;
#pragma unroll
        for (int i = 0; i < NV; i++) x = fmaf(cr.J(r, i), a[i], x), v = fmaf(cr.J(r, i), p[i], v);
        cr.W(r, 0) = x, cr.W(r, 1) = v;  // (the PGS M^-1 J' slot: unused by Newton)
      }
    }
  }

  // d/dalpha and d2/dalpha2 of the rows' cost at a + alpha p (Gauss part added by the caller)
  DEVI void ls_eval(const float a[NV], const float p[NV], float al, float& d1, float& d2) const {
#pragma unroll
    for (int i = 0; i < NA; i++) {
      const float fl = m.dof_frictionloss[i], R = fR[i];
      const float x = a[i] - fa[i] + al * p[i];
      const float f = x <= -R * fl ? fl : (x >= R * fl ? -fl : -x / R);
      d1 -= f * p[i];
      d2 += (x > -R * fl && x < R * fl && fl > 0.f) ? p[i] * p[i] / R : 0.f;
    }
    for (int l = 0; l < nlim; l++) {
      const int d = (int)L.lm(l, L_DOF);
      const float sg = L.lm(l, L_SGN), R = L.lm(l, L_R);
      float ad = 0.f, pd = 0.f;
#pragma unroll
      for (int i = 0; i < NA; i++) ad = i == d ? a[i] : ad, pd = i == d ? p[i] : pd;
      const float x = sg * (ad + al * pd) - L.lm(l, L_AREF), v = sg * pd;
      if (x < 0.f) d1 += x * v / R, d2 += v * v / R;
    }
    if constexpr (CON) {
      for (int c = 0; c < nl; c++) {
        const float D = 1.f / L.at(c, F_R);
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float v = L.ex(XS_LIST + 8 * c + 4 + ed);
          const float x = fmaf(al, v, L.ex(XS_LIST + 8 * c + ed));
          if (x < 0.f) d1 += x * v * D, d2 += v * v * D;
        }
      }
      for (int r = 4 * nl; r < 4 * ncon; r++) {
        const float D = 1.f / cr.S(r, 1), v = cr.W(r, 1);
        const float x = fmaf(al, v, cr.W(r, 0));
        if (x < 0.f) d1 += x * v * D, d2 += v * v * D;
      }
    }
  }
};

// M x for the block-diagonal M (arm block packed lower, free bodies' diagonal blocks)
template <int NA, int NF>
DEVI void mul_m(const Sim<NA, NF>& S, const float x[], float y[]) {
#pragma unroll
  for (int i = 0; i < NA; i++) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NA; k++) s = fmaf(S.MA[i >= k ? i * (i + 1) / 2 + k : k * (k + 1) / 2 + i], x[k], s);
    y[i] = s;
  }
#pragma unroll
  for (int f = 0; f < NF; f++)
#pragma unroll
    for (int i = 0; i < 6; i++) y[NA + 6 * f + i] = S.MF[f][i * (i + 1) / 2 + i] * x[NA + 6 * f + i];
}

// Primal Newton solve of the rows built by solve_constraints; sets S.qacc and S.fcon = J' f.
// Returns the iteration count.
template <int NA, int NF, bool CON>
DEVI int newton_solve(Sim<NA, NF>& S, const NewtonRows<NA, NF, CON>& R) {
  constexpr int NV = NA + 6 * NF, NH = NV * (NV + 1) / 2;
  const DModel& m = *S.mp;
  const float scale = m.pgs_scale, tol = m.tolerance;
  const float* a0 = S.qacc_s;
  auto gauss = [&](const float a[NV], float Ma[NV]) {  // 1/2 (a - a0)' M (a - a0); Ma = M (a - a0)
    float da[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) da[i] = a[i] - a0[i];
    mul_m(S, da, Ma);
    float c = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) c = fmaf(0.5f * da[i], Ma[i], c);
    return c;
  };
  float a[NV], jtf[NV], H[NH], Ma[NV];
  uint32_t sig = 0u;
  // warm start: qacc_warmstart unless qacc_smooth costs less
  {
    float js[NV];
    const float cs = R.template pass<false>(a0, js, H, sig);
    const float cw = gauss(S.warm, Ma) + R.template pass<false>(S.warm, jtf, H, sig);
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] = cw < cs ? S.warm[i] : a0[i];
  }
  // an arm-cube contact (or a generic overflow row) couples the arm and free-body blocks of H;
  // otherwise H is block diagonal and factors as two 6x6 blocks
  bool coupled = NF > 0 && CON && __any(R.ncon > R.nl);
  if constexpr (NF > 0 && CON)
    for (int c = 0; c < R.nl; c++) coupled |= __any((int)R.L.at(c, F_FLAGS) == (TOUCH_ARM | TOUCH_FREE));
#pragma unroll
  for (int i = 0; i < NH; i++) H[i] = 0.f;
  float cost = gauss(a, Ma) + R.template pass<true>(a, jtf, H, sig);
  int it = 0;
  for (; it < m.iterations; it++) {
    float g[NV], gn = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) g[i] = Ma[i] - jtf[i], gn = fmaf(g[i], g[i], gn);
    if (scale * sqrtf(gn) < tol) break;
    // H = M + rows' terms; p = -H^-1 g
#pragma unroll
    for (int i = 0; i < NA; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) H[i * (i + 1) / 2 + j] += S.MA[i * (i + 1) / 2 + j];
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const int d = NA + 6 * f + i;
        H[d * (d + 1) / 2 + d] += S.MF[f][i * (i + 1) / 2 + i];
      }
    float p[NV], mg[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) mg[i] = -g[i];
    if (NF == 0 || coupled) {
      float Hd[NV];
      ldl_factor<NV>(H, Hd);
      ldl_solve<NV>(H, Hd, p, mg);
    } else {
      // block diagonal: the arm block is H's first 21 packed entries; the free block is gathered
      float Ha[NA * (NA + 1) / 2], Hf[21], Had[NA], Hfd[6];
#pragma unroll
      for (int k = 0; k < NA * (NA + 1) / 2; k++) Ha[k] = H[k];
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) Hf[i * (i + 1) / 2 + j] = H[(NA + i) * (NA + i + 1) / 2 + NA + j];
      ldl_factor<NA>(Ha, Had);
      ldl_solve<NA>(Ha, Had, p, mg);
      ldl_factor<6>(Hf, Hfd);
      ldl_solve<6>(Hf, Hfd, p + NA, mg + NA);
    }
    // exact line search: phi'(al) = (a - a0)' M p + al p' M p + rows; 1-D Newton, bracketed
    float Mp[NV], g0 = 0.f, pMp = 0.f;
    mul_m(S, p, Mp);
#pragma unroll
    for (int i = 0; i < NV; i++) {
      g0 = fmaf(a[i] - a0[i], Mp[i], g0);
      pMp = fmaf(p[i], Mp[i], pMp);
    }
    R.ls_setup(a, p);
    auto deriv = [&](float al, float& d2) {
      float d1 = fmaf(al, pMp, g0);
      d2 = pMp;
      R.ls_eval(a, p, al, d1, d2);
      return d1;
    };
    float h0;
    const float dz = deriv(0.f, h0);
    if (!(dz < 0.f)) break;  // not a descent direction at fp32 resolution: converged
    float lo = 0.f, hi = 3.0e38f, al = 1.f;
    for (int ls = 0; ls < 30; ls++) {
      float d2;
      const float d1 = deriv(al, d2);
      if (d1 < 0.f)
        lo = al;
      else
        hi = al;
      if (d1 == 0.f) break;
      float an = al - d1 / d2;  // exact within the current piece
      if (!(an > lo && an < hi)) an = hi < 3.0e38f ? 0.5f * (lo + hi) : 2.f * al;
      if (fabsf(an - al) <= 1e-6f * al) {
        al = an;
        break;
      }
      al = an;
    }
    float an_[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) an_[i] = fmaf(al, p[i], a[i]);
    float jn[NV], Man[NV];
#pragma unroll
    for (int i = 0; i < NH; i++) H[i] = 0.f;
    const uint32_t sig0 = sig;
    const float cn = gauss(an_, Man) + R.template pass<true>(an_, jn, H, sig);
    if (!(cn <= cost)) break;  // rounding-level: no further progress (keep a)
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] = an_[i], jtf[i] = jn[i], Ma[i] = Man[i];
    const float improvement = cost - cn;
    cost = cn;
    // MuJoCo's test; its fp32 floor (a relative improvement at rounding level); and exactness:
    // a full Newton step that leaves every row in its zone minimised the one quadratic there
    if (scale * improvement < tol || improvement <= 1e-6f * fabsf(cn) ||
        (sig == sig0 && fabsf(al - 1.f) < 1e-3f)) {
      it++;
      break;
    }
  }
#pragma unroll
  for (int i = 0; i < NV; i++) S.qacc[i] = a[i], S.fcon[i] = jtf[i];
  return it;
}

}  // namespace soarm
