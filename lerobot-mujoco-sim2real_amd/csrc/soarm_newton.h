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
//   quadratic zone (D = 1/R);  p = -H^-1 g (dense LDL');  exact line search along p (1-D Newton
//   on the piecewise-linear derivative, bracketed);  stop when scale * improvement < tolerance
//   or scale * |g| < tolerance (scale = 1 / (meaninertia nv)).
//   Warm start: qacc_warmstart unless qacc_smooth costs less (mj_fwdConstraint).
//
// The problem is strictly convex (R > 0): its optimum is unique and Newton reaches it in a few
// iterations from the warm start, so the result equals the reference's to fp32 precision (the
// oracle restatement: oracle/oracle.c orc_solve_newton).
//
// Decomposition.  M is block diagonal (arm chain | free body) and a row couples the two blocks
// only if it is a contact between an arm link and the cube.  Without such a contact in the wave
// the cost separates, c(a) = c_arm(a_arm) + c_free(a_free), and the two 6-dof problems are solved
// one after the other (same optimum; half the Hessian, so half the registers); with one, the
// whole 12-dof problem is solved.  A contact contributes its frame Jacobian J_c = [J_n; J_t1;
// J_t2] once: its 4 pyramid edges e = J_n + s_e J_t(e) live in that 3-D space, and its Hessian
// term is J_c' K J_c with the 3x3 K = sum over quadratic edges of D u_e u_e' (u_e = (1, s_e on
// t(e))).
#pragma once

namespace soarm {

#ifdef SOARM_PHASE_PROF
// diagnostic build: [0] solves (one lane per env), [1] sum of iterations, [2] sum of line-search
// evaluations, [3] solves on the coupled (whole-problem) path, [4] sum of solve cycles, [5] max
// solve cycles, [6] max iterations, [7] max line-search evaluations of one solve; split solves
// (per env): [8] arm iterations, [9] arm evaluations, [10] free-body iterations, [11] free-body
// evaluations; per wave: [12] waves, [13] sum over waves of the wave's max evaluations, [14] of
// its max iterations, [15] sum of the wave's max solve cycles; per env (sum over both ranges):
// [16] warm-start cycles, [17] Hessian + factor + solve cycles, [18] line-search cycles,
// [19] cycles of the pass at the new point, [20] wave-max sum of [16], [21] of [17], [22] of [18],
// [23] of [19]
__device__ unsigned long long g_newton[24];
#define NT_STAMP(k)                          \
  {                                          \
    const long long t_ = clock64();          \
    ncyc[k] += t_ - nt_;                     \
    nt_ = t_;                                \
  }
DEVI int wave_max_i(int v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
#else
#define NT_STAMP(k)
#endif

template <int NA, int NF, bool CON>
struct NewtonRows {
  static constexpr int NV = NA + 6 * NF;
  const DModel& m;
  const RowLds& L;
  const ContactRows<NA, NF>& cr;
  const float *fR, *fiR, *fa;  // frictionloss rows: R, 1/R, aref (= -B qvel)
  // (1/R of contacts and limits: the record's F_IARD / L_IARD slot, written for Newton by the
  // row build; divisions by R are multiplications by it throughout)
  int nlim, nl, ncon;
  // wave-uniform: some lane of the wave has a contact owned by the arm (resp. free-body)
  // subsystem; a subsystem without one skips its contact loops (set by newton_solve)
  bool arm_c = true, free_c = true;
  template <int LO, int HI>
  DEVI bool has_contacts() const {
    if constexpr (LO == 0 && HI == NV) return true;
    else if constexpr (HI == NA) return arm_c;
    else return free_c;
  }

  // does the subsystem over dofs [LO, HI) own a contact of class fl?  (full range: all of them)
  template <int LO, int HI>
  static DEVI bool owns(int fl) {
    if constexpr (LO == 0 && HI == NV) return true;
    else if constexpr (HI == NA) return !(fl & TOUCH_FREE);
    else return fl == TOUCH_FREE;
  }
  static constexpr int hidx(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower, i >= j

  // Quad mode (lpe() = 4 lanes per env): the env's contacts (and overflow rows) are split over
  // its lanes, lane k taking contacts k, k+4, ...; the partial sums are combined by quad
  // butterflies (bit-identical on the 4 lanes), so every later step runs on identical values.
  // The dof rows (frictionloss, limits) are cheap and run on every lane.
  static constexpr int QL = lpe<NF>();
  static_assert(QL == 1 || QL == 4, "Newton lane split: 1 or 4 lanes per env");
  DEVI int ql() const { return QL == 1 ? 0 : (L.lane & 3); }
  static DEVI float qred(float x) {
    if constexpr (QL == 4) return qsum(x);
    else return x;
  }
  static DEVI float qmaxf(float x) {
    if constexpr (QL == 4) {
      const float t = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false)));
      return fmaxf(t, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x4E, 0xF, 0xF, false)));
    } else {
      return x;
    }
  }
  static DEVI float qminf(float x) { return -qmaxf(-x); }

  // one pass over the subsystem's rows at a: its cost, J' f (dofs LO..HI-1), (WANT_H) the rows'
  // Hessian terms added to H (packed lower over the subsystem's dofs; zero on entry), and sig, a
  // signature of this lane's rows' zones (quadratic / linear / inactive): Newton has converged
  // once a full step leaves every lane's unchanged (the cost is one quadratic there)
  // The signature is exact (no two zone patterns collide): per lane at most ceil(LDS_CON / QL) LDS
  // contacts x 4 edges (1 bit each), ceil(4 (SIM_MAXCON - LDS_CON) / QL) overflow edges (1 bit),
  // NA frictionloss rows (3 zones: < 2 bits) and <= 2 NA limit rows (1 bit) -- 42 bits at QL 4,
  // in a 64-bit word (a 32-bit shift signature dropped the oldest rows' zones).
  static constexpr int SIG_BITS = 4 * ((LDS_CON + QL - 1) / QL) + (4 * (SIM_MAXCON - LDS_CON) + QL - 1) / QL +
                                  2 * NA + 2 * NA;
  static_assert(!CON || SIG_BITS <= 64, "zone signature must fit its 64-bit word");
  // C0: also the rows' cost at a0 (cost0; no derivatives there) in the same pass -- the warm
  // start's two points (qacc_smooth and the warm start) share one read of the rows
  template <int LO, int HI, bool WANT_H, bool C0 = false>
  DEVI float pass(const float a[NV], float jtf[NV], float H[], uint64_t& sig, const float* a0 = nullptr,
                  float* cost0 = nullptr) const {
    constexpr int NR = HI - LO, NH = NR * (NR + 1) / 2;
    float cost = 0.f, c0 = 0.f;
    sig = 0ull;
#pragma unroll
    for (int i = LO; i < HI; i++) jtf[i] = 0.f;
    if constexpr (CON) {
      bool mine = false;
      // one contact over the dof range [CL, CH) its Jacobian can be nonzero on
      auto contact = [&](int c, auto cl, auto ch) {
        constexpr int CL = decltype(cl)::value, CH = decltype(ch)::value;
        float jc[3][NV];
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = CL; i < CH; i++) jc[q][i] = L.at(c, 12 * q + i);
        const float mu = L.at(c, F_MU), D = L.at(c, F_IARD);
        float y[3] = {0.f, 0.f, 0.f}, y0[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = CL; i < CH; i++) {
            y[q] = fmaf(jc[q][i], a[i], y[q]);
            if constexpr (C0) y0[q] = fmaf(jc[q][i], a0[i], y0[q]);
          }
        float F[3] = {0.f, 0.f, 0.f}, K[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // K: nn n1 n2 11 12 22
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float s = (ed & 1) ? -mu : mu;
          const int t = 1 + (ed >> 1);
          const float x = y[0] + s * y[t] - L.at(c, F_AREF + ed);
          if constexpr (C0) {
            const float x0 = y0[0] + s * y0[t] - L.at(c, F_AREF + ed);
            c0 += x0 < 0.f ? 0.5f * x0 * x0 * D : 0.f;
          }
          const bool act = x < 0.f;
          sig = sig * 2ull + (act ? 1ull : 0ull);
          const float xa = act ? x : 0.f, Da = act ? D : 0.f;  // (branch-free)
          cost += 0.5f * xa * xa * D;
          const float f = -xa * D;
          F[0] += f, F[t] += s * f;
          K[0] += Da, K[t] += s * Da, K[t == 1 ? 3 : 5] += s * s * Da;
        }
#pragma unroll
        for (int i = CL; i < CH; i++) jtf[i] += jc[0][i] * F[0] + jc[1][i] * F[1] + jc[2][i] * F[2];
        if constexpr (WANT_H) {  // H += J_c' K J_c
          float kj[3][NV];
#pragma unroll
          for (int i = CL; i < CH; i++) {
            kj[0][i] = K[0] * jc[0][i] + K[1] * jc[1][i] + K[2] * jc[2][i];
            kj[1][i] = K[1] * jc[0][i] + K[3] * jc[1][i] + K[4] * jc[2][i];
            kj[2][i] = K[2] * jc[0][i] + K[4] * jc[1][i] + K[5] * jc[2][i];
          }
#pragma unroll
          for (int i = CL; i < CH; i++)
#pragma unroll
            for (int j = CL; j <= i; j++)
              H[hidx(i - LO, j - LO)] += jc[0][i] * kj[0][j] + jc[1][i] * kj[1][j] + jc[2][i] * kj[2][j];
        }
      };
      for (int c = ql(); has_contacts<LO, HI>() && c < nl; c += QL) {
        const int fl = (int)L.at(c, F_FLAGS);
        if constexpr (LO == 0 && HI == NV) {
          mine = true;
          // whole problem: still skip the halves a contact cannot touch (choice uniform over
          // the lanes still in the loop)
          if (NF > 0 && __all(fl == TOUCH_FREE))
            contact(c, std::integral_constant<int, NA>{}, std::integral_constant<int, NV>{});
          else if (__all(!(fl & TOUCH_FREE)))
            contact(c, std::integral_constant<int, 0>{}, std::integral_constant<int, NA>{});
          else
            contact(c, std::integral_constant<int, 0>{}, std::integral_constant<int, NV>{});
        } else if (owns<LO, HI>(fl)) {
          mine = true;
          contact(c, std::integral_constant<int, LO>{}, std::integral_constant<int, HI>{});
        }
      }
      if constexpr (LO == 0 && HI == NV) {
        // contacts past the LDS records: per-edge rows in the global slab (rare; whole problem)
        for (int r = 4 * nl + ql(); r < 4 * ncon; r += QL) {
          mine = true;
          float J[NV], x = -cr.S(r, 0), x0 = -cr.S(r, 0);
#pragma unroll
          for (int i = 0; i < NV; i++) {
            J[i] = cr.J(r, i), x = fmaf(J[i], a[i], x);
            if constexpr (C0) x0 = fmaf(J[i], a0[i], x0);
          }
          if constexpr (C0) c0 += x0 < 0.f ? 0.5f * x0 * x0 * cr.S(r, 2) : 0.f;
          sig = sig * 2ull + (x < 0.f ? 1ull : 0ull);
          if (x < 0.f) {
            const float D = cr.S(r, 2), f = -x * D;
            cost += 0.5f * x * x * D;
#pragma unroll
            for (int i = 0; i < NV; i++) jtf[i] += J[i] * f;
            if constexpr (WANT_H)
#pragma unroll
              for (int i = 0; i < NV; i++)
#pragma unroll
                for (int j = 0; j <= i; j++) H[hidx(i, j)] += D * J[i] * J[j];
          }
        }
      }
      // combine the quad's partial sums (skipped, wave-uniformly, when no lane has a row here:
      // every partial is then zero)
      if constexpr (QL > 1) {
        if (__any(mine)) {
          cost = qred(cost);
          if constexpr (C0) c0 = qred(c0);
#pragma unroll
          for (int i = LO; i < HI; i++) jtf[i] = qred(jtf[i]);
          if constexpr (WANT_H)
#pragma unroll
            for (int k = 0; k < NH; k++) H[k] = qred(H[k]);
        }
      }
    }
    if constexpr (LO == 0) {
      // frictionloss rows (J = e_i)
#pragma unroll
      for (int i = 0; i < NA; i++) {
        // (branch-free: the zone decides values, not control flow)
        const float fl = m.dof_frictionloss[i], R = fR[i], iR = fiR[i];
        const float x = a[i] - fa[i], Rfl = R * fl;
        const bool lin = fabsf(x) >= Rfl;  // linear zones x <= -R fl, x >= R fl (all of it when fl = 0)
        const bool q = !lin;               // (fl > 0 here)
        const float flx = x < 0.f ? fl : -fl;
        jtf[i] += lin ? flx : -x * iR;
        cost += lin ? fmaf(fl, fabsf(x), -0.5f * Rfl * fl) : 0.5f * x * x * iR;
        if constexpr (C0) {
          const float x0 = a0[i] - fa[i];
          c0 += fabsf(x0) >= Rfl ? fmaf(fl, fabsf(x0), -0.5f * Rfl * fl) : 0.5f * x0 * x0 * iR;
        }
        sig = sig * 3ull + (q ? 1ull : (x < 0.f ? 2ull : 0ull));
        if constexpr (WANT_H) H[hidx(i, i)] += q ? iR : 0.f;
      }
      // joint limits (J = sign e_dof)
      for (int l = 0; l < nlim; l++) {
        const int d = (int)L.lm(l, L_DOF);
        const float sg = L.lm(l, L_SGN), iR = L.lm(l, L_IARD);
        float ad = 0.f, ad0 = 0.f;
#pragma unroll
        for (int i = 0; i < NA; i++) {
          ad = i == d ? a[i] : ad;
          if constexpr (C0) ad0 = i == d ? a0[i] : ad0;
        }
        const float x = sg * ad - L.lm(l, L_AREF);
        if constexpr (C0) {
          const float x0 = sg * ad0 - L.lm(l, L_AREF);
          c0 += x0 < 0.f ? 0.5f * x0 * x0 * iR : 0.f;
        }
        sig = sig * 2ull + (x < 0.f ? 1ull : 0ull);
        if (x < 0.f) {
          cost += 0.5f * x * x * iR;
          const float f = -x * iR;
#pragma unroll
          for (int i = 0; i < NA; i++) {
            jtf[i] += i == d ? sg * f : 0.f;
            if constexpr (WANT_H) H[hidx(i, i)] += i == d ? iR : 0.f;
          }
        }
      }
    }
    if constexpr (C0) *cost0 = c0;
    return cost;
  }

  // line-search data along p: per contact edge its residual at a, its rate along p and the step
  // length where it changes zone (a kink of the line cost), in LDS scratch (ext area, 12 floats
  // per contact; written and read by the lane that owns the contact)
  static constexpr int LS_STRIDE = 12;
  static_assert(XS_LIST + LS_STRIDE * LDS_CON <= XS_EXT, "line-search scratch fits the ext area");
  // per frictionloss row along p (registers): residual at a, the step lengths of its two kinks
  // (x = -R fl, x = R fl; +inf when p_i = 0 or fl = 0) and p_i / R_i
  struct FricLS {
    float x0[NA], k1[NA], k2[NA], piR[NA];
  };
  template <int LO, int HI>
  DEVI void ls_setup(const float a[NV], const float p[NV], FricLS& fr) const {
    if constexpr (LO == 0) {
#pragma unroll
      for (int i = 0; i < NA; i++) {
        const float fl = m.dof_frictionloss[i], R = fR[i], x0 = a[i] - fa[i];
        const bool live = fl > 0.f && p[i] != 0.f;
        const float rp = __builtin_amdgcn_rcpf(p[i]);  // (kinks to ~1 ulp: see ls_eval)
        fr.x0[i] = x0;
        fr.k1[i] = live ? (-R * fl - x0) * rp : 3.0e38f;
        fr.k2[i] = live ? (R * fl - x0) * rp : 3.0e38f;
        fr.piR[i] = p[i] * fiR[i];
      }
    } else {
      (void)fr;
    }
    if constexpr (CON) {
      for (int c = ql(); has_contacts<LO, HI>() && c < nl; c += QL) {
        if (!owns<LO, HI>((int)L.at(c, F_FLAGS))) continue;
        float ya[3] = {0.f, 0.f, 0.f}, yp[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = LO; i < HI; i++) {
            const float j = L.at(c, 12 * q + i);
            ya[q] = fmaf(j, a[i], ya[q]), yp[q] = fmaf(j, p[i], yp[q]);
          }
        const float mu = L.at(c, F_MU);
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float s = (ed & 1) ? -mu : mu;
          const int t = 1 + (ed >> 1);
          const float x0 = ya[0] + s * ya[t] - L.at(c, F_AREF + ed), v = yp[0] + s * yp[t];
          L.ex(XS_LIST + LS_STRIDE * c + ed) = x0;
          L.ex(XS_LIST + LS_STRIDE * c + 4 + ed) = v;
          L.ex(XS_LIST + LS_STRIDE * c + 8 + ed) = v != 0.f ? -x0 * __builtin_amdgcn_rcpf(v) : 3.0e38f;
        }
      }
      if constexpr (LO == 0 && HI == NV)
        for (int r = 4 * nl + ql(); r < 4 * ncon; r += QL) {
          float x = -cr.S(r, 0), v = 0.f;
#pragma unroll
          for (int i = 0; i < NV; i++) x = fmaf(cr.J(r, i), a[i], x), v = fmaf(cr.J(r, i), p[i], v);
          cr.W(r, 0) = x, cr.W(r, 1) = v;  // (the PGS M^-1 J' slot: unused by Newton)
        }
    }
  }

  // d/dalpha and d2/dalpha2 of the subsystem rows' cost at a + alpha p added to d1, d2 (Gauss
  // part: caller), and the piece [bl, br] of the piecewise-quadratic line cost that alpha lies in
  // (the nearest kinks at or below / above alpha): d/dalpha is linear there
  template <int LO, int HI>
  DEVI void ls_eval(const float a[NV], const float p[NV], const FricLS& fr, float al, float& d1, float& d2,
                    float& bl, float& br) const {
    auto kink = [&](float t, float& l, float& r) {
      r = t > al ? fminf(r, t) : r;
      l = t <= al ? fmaxf(l, t) : l;
    };
    if constexpr (CON) {
      float c1 = 0.f, c2 = 0.f, cl = -3.0e38f, cr_ = 3.0e38f;
      bool mine = false;
      for (int c = ql(); has_contacts<LO, HI>() && c < nl; c += QL) {
        if (!owns<LO, HI>((int)L.at(c, F_FLAGS))) continue;
        mine = true;
        const float D = L.at(c, F_IARD);
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          const float v = L.ex(XS_LIST + LS_STRIDE * c + 4 + ed);
          const float x = fmaf(al, v, L.ex(XS_LIST + LS_STRIDE * c + ed));
          if (x < 0.f) c1 += x * v * D, c2 += v * v * D;
          kink(L.ex(XS_LIST + LS_STRIDE * c + 8 + ed), cl, cr_);
        }
      }
      if constexpr (LO == 0 && HI == NV)
        for (int r = 4 * nl + ql(); r < 4 * ncon; r += QL) {
          mine = true;
          const float D = cr.S(r, 2), v = cr.W(r, 1), x0 = cr.W(r, 0);
          const float x = fmaf(al, v, x0);
          if (x < 0.f) c1 += x * v * D, c2 += v * v * D;
          if (v != 0.f) kink(-x0 * __builtin_amdgcn_rcpf(v), cl, cr_);
        }
      if constexpr (QL > 1) {
        if (__any(mine)) c1 = qred(c1), c2 = qred(c2), cl = qmaxf(cl), cr_ = qminf(cr_);
      }
      d1 += c1, d2 += c2, bl = fmaxf(bl, cl), br = fminf(br, cr_);
    }
    if constexpr (LO == 0) {
      // frictionloss rows: d/dalpha of the Huber cost is x p / R inside |x| < R fl, +-fl p outside
#pragma unroll
      for (int i = 0; i < NA; i++) {
        const float fl = m.dof_frictionloss[i], x = fmaf(al, p[i], fr.x0[i]);
        const bool in = fabsf(x) < fR[i] * fl;
        const float flp = fl * p[i];
        d1 += in ? x * fr.piR[i] : (x < 0.f ? -flp : flp);
        d2 += in ? p[i] * fr.piR[i] : 0.f;
        kink(fr.k1[i], bl, br);
        kink(fr.k2[i], bl, br);
      }
      for (int l = 0; l < nlim; l++) {
        const int d = (int)L.lm(l, L_DOF);
        const float sg = L.lm(l, L_SGN), iR = L.lm(l, L_IARD);
        float ad = 0.f, pd = 0.f;
#pragma unroll
        for (int i = 0; i < NA; i++) ad = i == d ? a[i] : ad, pd = i == d ? p[i] : pd;
        const float x0 = sg * ad - L.lm(l, L_AREF), v = sg * pd, x = fmaf(al, v, x0);
        if (x < 0.f) d1 += x * v * iR, d2 += v * v * iR;
        if (v != 0.f) kink(-x0 * __builtin_amdgcn_rcpf(v), bl, br);
      }
    }
  }
};

// y = M x over dofs [LO, HI) of the block-diagonal M (arm block packed lower, the free body's
// diagonal block); [LO, HI) is a union of whole blocks
template <int LO, int HI, int NA, int NF>
DEVI void mul_m(const Sim<NA, NF>& S, const float x[], float y[]) {
  if constexpr (LO < NA) {
#pragma unroll
    for (int i = 0; i < NA; i++) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NA; k++) s = fmaf(S.MA[i >= k ? i * (i + 1) / 2 + k : k * (k + 1) / 2 + i], x[k], s);
      y[i] = s;
    }
  }
  if constexpr (HI > NA) {
#pragma unroll
    for (int i = 0; i < 6 * NF; i++) y[NA + i] = S.MF[i / 6][(i % 6) * (i % 6 + 1) / 2 + i % 6] * x[NA + i];
  }
}

// Newton on the subsystem over dofs [LO, HI): a[] (all dofs; only this range moves) in/out,
// jtf[LO..HI) = J' f at the result.  Returns the iteration count.
template <int LO, int HI, int NA, int NF, bool CON>
DEVI int newton_range(const Sim<NA, NF>& S, const NewtonRows<NA, NF, CON>& R, float a[], float jtf[], int& nls,
                      long long* ncyc) {
#ifdef SOARM_PHASE_PROF
  long long nt_ = clock64();
#else
  (void)ncyc;
#endif
  constexpr int NV = NA + 6 * NF, NR = HI - LO, NH = NR * (NR + 1) / 2;
  const DModel& m = *S.mp;
  const float scale = m.pgs_scale, tol = m.tolerance;
  const float* a0 = S.qacc_s;
  auto gauss = [&](const float x[], float Mx[]) {  // 1/2 (x - a0)' M (x - a0) on the range; Mx = M (x - a0)
    float dx[NV];
#pragma unroll
    for (int i = LO; i < HI; i++) dx[i] = x[i] - a0[i];
    mul_m<LO, HI>(S, dx, Mx);
    float c = 0.f;
#pragma unroll
    for (int i = LO; i < HI; i++) c = fmaf(0.5f * dx[i], Mx[i], c);
    return c;
  };
  float H[NH], Ma[NV];
  uint64_t sig = 0ull;
  // warm start: qacc_warmstart unless qacc_smooth costs less (on this subsystem's cost); the
  // Hessian pass runs at the warm point, and again at qacc_smooth only in lanes where it wins
  float cost;
  {
    // (one pass over the rows for both points: the cost at qacc_smooth (its Gauss term is 0) and
    // cost, gradient and Hessian at the warm start)
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] = (i >= LO && i < HI) ? S.warm[i] : a[i];
#pragma unroll
    for (int i = 0; i < NH; i++) H[i] = 0.f;
    float cs;
    cost = gauss(a, Ma) + R.template pass<LO, HI, true, true>(a, jtf, H, sig, a0, &cs);
    if (cs < cost) {
#pragma unroll
      for (int i = LO; i < HI; i++) a[i] = a0[i], Ma[i] = 0.f;
#pragma unroll
      for (int i = 0; i < NH; i++) H[i] = 0.f;
      cost = R.template pass<LO, HI, true>(a, jtf, H, sig);
    }
  }
  NT_STAMP(0);
  // Zone prediction (the arm's own range, or a scene without a free body): the frictionloss rows of
  // a servo holding position chatter with period 2 -- their zones at the optimum repeat those of
  // two substeps back far more often (71-89% on the headline workload) than they match the zones
  // at the warm start (62%), so the first iteration may take its gradient and Hessian terms of
  // those rows from S.zpred.  The true cost, its gradient and the exact line search are unchanged:
  // the step is used only if it descends, and a step that lands where the true zones equal the
  // predicted ones with al = 1 is the optimum (the quadratic of those zones is minimised there).
  constexpr bool ZP = LO == 0 && HI == NA;
  bool force = false;
  if constexpr (ZP) force = (S.zpred >> 31) != 0u;
  int it = 0;
  for (; it < m.iterations; it++) {
    float g[NV], gn = 0.f;
#pragma unroll
    for (int i = LO; i < HI; i++) g[i] = Ma[i] - jtf[i], gn = fmaf(g[i], g[i], gn);
    if (scale * sqrtf(gn) < tol) break;
    // H = M + rows' terms (relative dof indices); p = -H^-1 g
    if constexpr (LO < NA) {
#pragma unroll
      for (int i = 0; i < NA; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) H[(i - LO) * (i - LO + 1) / 2 + j - LO] += S.MA[i * (i + 1) / 2 + j];
    }
    if constexpr (HI > NA) {
#pragma unroll
      for (int i = NA; i < NV; i++)
        H[(i - LO) * (i - LO + 1) / 2 + i - LO] += S.MF[(i - NA) / 6][((i - NA) % 6) * ((i - NA) % 6 + 1) / 2 + (i - NA) % 6];
    }
    float Hd[NR], pr[NR], mg[NR], p[NV];
    uint64_t sigf = sig;  // the zone signature the step's quadratic belongs to
    if constexpr (ZP) {
      if (force) {
        // predicted zones of the frictionloss rows: g and H's diagonal terms of those rows swapped
        // for the predicted zone's (J = e_i); the signature's frictionloss digits likewise
        float Hc[NH];
#pragma unroll
        for (int k = 0; k < NH; k++) Hc[k] = H[k];
        uint64_t fa_ = 0ull, fp_ = 0ull;
#pragma unroll
        for (int i = 0; i < NA; i++) {
          const float fl = m.dof_frictionloss[i], Rr = R.fR[i], iR = R.fiR[i];
          const float x = a[i] - R.fa[i];
          const bool lin = fabsf(x) >= Rr * fl;
          const uint32_t ca = lin ? (x < 0.f ? 2u : 0u) : 1u, cp = (S.zpred >> (2 * i)) & 3u;
          const float ja = ca == 1u ? -x * iR : (ca == 2u ? fl : -fl);
          const float jp = cp == 1u ? -x * iR : (cp == 2u ? fl : -fl);
          mg[i] = -(g[i] + ja - jp);
          H[i * (i + 1) / 2 + i] += (cp == 1u ? iR : 0.f) - (ca == 1u ? iR : 0.f);
          fa_ = fa_ * 3ull + ca, fp_ = fp_ * 3ull + cp;
        }
        sigf = sig + ((fp_ - fa_) << R.nlim);
        ldl_factor<NR>(H, Hd);
        ldl_solve<NR>(H, Hd, pr, mg);
        float dzf = 0.f;
#pragma unroll
        for (int i = 0; i < NR; i++) dzf = fmaf(g[i], pr[i], dzf);
        if (!(dzf < 0.f)) {  // not a descent direction of the true cost: the plain Newton step
#pragma unroll
          for (int k = 0; k < NH; k++) H[k] = Hc[k];
          force = false;
          sigf = sig;
        }
      }
    }
    if (!force) {
#pragma unroll
      for (int i = 0; i < NR; i++) mg[i] = -g[LO + i];
      ldl_factor<NR>(H, Hd);
      ldl_solve<NR>(H, Hd, pr, mg);
    }
    force = false;  // (first iteration only)
#pragma unroll
    for (int i = 0; i < NV; i++) p[i] = (i >= LO && i < HI) ? pr[i - LO] : 0.f;
    // exact line search: phi'(al) = (a - a0)' M p + al p' M p + rows, continuous and piecewise
    // linear in al.  From al = 1 (the Newton step): evaluate phi', phi'' and the piece around al;
    // the 1-D Newton target is the exact minimiser when it lies in that piece (usually the first
    // evaluation), else it moves the bracket and the next point is that target, or the secant
    // of the bracket when the target leaves it.  phi'(0) = g'p needs no evaluation.
    NT_STAMP(1);
    float Mp[NV], g0 = 0.f, pMp = 0.f, dz = 0.f;
    mul_m<LO, HI>(S, p, Mp);
#pragma unroll
    for (int i = LO; i < HI; i++) {
      g0 = fmaf(a[i] - a0[i], Mp[i], g0);
      pMp = fmaf(p[i], Mp[i], pMp);
      dz = fmaf(g[i], p[i], dz);
    }
    if (!(dz < 0.f)) break;  // not a descent direction at fp32 resolution: converged
    typename NewtonRows<NA, NF, CON>::FricLS fr;
    R.template ls_setup<LO, HI>(a, p, fr);
    float lo = 0.f, dlo = dz, hi = 3.0e38f, dhi = 0.f, al = 1.f;
    for (int ls = 0; ls < 24; ls++) {
      nls++;
      float d1 = fmaf(al, pMp, g0), d2 = pMp, bl = -3.0e38f, br = 3.0e38f;
      R.template ls_eval<LO, HI>(a, p, fr, al, d1, d2, bl, br);
      // (the target within its piece is exact up to rounding: the approximate reciprocal suffices)
      float an = al - d1 * __builtin_amdgcn_rcpf(d2);
      if (an >= bl && an <= br) {
        al = an;
        break;
      }
      if (d1 < 0.f)
        lo = al, dlo = d1;
      else
        hi = al, dhi = d1;
      if (!(an > lo && an < hi)) an = lo + (hi - lo) * (dlo / (dlo - dhi));
      if (!(an > lo && an < hi)) break;  // bracket exhausted at fp32 resolution
      al = an;
    }
    NT_STAMP(2);
    float an_[NV], jn[NV], Man[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) an_[i] = fmaf(al, p[i], a[i]);
#pragma unroll
    for (int i = 0; i < NH; i++) H[i] = 0.f;
    const uint64_t sig0 = sigf;
    const float cn = gauss(an_, Man) + R.template pass<LO, HI, true>(an_, jn, H, sig);
    NT_STAMP(3);
    if (!(cn <= cost + 1e-5f * fabsf(cost))) break;  // a real increase (numerical trouble): keep a
#pragma unroll
    for (int i = LO; i < HI; i++) a[i] = an_[i], jtf[i] = jn[i], Ma[i] = Man[i];
    cost = cn;
    // MuJoCo's stopping test on the cost improvement, with the improvement taken from the
    // quadratic model along p, -al phi'(0) / 2, instead of the difference of two costs: in fp32
    // that difference is rounding noise (~1e-7 of a cost of order 1) long before the light
    // rotational dofs of the cube (inertia 4.5e-6) have converged.  And exactness: a full
    // Newton step that leaves every row in its zone has minimised the one quadratic there.
    bool same = sig == sig0;  // every lane of the env: its rows kept their zones
    if constexpr (NewtonRows<NA, NF, CON>::QL > 1) same = qsum(same ? 0.f : 1.f) == 0.f;
    if (scale * (-0.5f * al * dz) < tol || (same && fabsf(al - 1.f) < 1e-3f)) {
      it++;
      break;
    }
  }
  return it;
}

// Primal Newton solve of the rows built by solve_constraints; sets S.qacc and S.fcon = J' f.
// Returns the iteration count (both subsystems').
template <int NA, int NF, bool CON>
DEVI int newton_solve(Sim<NA, NF>& S, const NewtonRows<NA, NF, CON>& R) {
  constexpr int NV = NA + 6 * NF;
  float a[NV], jtf[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) a[i] = S.qacc_s[i], jtf[i] = 0.f;
  // an arm-cube contact (or a generic overflow row) in any lane of the wave couples the blocks
  // (wave-uniform: every lane takes part in every vote)
  bool coupled = false;
  if constexpr (NF > 0 && CON) {
    coupled = __any(R.ncon > R.nl);
#pragma unroll
    for (int c = 0; c < LDS_CON; c++)
      coupled |= __any(c < R.nl && (int)R.L.at(c < R.nl ? c : 0, F_FLAGS) == (TOUCH_ARM | TOUCH_FREE));
  }
  NewtonRows<NA, NF, CON> Rs = R;  // (+ the per-subsystem contact flags)
  if constexpr (NF > 0 && CON) {
    bool arm = false, fre = false;
#pragma unroll
    for (int c = 0; c < LDS_CON; c++) {
      const int fl = c < R.nl ? (int)R.L.at(c, F_FLAGS) : 0;
      arm |= __any(c < R.nl && !(fl & TOUCH_FREE));
      fre |= __any(c < R.nl && fl == TOUCH_FREE);
    }
    Rs.arm_c = arm, Rs.free_c = fre;
  }
  int it, nls = 0;
  long long ncyc[4] = {0, 0, 0, 0};
#ifdef SOARM_PHASE_PROF
  const long long t0 = clock64();
  int it_arm = 0, nls_arm = 0;
#endif
  if constexpr (NF == 0) {
    it = newton_range<0, NV>(S, R, a, jtf, nls, ncyc);
  } else {
    if (coupled) {
      it = newton_range<0, NV>(S, R, a, jtf, nls, ncyc);
    } else {
      it = newton_range<0, NA>(S, Rs, a, jtf, nls, ncyc);
#ifdef SOARM_PHASE_PROF
      it_arm = it, nls_arm = nls;
#endif
      it += newton_range<NA, NV>(S, Rs, a, jtf, nls, ncyc);
    }
  }
  {  // the frictionloss rows' zones at the result (the caller's history for the next prediction)
    uint32_t z = 1u << 31;
#pragma unroll
    for (int i = 0; i < NA; i++) {
      const float x = a[i] - R.fa[i];
      const bool lin = fabsf(x) >= R.fR[i] * S.mp->dof_frictionloss[i];
      z |= (lin ? (x < 0.f ? 2u : 0u) : 1u) << (2 * i);
    }
    S.zfin = z;
  }
#ifdef SOARM_PHASE_PROF
  {
    // reduced over the wave first (one lane per env counts), then one atomic per counter and
    // wave: per-env atomics on shared counters serialise in L2 and stall the waves being measured
    const long long dt = clock64() - t0;
    const bool one = (threadIdx.x & (lpe<NF>() - 1)) == 0;
    auto wsum = [](double v) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
      return v;
    };
    const double sv[16] = {1.0, (double)it, (double)nls, (double)coupled, (double)dt, (double)it_arm,
                           (double)nls_arm, (double)(it - it_arm), (double)(nls - nls_arm),
                           (double)ncyc[0], (double)ncyc[1], (double)ncyc[2], (double)ncyc[3], 0.0, 0.0, 0.0};
    const int sk[13] = {0, 1, 2, 3, 4, 8, 9, 10, 11, 16, 17, 18, 19};
    for (int k = 0; k < 13; k++) {
      const double w = wsum(one ? sv[k] : 0.0);
      if ((threadIdx.x & 63) == 0) atomicAdd(&g_newton[sk[k]], (unsigned long long)w);
    }
    const int mx[4] = {wave_max_i((int)dt), wave_max_i(it), wave_max_i(nls), 0};
    const int wc[4] = {wave_max_i((int)ncyc[0]), wave_max_i((int)ncyc[1]), wave_max_i((int)ncyc[2]),
                       wave_max_i((int)ncyc[3])};
    if ((threadIdx.x & 63) == 0) {
      atomicMax(&g_newton[5], (unsigned long long)mx[0]);
      atomicMax(&g_newton[6], (unsigned long long)mx[1]);
      atomicMax(&g_newton[7], (unsigned long long)mx[2]);
      atomicAdd(&g_newton[12], 1ull);
      atomicAdd(&g_newton[13], (unsigned long long)mx[2]);
      atomicAdd(&g_newton[14], (unsigned long long)mx[1]);
      atomicAdd(&g_newton[15], (unsigned long long)mx[0]);
      for (int k = 0; k < 4; k++) atomicAdd(&g_newton[20 + k], (unsigned long long)wc[k]);
    }
  }
#endif
#pragma unroll
  for (int i = 0; i < NV; i++) S.qacc[i] = a[i], S.fcon[i] = jtf[i];
  return it;
}

}  // namespace soarm
