// soarm_cpu.hip — the CPU backend behind the same C ABI (`sim_batch_create(..., device = -1,
// ...)`; SURVEY.md §8(b) "CPU backend uses the same ABI with device = -1", "Threading: CPU
// backend: OpenMP over envs").  Built host-only (--offload-host-only) into libsoarm_sim.so.
//
// Per env it runs the kernels' own per-env code, compiled for the host (HDI functions of
// soarm_step.h / soarm_collide.h / soarm_env.h): kinematics, CRBA + LDL', RNE + passive +
// actuation, geom poses, the candidate-pair midphase and narrowphase (box-box, plane-*,
// MPR or native GJK/EPA, with the separating-axis cache), implicit-damping Euler, resets,
// observations, bias forces and DLS IK.  What differs is the constraint solve: the device
// kernels' solvers are lane-cooperative (quad / 16-lane PGS sweeps, split Newton), so here
// the rows are built densely in MuJoCo's order (dof frictionloss, joint limits lower/upper,
// contacts x 4 pyramid edges; mj_makeConstraint) and solved by a scalar fp32 restatement of
// mj_solPGS (Gauss-Seidel in row order, the scaled-improvement stop) or mj_solNewton (primal
// Newton, exact line search), the model's `solver`.  Envs are split over host threads
// (SOARM_CPU_THREADS, else OMP_NUM_THREADS, else all cores); every env is independent, so the
// result does not depend on the thread count.
//
// All buffers are caller-owned host memory in the same layouts as the device path ([field][env]
// SoA state, [env][k] obs/actions); calls are synchronous.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "sim_internal.h"
#include "soarm_collide.h"
#include "soarm_env.h"

using namespace soarm;

struct CpuBatch {
  const sim_model* model = nullptr;
  int n = 0;
  DModel dm;                 // the model with host hull pointers
  std::vector<float> sepax;  // separating-axis cache [pair*3+k][env] (soarm_collide.h SepCache)
};

namespace {

int cpu_threads(int n) {
  int t = 0;
  for (const char* v : {"SOARM_CPU_THREADS", "OMP_NUM_THREADS"})
    if (!t)
      if (const char* s = getenv(v)) t = atoi(s);
  if (t <= 0) t = (int)std::max(1u, std::thread::hardware_concurrency());
  return std::max(1, std::min(t, n));
}

// f(e) for e in [0, n), contiguous chunks over the threads (this thread takes the first)
template <class F>
void parallel_envs(int n, F&& f) {
  const int t = cpu_threads(n);
  auto run = [&](int k) {
    const int e0 = (int)((long long)n * k / t), e1 = (int)((long long)n * (k + 1) / t);
    for (int e = e0; e < e1; e++) f(e);
  };
  std::vector<std::thread> pool;
  pool.reserve(t - 1);
  for (int k = 1; k < t; k++) pool.emplace_back(run, k);
  run(0);
  for (auto& th : pool) th.join();
}

template <class F>
void dispatch_nf(int nf, F&& f) {
  if (nf == 0)
    f(std::integral_constant<int, 0>{});
  else
    f(std::integral_constant<int, 1>{});
}

// one env's contacts at the current geom poses: collide every candidate pair (pair order,
// each pair's contacts in slot order), at most SIM_MAXCON kept
struct CpuContact {
  float dist, pos[3], n[3];
  int pair;
};

template <int NA, int NF>
int collide_env(const CpuBatch& B, Sim<NA, NF>& S, int e, CpuContact* con, int& status) {
  const DModel& m = B.dm;
  float gpose[SIM_MAXBODY * BREC];
  float cbuf[PAIR_MAXCON * 7];
  write_body_frames(S, gpose, 1, 0, 0, 1);
  float* sep = const_cast<float*>(B.sepax.data());
  int nc = 0;
  for (int p = 0; p < m.npair; p++) {
    PairOut o{cbuf, 1, 0, 0, m.pair_cap[p], 0};  // the pair's slots, re-based to this scratch
    collide_pair(m, p, gpose, 1, 0, o, SepCache{sep, B.n, e});
    for (int k = 0; k < o.n; k++) {
      if (nc >= SIM_MAXCON) {
        status |= SIM_ST_CONOVERFLOW;
        break;
      }
      CpuContact& c = con[nc++];
      c.dist = cbuf[7 * k];
      for (int q = 0; q < 3; q++) c.pos[q] = cbuf[7 * k + 1 + q], c.n[q] = cbuf[7 * k + 4 + q];
      c.pair = p;
    }
  }
  return nc;
}

// ------------------------------------------------------------------ constraint rows
enum { ROW_FRICTION = 0, ROW_LIMIT = 1, ROW_CONTACT = 2 };

template <int NA, int NF>
struct Rows {
  static constexpr int NV = NA + 6 * NF;
  static constexpr int MAXR = NV + 2 * NA + 4 * SIM_MAXCON;
  int nr = 0;
  int type[MAXR];
  float J[MAXR][NV], aref[MAXR], R[MAXR], fl[MAXR];
};

// mj_makeConstraint in MuJoCo's row order, from the same model constants as the kernels
// (soarm_pgs.h solve_constraints: dof_fricR/B, jnt_KB, pair_KB / tran / solimp / margin)
template <int NA, int NF>
void make_rows(const Sim<NA, NF>& S, const CpuContact* con, int ncon, Rows<NA, NF>& X) {
  constexpr int NV = Sim<NA, NF>::NV;
  const DModel& m = *S.mp;
  int r = 0;
  for (int i = 0; i < NV; i++) {  // dof frictionloss
    if (!(m.dof_frictionloss[i] > 0.f)) continue;
    for (int k = 0; k < NV; k++) X.J[r][k] = k == i ? 1.f : 0.f;
    X.type[r] = ROW_FRICTION;
    X.aref[r] = -m.dof_fricB[i] * S.qvel[i];
    X.R[r] = m.dof_fricR[i];
    X.fl[r] = m.dof_frictionloss[i];
    r++;
  }
  for (int i = 0; i < NA; i++) {  // joint limits, lower then upper
    if (!m.jnt_limited[i]) continue;
    for (int side = 0; side < 2; side++) {
      const float dist = side == 0 ? S.qpos[i] - m.jnt_range[i][0] : m.jnt_range[i][1] - S.qpos[i];
      if (!(dist < m.jnt_margin[i])) continue;
      const float sg = side == 0 ? 1.f : -1.f;
      const float imp = impedance(m.jnt_solimp[i], dist, m.jnt_margin[i]);
      for (int k = 0; k < NV; k++) X.J[r][k] = k == i ? sg : 0.f;
      X.type[r] = ROW_LIMIT;
      X.aref[r] = -m.jnt_KB[i][1] * (sg * S.qvel[i]) - m.jnt_KB[i][0] * imp * (dist - m.jnt_margin[i]);
      X.R[r] = fmaxf(MINVALF, (1.f - imp) * m.dof_invweight0[i] / imp);
      X.fl[r] = 0.f;
      r++;
    }
  }
  for (int c = 0; c < ncon; c++) {  // contacts: 4 pyramid edges each (condim 3)
    const CpuContact& cc = con[c];
    const int p = cc.pair, b1 = m.pair_body1[p], b2 = m.pair_body2[p];
    const float mu = S.fric >= 0.f ? S.fric : m.pair_friction[p];
    float fr[9] = {cc.n[0], cc.n[1], cc.n[2], 0, 0, 0, 0, 0, 0};
    {  // contact frame (mju_makeFrame)
      float y[3];
      if (fabsf(fr[1]) < 0.5f)
        y[0] = 0, y[1] = 1, y[2] = 0;
      else
        y[0] = 0, y[1] = 0, y[2] = 1;
      const float dd = dot3(fr, y);
      y[0] -= dd * fr[0], y[1] -= dd * fr[1], y[2] -= dd * fr[2];
      const float inv = 1.f / sqrtf(dot3(y, y));
      fr[3] = y[0] * inv, fr[4] = y[1] * inv, fr[5] = y[2] * inv;
      cross(fr + 6, fr, fr + 3);
    }
    // relative translational Jacobian (body2 - body1) at the contact point, contact frame
    float jd[3][NV] = {};
    for (int side = 0; side < 2; side++) {
      const int b = side ? b2 : b1;
      const float sg = side ? 1.f : -1.f;
      for (int i = 0; i < NA; i++)
        if (b >= i + 2 && b < 2 + NA) {  // hinge i moves chain bodies i+2.. (reference point: origin)
          float l[3];
          cross(l, S.cdof[i], cc.pos);
          const float jp[3] = {S.cdof[i][3] + l[0], S.cdof[i][4] + l[1], S.cdof[i][5] + l[2]};
          for (int q = 0; q < 3; q++) jd[q][i] += sg * dot3(fr + 3 * q, jp);
        }
      for (int f = 0; f < NF; f++) {
        const int fb = 2 + NA + f, d0 = NA + 6 * f;
        if (b != fb) continue;
        const float off[3] = {cc.pos[0] - S.xpos[fb][0], cc.pos[1] - S.xpos[fb][1], cc.pos[2] - S.xpos[fb][2]};
        for (int i = 0; i < 6; i++) {
          float l[3];
          cross(l, S.cdof[d0 + i], off);
          const float jp[3] = {S.cdof[d0 + i][3] + l[0], S.cdof[d0 + i][4] + l[1], S.cdof[d0 + i][5] + l[2]};
          for (int q = 0; q < 3; q++) jd[q][d0 + i] += sg * dot3(fr + 3 * q, jp);
        }
      }
    }
    const float imp = impedance(m.pair_solimp[p], cc.dist, m.pair_margin[p]);
    const float tran = m.pair_tran[p];
    const float R0 = fmaxf(MINVALF, (1.f - imp) * (tran + mu * mu * tran) / imp);
    const float Rpy = 2.f * mu * mu * R0 / m.impratio;
    for (int ed = 0; ed < 4; ed++) {
      const float s = (ed & 1) ? -mu : mu;
      const float* jt = jd[1 + (ed >> 1)];
      float vel = 0.f;
      for (int k = 0; k < NV; k++) {
        X.J[r][k] = jd[0][k] + s * jt[k];
        vel += X.J[r][k] * S.qvel[k];
      }
      X.type[r] = ROW_CONTACT;
      X.aref[r] = -m.pair_KB[p][1] * vel - m.pair_KB[p][0] * imp * (cc.dist - m.pair_margin[p]);
      X.R[r] = Rpy;
      X.fl[r] = 0.f;
      r++;
    }
  }
  X.nr = r;
}

// M x with the block-diagonal packed M of Sim (arm NA x NA | one 6x6 per free body)
template <int NA, int NF>
void mul_m(const Sim<NA, NF>& S, const float* x, float* y) {
  for (int i = 0; i < NA; i++) {
    float s = 0.f;
    for (int k = 0; k < NA; k++) s += S.MA[i >= k ? i * (i + 1) / 2 + k : k * (k + 1) / 2 + i] * x[k];
    y[i] = s;
  }
  for (int f = 0; f < NF; f++) {
    const int d0 = NA + 6 * f;
    for (int i = 0; i < 6; i++) {
      float s = 0.f;
      for (int k = 0; k < 6; k++) s += S.MF[f][i >= k ? i * (i + 1) / 2 + k : k * (k + 1) / 2 + i] * x[d0 + k];
      y[d0 + i] = s;
    }
  }
}

// ------------------------------------------------------------------ mj_solPGS
template <int NA, int NF>
void solve_pgs(Sim<NA, NF>& S, const Rows<NA, NF>& X) {
  constexpr int NV = Sim<NA, NF>::NV, MAXR = Rows<NA, NF>::MAXR;
  const DModel& m = *S.mp;
  const int nr = X.nr;
  float W[MAXR][NV], ARd[MAXR], f[MAXR], v[NV];
  for (int r = 0; r < nr; r++) {
    S.solve_m(W[r], X.J[r]);
    float s = 0.f;
    for (int i = 0; i < NV; i++) s += X.J[r][i] * W[r][i];
    ARd[r] = s + X.R[r];
  }
  // warm start: the forces implied by qacc_warmstart, kept if their dual cost beats f = 0
  for (int r = 0; r < nr; r++) {
    float jar = -X.aref[r];
    for (int i = 0; i < NV; i++) jar += X.J[r][i] * S.warm[i];
    if (X.type[r] == ROW_FRICTION) {
      const float fl = X.fl[r];
      f[r] = jar <= -fl * X.R[r] ? fl : jar >= fl * X.R[r] ? -fl : -jar / X.R[r];
    } else {
      f[r] = jar < 0.f ? -jar / X.R[r] : 0.f;
    }
  }
  for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
  for (int r = 0; r < nr; r++)
    for (int i = 0; i < NV; i++) v[i] += W[r][i] * f[r];
  float cost = 0.f;
  for (int r = 0; r < nr; r++) {
    float jv = 0.f, jq = 0.f;
    for (int i = 0; i < NV; i++) jv += X.J[r][i] * v[i], jq += X.J[r][i] * S.qacc_s[i];
    cost += 0.5f * f[r] * (jv - X.aref[r] + X.R[r] * f[r]) + 0.5f * f[r] * (jq - X.aref[r]);
  }
  if (cost > 0.f) {
    for (int r = 0; r < nr; r++) f[r] = 0.f;
    for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
  }
  // Gauss-Seidel sweeps in row order; stop when the sweep's improvement, scaled by
  // 1 / (meaninertia * max(1, nv)), is below the tolerance
  for (int it = 0; it < m.iterations; it++) {
    float improvement = 0.f;
    for (int r = 0; r < nr; r++) {
      float res = -X.aref[r] + X.R[r] * f[r];
      for (int i = 0; i < NV; i++) res += X.J[r][i] * v[i];
      float fn = f[r] - res / ARd[r];
      fn = X.type[r] == ROW_FRICTION ? fminf(fmaxf(fn, -X.fl[r]), X.fl[r]) : fmaxf(fn, 0.f);
      const float df = fn - f[r];
      if (df != 0.f) {
        for (int i = 0; i < NV; i++) v[i] += W[r][i] * df;
        f[r] = fn;
        improvement -= df * (res + 0.5f * ARd[r] * df);
      }
    }
    if (improvement * m.pgs_scale < m.tolerance) break;
  }
  for (int i = 0; i < NV; i++) {
    S.qacc[i] = v[i];
    float s = 0.f;
    for (int r = 0; r < nr; r++) s += X.J[r][i] * f[r];
    S.fcon[i] = s;
  }
}

// ------------------------------------------------------------------ mj_solNewton
// row r at x = J_r a - aref_r: force -s_r'(x) and whether the row is in its quadratic zone
template <int NA, int NF>
float row_force(const Rows<NA, NF>& X, int r, float x, bool& quad) {
  const float R = X.R[r];
  if (X.type[r] == ROW_FRICTION) {
    const float fl = X.fl[r];
    quad = x > -R * fl && x < R * fl;
    return x <= -R * fl ? fl : x >= R * fl ? -fl : -x / R;
  }
  quad = x < 0.f;
  return quad ? -x / R : 0.f;
}
template <int NA, int NF>
float row_cost(const Rows<NA, NF>& X, int r, float x) {
  const float R = X.R[r];
  if (X.type[r] == ROW_FRICTION) {
    const float fl = X.fl[r];
    if (x <= -R * fl) return -fl * x - 0.5f * R * fl * fl;
    if (x >= R * fl) return fl * x - 0.5f * R * fl * fl;
    return 0.5f * x * x / R;
  }
  return x < 0.f ? 0.5f * x * x / R : 0.f;
}

template <int NA, int NF>
struct NewtonCtx {
  static constexpr int NV = Sim<NA, NF>::NV, MAXR = Rows<NA, NF>::MAXR;
  const Sim<NA, NF>& S;
  const Rows<NA, NF>& X;
  // c(a) = 1/2 (a - a0)' M (a - a0) + sum_r s_r(J_r a - aref_r); jar = J a - aref
  float cost(const float* a, float* jar) const {
    float da[NV], Mda[NV], c = 0.f;
    for (int i = 0; i < NV; i++) da[i] = a[i] - S.qacc_s[i];
    mul_m(S, da, Mda);
    for (int i = 0; i < NV; i++) c += 0.5f * da[i] * Mda[i];
    for (int r = 0; r < X.nr; r++) {
      float x = -X.aref[r];
      for (int i = 0; i < NV; i++) x += X.J[r][i] * a[i];
      jar[r] = x;
      c += row_cost(X, r, x);
    }
    return c;
  }
  // d/dalpha c(a + alpha p) = g0 + alpha pMp - sum_r f_r(jar_r + alpha jv_r) jv_r
  float deriv(float g0, float pMp, const float* jar, const float* jv, float alpha, float* curv) const {
    float g = g0 + alpha * pMp, h = pMp;
    for (int r = 0; r < X.nr; r++) {
      bool q;
      g -= row_force(X, r, jar[r] + alpha * jv[r], q) * jv[r];
      if (q) h += jv[r] * jv[r] / X.R[r];
    }
    if (curv) *curv = h;
    return g;
  }
  // exact minimiser over alpha >= 0 of the convex piecewise-quadratic c(a + alpha p): the root
  // of its piecewise-linear derivative, bracketed between the sorted zone breakpoints
  float line_search(float g0, float pMp, const float* jar, const float* jv) const {
    float glo = deriv(g0, pMp, jar, jv, 0.f, nullptr);
    if (glo >= 0.f) return 0.f;
    float bp[2 * MAXR];
    int nb = 0;
    for (int r = 0; r < X.nr; r++) {
      if (jv[r] == 0.f) continue;
      const float R = X.R[r];
      const float xs[2] = {X.type[r] == ROW_FRICTION ? -R * X.fl[r] : 0.f, R * X.fl[r]};
      for (int k = 0; k < (X.type[r] == ROW_FRICTION ? 2 : 1); k++) {
        const float al = (xs[k] - jar[r]) / jv[r];
        if (al > 0.f) bp[nb++] = al;
      }
    }
    std::sort(bp, bp + nb);
    float lo = 0.f;
    for (int k = 0; k < nb; k++) {
      const float hi = bp[k];
      if (hi <= lo) continue;
      const float ghi = deriv(g0, pMp, jar, jv, hi, nullptr);
      if (ghi >= 0.f) return lo + (hi - lo) * (-glo) / (ghi - glo);
      lo = hi, glo = ghi;
    }
    float h;
    deriv(g0, pMp, jar, jv, lo + 1.f, &h);  // the last (unbounded) piece's curvature
    return lo - glo / h;
  }
};

// dense Cholesky solve of the SPD H (n x n, row-major n x n); false on a non-positive pivot
template <int N>
bool chol_solve(float (&A)[N][N], float* x, const float* b) {
  float L[N][N];
  for (int i = 0; i < N; i++)
    for (int j = 0; j <= i; j++) {
      float s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (!(s > 0.f)) return false;
        L[i][i] = sqrtf(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  float y[N];
  for (int i = 0; i < N; i++) {
    float s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = N - 1; i >= 0; i--) {
    float s = y[i];
    for (int k = i + 1; k < N; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return true;
}

template <int NA, int NF>
void solve_newton(Sim<NA, NF>& S, const Rows<NA, NF>& X) {
  constexpr int NV = Sim<NA, NF>::NV, MAXR = Rows<NA, NF>::MAXR;
  const DModel& m = *S.mp;
  const NewtonCtx<NA, NF> C{S, X};
  const float scale = m.pgs_scale, tol = m.tolerance;
  float a[NV], jar[MAXR], jv[MAXR];
  // warm start (mj_fwdConstraint): qacc_warmstart unless qacc_smooth costs less
  const float cw = C.cost(S.warm, jar), cs = C.cost(S.qacc_s, jar);
  for (int i = 0; i < NV; i++) a[i] = cw < cs ? S.warm[i] : S.qacc_s[i];
  float cost = C.cost(a, jar);
  for (int it = 0; it < m.iterations; it++) {
    float da[NV], g[NV], H[NV][NV];
    for (int i = 0; i < NV; i++) da[i] = a[i] - S.qacc_s[i];
    mul_m(S, da, g);
    for (int k = 0; k < NV; k++) {  // H = M (columns of the packed blocks)
      float e[NV] = {}, Me[NV];
      e[k] = 1.f;
      mul_m(S, e, Me);
      for (int i = 0; i < NV; i++) H[i][k] = Me[i];
    }
    for (int r = 0; r < X.nr; r++) {
      bool q;
      const float f = row_force(X, r, jar[r], q);
      for (int i = 0; i < NV; i++) g[i] -= X.J[r][i] * f;
      if (q) {
        const float D = 1.f / X.R[r];
        for (int i = 0; i < NV; i++)
          for (int k = 0; k < NV; k++) H[i][k] += D * X.J[r][i] * X.J[r][k];
      }
    }
    float gn = 0.f;
    for (int i = 0; i < NV; i++) gn += g[i] * g[i];
    if (scale * sqrtf(gn) < tol || gn == 0.f) break;
    float p[NV], mg[NV];
    for (int i = 0; i < NV; i++) mg[i] = -g[i];
    if (!chol_solve<NV>(H, p, mg)) break;
    float Mp[NV], pMp = 0.f, g0 = 0.f;
    mul_m(S, p, Mp);
    for (int i = 0; i < NV; i++) pMp += p[i] * Mp[i], g0 += da[i] * Mp[i];
    for (int r = 0; r < X.nr; r++) {
      float s = 0.f;
      for (int i = 0; i < NV; i++) s += X.J[r][i] * p[i];
      jv[r] = s;
    }
    const float alpha = C.line_search(g0, pMp, jar, jv);
    if (!(alpha > 0.f)) break;
    float an[NV], jn[MAXR];
    for (int i = 0; i < NV; i++) an[i] = a[i] + alpha * p[i];
    const float cn = C.cost(an, jn);
    if (!(cn <= cost)) break;  // rounding level: no further progress
    const float improvement = scale * (cost - cn);
    for (int i = 0; i < NV; i++) a[i] = an[i];
    for (int r = 0; r < X.nr; r++) jar[r] = jn[r];
    cost = cn;
    if (improvement < tol) break;
  }
  for (int i = 0; i < NV; i++) S.qacc[i] = a[i], S.fcon[i] = 0.f;
  for (int r = 0; r < X.nr; r++) {
    bool q;
    const float f = row_force(X, r, jar[r], q);
    for (int i = 0; i < NV; i++) S.fcon[i] += X.J[r][i] * f;
  }
}

// one mj_forward after the collision: smooth dynamics, rows, solve (sets S.qacc / S.fcon)
template <int NA, int NF>
void forward_env(Sim<NA, NF>& S, int sol, const CpuContact* con, int ncon, const float* applied, int n, int e) {
  constexpr int NV = Sim<NA, NF>::NV;
  S.kinematics();
  S.com_crb();
  S.factor();
  S.smooth_forces();
  if (applied) S.add_applied(applied, n, e);
  S.solve_m(S.qacc_s, S.fsmooth);
  Rows<NA, NF> X;
  make_rows(S, con, ncon, X);
  if (X.nr == 0) {
    for (int i = 0; i < NV; i++) S.qacc[i] = S.qacc_s[i], S.fcon[i] = 0.f;
    return;
  }
  if (sol == SIM_SOL_NEWTON)
    solve_newton(S, X);
  else
    solve_pgs(S, X);
}

// frame_skip x mj_step of env e (mj_checkPos/Vel, collision at the substep's positions,
// forward, mj_checkAcc, Euler); the device path's order of state / obs / contact-count writes
template <int NA, int NF>
void step_env(const CpuBatch& B, const sim_state& st, const sim_params& pp, const float* action, int nsub,
              float* obs, int e) {
  constexpr int NV = Sim<NA, NF>::NV;
  const DModel& m = B.dm;
  const int n = B.n;
  Sim<NA, NF> S(&m, pp.mass_scale ? pp.mass_scale[e] : 1.f, pp.friction ? pp.friction[e] : -1.f,
                pp.damping_scale ? pp.damping_scale[e] : 1.f);
  load_state(S, st, n, e);
  if (action)
    for (int k = 0; k < NA; k++)
      if (k < m.nact) S.ctrl[k] = action[(size_t)e * m.nact + k];
  const bool con = !m.disable_contact && m.npair > 0;
  const int sol = B.model->desc.solver;
  float* const applied = st.qfrc_applied;
  CpuContact cl[SIM_MAXCON];
  float nsum = 0.f;
  for (int s = 0; s < nsub; s++) {
    if (S.check_state() && applied) zero_applied(applied, NV, n, e);
    int nc = 0;
    if (con) {
      S.kinematics();
      nc = collide_env(B, S, e, cl, S.status);
    }
    forward_env(S, sol, cl, nc, applied, n, e);
    if (S.acc_bad()) {
      S.soft_reset(SIM_ST_BADQACC);
      if (applied) zero_applied(applied, NV, n, e);
      nc = 0;
      if (con) {  // mj_forward at qpos0, collision included
        S.kinematics();
        nc = collide_env(B, S, e, cl, S.status);
      }
      forward_env(S, sol, cl, nc, nullptr, n, e);
    }
    nsum += (float)nc;
    const float ee[3] = {S.ee[0], S.ee[1], S.ee[2]};
    S.integrate();
    S.ee[0] = ee[0], S.ee[1] = ee[1], S.ee[2] = ee[2];
  }
  store_state(S, st, n, e);
  if (con && st.ncon) st.ncon[e] += nsum;
  if (obs) write_obs(S, obs, e);
}

int check(const CpuBatch* c, const sim_state* s) {
  if (!c || !s) return soarm_set_error(SIM_E_ARG, "null argument");
  if (!s->qpos || !s->qvel || !s->qacc_warmstart || !s->ctrl || !s->status)
    return soarm_set_error(SIM_E_ARG, "state buffers must all be set");
  return SIM_OK;
}

}  // namespace

// ===================================================================== entry points
int cpu_batch_create(const sim_model* m, int n, CpuBatch** out) {
  CpuBatch* c = new CpuBatch();
  c->model = m;
  c->n = n;
  c->dm = m->dm;
  c->dm.hull_vert = m->hull_vert.empty() ? nullptr : m->hull_vert.data();
  c->dm.hull_adr = m->hull_adr.empty() ? nullptr : m->hull_adr.data();
  c->dm.hull_adj = m->hull_adj.empty() ? nullptr : m->hull_adj.data();
  c->dm.hull_lut = m->hull_lut.empty() ? nullptr : m->hull_lut.data();
  c->dm.hull_rec = m->hull_rec.empty() ? nullptr : m->hull_rec.data();
  c->dm.hull_lutrec = m->hull_lutrec.empty() ? nullptr : m->hull_lutrec.data();
  c->dm.hull_ovf = m->hull_ovf.empty() ? nullptr : m->hull_ovf.data();
  c->dm.hull_sb = m->hull_sb.empty() ? nullptr : m->hull_sb.data();
  for (int g = 0; g < SIM_MAXGEOM; g++) {
    c->dm.geom_lutadr[g] = g < m->desc.ngeom ? m->lutadr[g] : -1;
    c->dm.geom_sbadr[g] = g < m->desc.ngeom ? m->sbadr[g] : -1;
  }
  if (!m->desc.disable_contact) c->sepax.assign((size_t)std::max(m->desc.npair, 1) * 3 * n, 0.f);
  *out = c;
  return SIM_OK;
}

void cpu_batch_free(CpuBatch* c) { delete c; }

// the contacts at qpos0 into m->dm.c0_* (dmodel.h): kinematics at qpos0, then every candidate pair
// through the kernels' collide code, as k_collide writes them (mask bit per pair with contacts,
// count word for multi-contact pairs, records in the pair's slots)
int cpu_qpos0_contacts(sim_model* m) {
  DModel& d = m->dm;
  memset(d.c0_w, 0, sizeof(d.c0_w));
  d.c0_n = 0;
  if (m->desc.disable_contact || d.npair == 0) return SIM_OK;
  CpuBatch* c = nullptr;
  cpu_batch_create(m, 1, &c);
  const int nw = (d.npair + 31) >> 5;
  dispatch_nf(m->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    Sim<6, NF> S(&c->dm, 1.f, -1.f, 1.f);
    S.soft_reset(0);
    S.kinematics();
    float gpose[SIM_MAXBODY * BREC];
    write_body_frames(S, gpose, 1, 0, 0, 1);
    float cb[PAIR_MAXCON * 7];
    for (int p = 0; p < d.npair; p++) {
      PairOut o{cb, 1, 0, 0, d.pair_cap[p], 0};
      collide_pair(c->dm, p, gpose, 1, 0, o, SepCache{c->sepax.data(), 1, 0});
      if (o.n == 0) continue;
      d.c0_w[p >> 5] |= 1u << (p & 31);
      if (d.pair_cq[p] >= 0) d.c0_w[nw] |= (uint32_t)(o.n - 1) << (2 * d.pair_cq[p]);
      for (int k = 0; k < o.n && d.c0_n < SIM_MAXCON; k++, d.c0_n++) {
        d.c0_slot[d.c0_n] = d.pair_slot[p] + k;
        for (int f = 0; f < 7; f++) d.c0_rec[d.c0_n][f] = cb[7 * k + f];
      }
    }
  });
  cpu_batch_free(c);
  return SIM_OK;
}

extern "C" int soarm_test_hull_support(const sim_model* m, int g, const float* dirs, int nd, float* out) {
  if (!m || !dirs || !out || nd < 0) return soarm_set_error(SIM_E_ARG, "null argument");
  if (g < 0 || g >= m->desc.ngeom || m->desc.geom_type[g] != SIM_GEOM_MESH || m->lutadr[g] < 0)
    return soarm_set_error(SIM_E_ARG, "not a mesh geom");
  CpuBatch* c = nullptr;
  cpu_batch_create(m, 1, &c);
  for (int i = 0; i < nd; i++) {
    const float3 v = hull_support(c->dm, g, dirs + 3 * i);
    out[3 * i] = v.x, out[3 * i + 1] = v.y, out[3 * i + 2] = v.z;
  }
  cpu_batch_free(c);
  return SIM_OK;
}

int cpu_reset(CpuBatch* c, const sim_state* s, const float* init_qpos, const float* init_qvel,
              const float* extra_qpos, uint64_t seed, int64_t env_offset, const uint8_t* mask, float* obs) {
  if (int rc = check(c, s)) return rc;
  const sim_state st = *s;
  dispatch_nf(c->model->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    parallel_envs(c->n, [&](int e) {
      env_reset<6, NF>(&c->dm, c->n, e, st, init_qpos, init_qvel, extra_qpos, (uint32_t)seed,
                       (uint32_t)(seed >> 32), (long long)env_offset, mask, obs);
    });
  });
  return SIM_OK;
}

int cpu_step(CpuBatch* c, const sim_state* s, const sim_params& p, const float* action, int frame_skip,
             float* obs) {
  if (int rc = check(c, s)) return rc;
  if (frame_skip < 1) return soarm_set_error(SIM_E_ARG, "frame_skip must be >= 1");
  const sim_state st = *s;
  dispatch_nf(c->model->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    parallel_envs(c->n, [&](int e) { step_env<6, NF>(*c, st, p, action, frame_skip, obs, e); });
  });
  return SIM_OK;
}

int cpu_bias(CpuBatch* c, const sim_state* s, const sim_params& p, float* qfrc_bias) {
  if (int rc = check(c, s)) return rc;
  if (!qfrc_bias) return soarm_set_error(SIM_E_ARG, "qfrc_bias is null");
  const sim_state st = *s;
  dispatch_nf(c->model->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    parallel_envs(c->n, [&](int e) { env_bias<6, NF>(&c->dm, c->n, e, st, qfrc_bias, p); });
  });
  return SIM_OK;
}

int cpu_observe(CpuBatch* c, const sim_state* s, float* obs) {
  if (int rc = check(c, s)) return rc;
  if (!obs) return soarm_set_error(SIM_E_ARG, "obs is null");
  const sim_state st = *s;
  dispatch_nf(c->model->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    parallel_envs(c->n, [&](int e) { env_observe<6, NF>(&c->dm, c->n, e, st, obs); });
  });
  return SIM_OK;
}

int cpu_contacts(CpuBatch* c, const sim_state* s, float* out, int32_t* ncon) {
  if (int rc = check(c, s)) return rc;
  if (!out || !ncon) return soarm_set_error(SIM_E_ARG, "null output");
  if (c->model->desc.disable_contact) return soarm_set_error(SIM_E_ARG, "model compiled with contacts disabled");
  const sim_state st = *s;
  dispatch_nf(c->model->nf, [&](auto nfc) {
    constexpr int NF = decltype(nfc)::value;
    parallel_envs(c->n, [&](int e) {
      Sim<6, NF> S(&c->dm, 1.f, -1.f, 1.f);
      load_state(S, st, c->n, e);
      S.kinematics();
      CpuContact cl[SIM_MAXCON];
      int status = 0;
      const int nc = collide_env(*c, S, e, cl, status);
      for (int k = 0; k < nc; k++) {
        float* o = out + ((size_t)e * SIM_MAXCON + k) * 8;
        o[0] = cl[k].dist;
        for (int q = 0; q < 3; q++) o[1 + q] = cl[k].pos[q], o[4 + q] = cl[k].n[q];
        memcpy(o + 7, &cl[k].pair, 4);
      }
      ncon[e] = nc;
    });
  });
  return SIM_OK;
}

int cpu_rand_uniform(CpuBatch* c, uint64_t seed, int64_t env_offset, uint32_t counter, int k, float lo, float hi,
                     float* out) {
  if (!c || !out) return soarm_set_error(SIM_E_ARG, "null argument");
  parallel_envs(c->n, [&](int e) {
    env_rand(e, (uint32_t)seed, (uint32_t)(seed >> 32), (long long)env_offset, counter, k, lo, hi - lo, out);
  });
  return SIM_OK;
}

int cpu_ik(CpuBatch* c, const float* target, const float* target_quat, float* q, int32_t* ok, int32_t* iters,
           const sim_ik_opts& o) {
  parallel_envs(c->n, [&](int e) { env_ik<6>(&c->dm, c->n, e, target, target_quat, q, ok, iters, o); });
  return SIM_OK;
}
