// soarm_collide.h — per-env collision for the fused step kernel (gfx950).
//
// Restates mj_collision for the hot-path scenes:
//   * the candidate pairs are the compiler's static list in MuJoCo's contact
//     order; every lane walks the same list, so the pair loop and the
//     geom/body lookups are wave-uniform;
//   * midphase: bounding sphere + world AABB about each geom's collision box;
//   * narrowphase: MPR penetration (hull / box vs hull, tolerance 1e-6,
//     <= 50 refinement steps), box-box SAT + face clipping (<= 4 contacts),
//     plane-box corners (<= 4), plane-hull deepest vertex;
//   * hull support = steepest-ascent hill climbing on the hull vertex graph
//     (L2-resident float4 vertices, CSR adjacency).
// Work decomposition: k_collide runs one lane per (env, pair) — one pair per
// block so geom types and model lookups are wave-uniform, and 4096 envs x 86
// pairs give ~5.5k waves to hide the hill-climbing load latency.  Each pair
// writes <= 4 contacts into its own fixed slots; the dynamics kernel gathers
// them by walking the pairs in order, which makes contact indexing identical
// to the serial mj_collision order.
#pragma once
#include "soarm_step.h"
#ifdef SOARM_DIAG_SUPPORT
#include <atomic>
#include <cstdio>
#endif

namespace soarm {

constexpr int CON_MAXG = 16;  // collidable geoms supported by the contact kernel
// MPR's zero tests.  libccd (and the oracle) use DBL_EPSILON as an ABSOLUTE
// threshold, i.e. effectively exact sign tests on lengths, triple products and
// squared cross products.  An fp32 epsilon (1.2e-7) in that role is NOT small
// for these unnormalised quantities at centimetre scale (|v0 x v1|^2 ~ 1e-7 m^4
// for 2 cm geoms): it declared non-collinear portals collinear and produced
// phantom penetrations several millimetres deep.  So: exact-sign tests here too.
constexpr float FEPS = 1e-30f;
constexpr float MPR_TOLF = 1e-6f;
constexpr int MPR_ITERS = 50;
// m: a support-bound test declares a pair apart only beyond this (fp32 rounding of the bound
// is ~1e-8 m at the arm's scale, so such a pair is apart for MPR in any precision as well)
constexpr float SEP_MARGIN = 1e-6f;

// per-lane contact list of the dynamics kernel (LDS, [slot][lane])
struct ConLds {
  float (*a)[64];  // [SIM_MAXCON * 8][64]: dist, pos(3), n(3), pair
  int lane;
  HDI float& dist(int c) const { return a[c * 8][lane]; }
  HDI float& pos(int c, int k) const { return a[c * 8 + 1 + k][lane]; }
  HDI float& n(int c, int k) const { return a[c * 8 + 4 + k][lane]; }
  DEVI int pair(int c) const { return __float_as_int(a[c * 8 + 7][lane]); }
  DEVI void set_pair(int c, int p) const { a[c * 8 + 7][lane] = __int_as_float(p); }
};

struct GeomPose {
  float p[3], R[9];
};

// body world frames in global memory, SoA [body*BREC + k][env]: position (3), rotation (9) of every
// body but the world (its slot stays unused).  The collide composes a geom's pose and midphase bound
// from its body's frame (load_pose / geom_bound below, the expressions that wrote per-geom records
// until round 5, so every value is the same): 12 floats per body instead of 18 per geom -- the 8
// body frames of the pick scene are 96 floats per env against the 15 geom records' 270, written by
// every substep and read by every collide.
constexpr int BREC = 12;

// contacts of one candidate pair (<= 4: box-box / plane-box corners; 1 otherwise), written
// straight to the pair's slots of the contact buffer cbuf [slot*7 + f][env]: f = dist, pos(3),
// normal(3) geom1 -> geom2.  (A register array indexed by the running count ends up in
// scratch memory: the count differs per lane.)
constexpr int PAIR_MAXCON = 4;
struct PairOut {
  float* cbuf;
  int nenv, e, s0, cap;  // env count / env, first slot and slot count of the pair
  int n;                 // contacts written
  int xc = 0;            // diagnostic (SOARM_COLLIDE_STATS): which test decided the pair
};

// hill-climbing support on a mesh hull; returns the local vertex.  Opens at the cube-map
// cell's start record (coordinates + neighbour ids in one load) and climbs to the best
// neighbour while one improves; each step loads all candidates' records together (their
// coordinates to compare, their neighbour ids for the next step), so a step is one
// dependent round trip.  Same comparisons, order and result as a CSR walk.
// (the hull tables are read through global-address-space pointers: the DModel holds them as
// plain pointers, which would otherwise compile to flat loads)
#if SOARM_DEVICE_PASS
template <class T>
using gptr = const __attribute__((address_space(1))) T*;
#else
template <class T>
using gptr = const T*;
#endif
HDI uint4 ldg(gptr<uint4> p, int i) {  // (dword loads, merged into one 16-B load)
  const gptr<uint32_t> q = (gptr<uint32_t>)(p + i);
  return make_uint4(q[0], q[1], q[2], q[3]);
}
#if defined(SOARM_DIAG_SUPPORT) && !SOARM_DEVICE_PASS
// (diagnostic build, CPU backend: the same counts with the lane's history reset per pair call --
// what a cache that lives for one narrowphase call could reuse)
struct DiagSupHost {
  std::atomic<unsigned long long> c[CON_MAXG][4];
  ~DiagSupHost() {
    for (int g = 0; g < CON_MAXG; g++)
      if (c[g][0])
        fprintf(stderr, "host support geom %d: queries %llu, same cell %llu, same answer %llu, climb trips %llu\n", g,
                c[g][0].load(), c[g][1].load(), c[g][2].load(), c[g][3].load());
  }
};
inline DiagSupHost g_diag_sup_host;
inline thread_local uint32_t g_diag_prev_host[2] = {~0u, ~0u};
inline void diag_support(int g, int cell, uint4 r0, int steps) {
  const uint32_t key = ((uint32_t)g << 20) | (uint32_t)cell, ans = r0.x ^ (r0.y * 3u) ^ (r0.z * 7u);
  g_diag_sup_host.c[g][0]++;
  if (g_diag_prev_host[0] == key) g_diag_sup_host.c[g][1]++;
  if (g_diag_prev_host[1] == ans && (g_diag_prev_host[0] >> 20) == (uint32_t)g) g_diag_sup_host.c[g][2]++;
  g_diag_sup_host.c[g][3] += steps;
  g_diag_prev_host[0] = key, g_diag_prev_host[1] = ans;
}
#endif
#if defined(SOARM_DIAG_SUPPORT) && SOARM_DEVICE_PASS
// (diagnostic build: per geom, support queries, queries whose cube-map cell / answer repeats the
// lane's previous query on that geom, and climbing round trips)
// (g_diag_sup, g_diag_prev: soarm_sim.hip)
DEVI void diag_support(int g, int cell, uint4 r0, int steps) {
  const int t = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= 128 * 8192) return;
  const uint32_t key = ((uint32_t)g << 20) | (uint32_t)cell, ans = r0.x ^ (r0.y * 3u) ^ (r0.z * 7u);
  atomicAdd(&g_diag_sup[g][0], 1ull);
  if (g_diag_prev[0][t] == key) atomicAdd(&g_diag_sup[g][1], 1ull);
  if (g_diag_prev[1][t] == ans && (g_diag_prev[0][t] >> 20) == (uint32_t)g) atomicAdd(&g_diag_sup[g][2], 1ull);
  atomicAdd(&g_diag_sup[g][3], (unsigned long long)steps);
  g_diag_prev[0][t] = key, g_diag_prev[1][t] = ans;
}
#endif
HDI float3 hull_support(const DModel& m, int g, const float l[3]) {
  const gptr<uint4> rec = (gptr<uint4>)m.hull_rec + HULL_LUTREC * m.geom_hulladr[g];
#if defined(SOARM_DIAG_SUPPORT)
  const int dcell = lut_cell(l[0], l[1], l[2]);
  int dsteps = 0;
#endif
  // the cell's copy of its start vertex's record, then per climbing step the record of the vertex
  // moved to: each carries its first 8 neighbours' coordinates, so a step is one round trip and
  // the last (no neighbour improves) none
  const gptr<uint4> lr = (gptr<uint4>)m.hull_lutrec + HULL_LUTREC * (m.geom_lutadr[g] + lut_cell(l[0], l[1], l[2]));
  uint4 r0 = ldg(lr, 0), nb[8];
#pragma unroll
  for (int k = 0; k < 8; k++) nb[k] = ldg(lr, 2 + k);
  const int nvert = m.geom_hullnum[g];
  auto dotr = [&](const uint4& r) {
    return l[0] * fbits(r.x) + l[1] * fbits(r.y) + l[2] * fbits(r.z);
  };
  float cd = dotr(r0);
  for (int guard = 0; guard < nvert; guard++) {
    float nd = cd;
    int best = -1;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float s = dotr(nb[k]);
      if (s > nd) nd = s, best = k;
    }
    uint32_t u = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (k == best) u = nb[k].w;
    const int deg = (int)(r0.w & 255u);
    if (deg > 8) {  // hub vertex (~2%): the rest of its neighbours, 8 per round trip
      const gptr<uint16_t> ov = (gptr<uint16_t>)m.hull_ovf + (r0.w >> 8);
      for (int a = 8; a < deg; a += 8) {
        uint32_t id[8];
        uint4 c[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          id[k] = (a + k < deg) ? ov[a - 8 + k] : ov[a - 8];
          c[k] = ldg(rec, HULL_LUTREC * id[k]);
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const float s = dotr(c[k]);
          if (s > nd) nd = s, u = id[k], best = 8;
        }
      }
    }
    if (best < 0) break;
    const gptr<uint4> r = rec + HULL_LUTREC * u;
    r0 = ldg(r, 0), cd = nd;
#pragma unroll
    for (int k = 0; k < 8; k++) nb[k] = ldg(r, 2 + k);
#if defined(SOARM_DIAG_SUPPORT)
    dsteps++;
#endif
  }
#if defined(SOARM_DIAG_SUPPORT)
  diag_support(g, dcell, r0, dsteps);
#endif
  return make_float3(fbits(r0.x), fbits(r0.y), fbits(r0.z));
}

// world support point of geom g (type uniform across the wave)
// upper bound on a mesh hull's support value along a (not necessarily unit) local direction l
// from the support-bound table (dmodel.h HULL_SB_K): 3 table loads, no hull data
HDI float support_ub(const DModel& m, int g, const float l[3]) {
  const float a0 = fabsf(l[0]), a1 = fabsf(l[1]), a2 = fabsf(l[2]);
  int face;
  float u, v, mx;
  if (a0 >= a1 && a0 >= a2) {
    face = l[0] >= 0.f ? 0 : 1, mx = a0, u = l[1], v = l[2];
  } else if (a1 >= a2) {
    face = l[1] >= 0.f ? 2 : 3, mx = a1, u = l[0], v = l[2];
  } else {
    face = l[2] >= 0.f ? 4 : 5, mx = a2, u = l[0], v = l[1];
  }
  const float s = 0.5f * HULL_SB_K / mx;
  const float fu = fminf(fmaxf((u + mx) * s, 0.f), (float)HULL_SB_K), fv = fminf(fmaxf((v + mx) * s, 0.f), (float)HULL_SB_K);
  const int i = min((int)fu, HULL_SB_K - 1), j = min((int)fv, HULL_SB_K - 1);
  const float a = fu - i, b = fv - j;
  const gptr<float> t = (gptr<float>)m.hull_sb + m.geom_sbadr[g] + face * HULL_SB_FACE + i * (HULL_SB_K + 1) + j;
  const float h00 = t[0], h10 = t[HULL_SB_K + 1], h01 = t[1], h11 = t[HULL_SB_K + 2];
  const float q = (a + b <= 1.f) ? (1.f - a - b) * h00 + a * h10 + b * h01
                                 : (a + b - 1.f) * h11 + (1.f - a) * h01 + (1.f - b) * h10;
  return mx * q;
}

HDI void support(const DModel& m, int g, const GeomPose& P, const float d[3], float out[3]) {
  float l[3];
  mtv(l, P.R, d);
  float p[3] = {0, 0, 0};
  const int t = m.geom_type[g];
  if (t == SIM_GEOM_BOX) {
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = (l[k] >= 0.f ? 1.f : -1.f) * m.geom_size[g][k];
  } else if (t == SIM_GEOM_MESH) {
    const float3 v = hull_support(m, g, l);
    p[0] = v.x, p[1] = v.y, p[2] = v.z;
  }
  float w[3];
  mv(w, P.R, p);
  out[0] = P.p[0] + w[0], out[1] = P.p[1] + w[1], out[2] = P.p[2] + w[2];
}

HDI void geom_center(const DModel& m, int g, const GeomPose& P, float c[3]) {
  const float lc[3] = {m.geom_center[g][0], m.geom_center[g][1], m.geom_center[g][2]};
  float w[3];
  mv(w, P.R, lc);
  c[0] = P.p[0] + w[0], c[1] = P.p[1] + w[1], c[2] = P.p[2] + w[2];
}

// ---------------------------------------------------------------------- MPR
HDI double dotd(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
HDI void subd(double r[3], const double a[3], const double b[3]) {
  r[0] = a[0] - b[0], r[1] = a[1] - b[1], r[2] = a[2] - b[2];
}
HDI void crossd(double r[3], const double a[3], const double b[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1], r[1] = a[2] * b[0] - a[0] * b[2], r[2] = a[0] * b[1] - a[1] * b[0];
}
struct MSup {
  float v[3], v1[3], v2[3];
};
struct MPair {
  const DModel& m;
  int g1, g2;
  const GeomPose &P1, &P2;
  HDI void sup(const float d[3], MSup& s) const {
    const float nd[3] = {-d[0], -d[1], -d[2]};
    support(m, g1, P1, d, s.v1);
    support(m, g2, P2, nd, s.v2);
    s.v[0] = s.v1[0] - s.v2[0], s.v[1] = s.v1[1] - s.v2[1], s.v[2] = s.v1[2] - s.v2[2];
  }
};
HDI bool fz(float x) { return fabsf(x) < FEPS; }
HDI void nrm(float a[3]) {
  const float n2 = dot3(a, a);
  if (n2 > 0.f) {
    const float s = frsqrt(n2);
    a[0] *= s, a[1] *= s, a[2] *= s;
  }
}
HDI void sub(float r[3], const float a[3], const float b[3]) {
  r[0] = a[0] - b[0], r[1] = a[1] - b[1], r[2] = a[2] - b[2];
}
HDI void portal_dir(const MSup p[4], float d[3]) {
  float a[3], b[3];
  sub(a, p[2].v, p[1].v);
  sub(b, p[3].v, p[1].v);
  cross(d, a, b);
  nrm(d);
}
HDI bool reach_tol(const MSup p[4], const MSup& v4, const float d[3]) {
  const float d4 = dot3(v4.v, d);
  const float mn = fminf(fminf(d4 - dot3(p[1].v, d), d4 - dot3(p[2].v, d)), d4 - dot3(p[3].v, d));
  return mn <= MPR_TOLF;
}
// dst = c ? src : dst, element by element (v_cndmask): a branchy `p[i] = v4` lets the
// compiler sink the stores into one store through a computed index, which puts the whole
// portal in scratch memory
HDI void sel(MSup& dst, bool c, const MSup& src) {
#pragma unroll
  for (int k = 0; k < 3; k++) {
    dst.v[k] = c ? src.v[k] : dst.v[k];
    dst.v1[k] = c ? src.v1[k] : dst.v1[k];
    dst.v2[k] = c ? src.v2[k] : dst.v2[k];
  }
}
HDI void expand(MSup p[4], const MSup& v4) {
  float x[3];
  cross(x, v4.v, p[0].v);
  const bool c1 = dot3(p[1].v, x) > 0.f, c2 = dot3(p[2].v, x) > 0.f, c3 = dot3(p[3].v, x) > 0.f;
  // c1: (c2 ? p1 : p3) = v4;  !c1: (c3 ? p2 : p1) = v4
  sel(p[1], c1 ? c2 : !c3, v4);
  sel(p[2], !c1 && c3, v4);
  sel(p[3], c1 && !c2, v4);
}
// -1 separated, 0 portal, 1 origin on v1, 2 origin on segment v0-v1.  On a separated exit
// found by a support query, sep = that query's direction (the Minkowski difference lies
// on its negative side: a separating axis); otherwise sep is left as it was.
HDI void setsep(float sep[3], const float d[3]) { sep[0] = d[0], sep[1] = d[1], sep[2] = d[2]; }
HDI int discover(const MPair& P, MSup p[4], float sep[3]) {
  float c1[3], c2[3], d[3], va[3], vb[3];
  geom_center(P.m, P.g1, P.P1, c1);
  geom_center(P.m, P.g2, P.P2, c2);
#pragma unroll
  for (int k = 0; k < 3; k++) p[0].v1[k] = c1[k], p[0].v2[k] = c2[k], p[0].v[k] = c1[k] - c2[k];
  if (fz(p[0].v[0]) && fz(p[0].v[1]) && fz(p[0].v[2])) p[0].v[0] += 10.f * FEPS;
  d[0] = -p[0].v[0], d[1] = -p[0].v[1], d[2] = -p[0].v[2];
  nrm(d);
  P.sup(d, p[1]);
  float dt = dot3(p[1].v, d);
  if (fz(dt) || dt < 0.f) {
    setsep(sep, d);
    return -1;
  }
  cross(d, p[0].v, p[1].v);
  if (fz(dot3(d, d))) {
    if (fz(p[1].v[0]) && fz(p[1].v[1]) && fz(p[1].v[2])) return 1;
    return 2;
  }
  nrm(d);
  P.sup(d, p[2]);
  dt = dot3(p[2].v, d);
  if (fz(dt) || dt < 0.f) {
    setsep(sep, d);
    return -1;
  }
  sub(va, p[1].v, p[0].v);
  sub(vb, p[2].v, p[0].v);
  cross(d, va, vb);
  nrm(d);
  if (dot3(d, p[0].v) > 0.f) {
    const MSup t = p[1];
    p[1] = p[2];
    p[2] = t;
    d[0] = -d[0], d[1] = -d[1], d[2] = -d[2];
  }
  for (int guard = 0; guard < 1000; guard++) {
    P.sup(d, p[3]);
    dt = dot3(p[3].v, d);
    if (fz(dt) || dt < 0.f) {
      setsep(sep, d);
      return -1;
    }
    cross(va, p[1].v, p[3].v);
    dt = dot3(va, p[0].v);
    const bool r2 = dt < 0.f && !fz(dt);
    cross(va, p[3].v, p[2].v);
    dt = dot3(va, p[0].v);
    const bool r1 = !r2 && dt < 0.f && !fz(dt);
    if (!r1 && !r2) return 0;
    sel(p[2], r2, p[3]);
    sel(p[1], r1, p[3]);
    sub(va, p[1].v, p[0].v);
    sub(vb, p[2].v, p[0].v);
    cross(d, va, vb);
    nrm(d);
  }
  return -1;
}
template <class T>
HDI T dot3t(const T a[3], const T b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
// closest point of triangle abc to the origin (T = double: MPR's final depth and normal, below)
template <class T>
HDI void closest_tri(const T a[3], const T b[3], const T c[3], T o[3]) {
  T ab[3], ac[3];
#pragma unroll
  for (int k = 0; k < 3; k++) ab[k] = b[k] - a[k], ac[k] = c[k] - a[k];
  const T ap[3] = {-a[0], -a[1], -a[2]};
  const T d1 = dot3t(ab, ap), d2 = dot3t(ac, ap);
  if (d1 <= T(0) && d2 <= T(0)) {
    o[0] = a[0], o[1] = a[1], o[2] = a[2];
    return;
  }
  const T bp[3] = {-b[0], -b[1], -b[2]};
  const T d3 = dot3t(ab, bp), d4 = dot3t(ac, bp);
  if (d3 >= T(0) && d4 <= d3) {
    o[0] = b[0], o[1] = b[1], o[2] = b[2];
    return;
  }
  const T vc = d1 * d4 - d3 * d2;
  if (vc <= T(0) && d1 >= T(0) && d3 <= T(0)) {
    const T v = d1 / (d1 - d3);
#pragma unroll
    for (int k = 0; k < 3; k++) o[k] = a[k] + v * ab[k];
    return;
  }
  const T cp[3] = {-c[0], -c[1], -c[2]};
  const T d5 = dot3t(ab, cp), d6 = dot3t(ac, cp);
  if (d6 >= T(0) && d5 <= d6) {
    o[0] = c[0], o[1] = c[1], o[2] = c[2];
    return;
  }
  const T vb = d5 * d2 - d1 * d6;
  if (vb <= T(0) && d2 >= T(0) && d6 <= T(0)) {
    const T w = d2 / (d2 - d6);
#pragma unroll
    for (int k = 0; k < 3; k++) o[k] = a[k] + w * ac[k];
    return;
  }
  const T va = d3 * d6 - d5 * d4;
  if (va <= T(0) && (d4 - d3) >= T(0) && (d5 - d6) >= T(0)) {
    const T w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
#pragma unroll
    for (int k = 0; k < 3; k++) o[k] = b[k] + w * (c[k] - b[k]);
    return;
  }
  const T den = T(1) / (va + vb + vc);
  const T v = vb * den, w = vc * den;
#pragma unroll
  for (int k = 0; k < 3; k++) o[k] = a[k] + ab[k] * v + ac[k] * w;
}
// contact position: the origin's barycentric weights on the portal tetrahedron (or its face),
// applied to both geoms' support points -- in fp64 on the exact Minkowski points (the weights are
// triple products of coordinates ~1 m whose result is ~depth x area: the same cancellation as the
// normal's, mpr below).  pd: the portal direction.
HDI void portal_pos(const MSup p[4], const double pd[3], float pos[3]) {
  double v[4][3], x[3], b[4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) v[i][k] = (double)p[i].v1[k] - (double)p[i].v2[k];
  crossd(x, v[1], v[2]);
  b[0] = dotd(x, v[3]);
  crossd(x, v[3], v[2]);
  b[1] = dotd(x, v[0]);
  crossd(x, v[0], v[1]);
  b[2] = dotd(x, v[3]);
  crossd(x, v[2], v[1]);
  b[3] = dotd(x, v[0]);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (fabs(sum) < 2.220446049250313e-16 || sum < 0.0) {  // (libccd's zero test in double)
    b[0] = 0.0;
    crossd(x, v[2], v[3]);
    b[1] = dotd(x, pd);
    crossd(x, v[3], v[1]);
    b[2] = dotd(x, pd);
    crossd(x, v[1], v[2]);
    b[3] = dotd(x, pd);
    sum = b[1] + b[2] + b[3];
  }
  const double inv = 1.0 / sum;
  double s1[3] = {0, 0, 0}, s2[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) s1[k] += b[i] * (double)p[i].v1[k], s2[k] += b[i] * (double)p[i].v2[k];
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = (float)(0.5 * (s1[k] + s2[k]) * inv);
}
// returns 1 with depth/dir(geom1->geom2)/pos when penetrating; sep = a separating axis
// when it proved the pair apart by a support query (else unchanged)
HDI int mpr(const MPair& P, float& depth, float dir[3], float pos[3], float sep[3]) {
  MSup p[4];
  const int res = discover(P, p, sep);
  if (res < 0 || res == 1) return 0;
  if (res == 2) {
    depth = sqrtf(dot3(p[1].v, p[1].v));
#pragma unroll
    for (int k = 0; k < 3; k++) dir[k] = p[1].v[k], pos[k] = 0.5f * (p[1].v1[k] + p[1].v2[k]);
    nrm(dir);
    return depth > 0.f;
  }
  // refine the portal until it contains the origin
  for (int it = 0;; it++) {
    if (it >= 1000) return 0;
    float d[3];
    portal_dir(p, d);
    const float dt = dot3(d, p[1].v);
    if (fz(dt) || dt > 0.f) break;
    MSup v4;
    P.sup(d, v4);
    const float d4 = dot3(v4.v, d);
    if (!(fz(d4) || d4 > 0.f)) {
      setsep(sep, d);
      return 0;
    }
    if (reach_tol(p, v4, d)) return 0;
    expand(p, v4);
  }
  // penetration: expand towards the boundary
  for (int it = 0;; it++) {
    float d[3];
    portal_dir(p, d);
    MSup v4;
    P.sup(d, v4);
    if (reach_tol(p, v4, d) || it > MPR_ITERS) {
      // depth and normal = the portal's closest point to the origin, in fp64 on the exact Minkowski
      // points s1 - s2 of the fp32 support points: a grazing contact's depth (~1e-6 m) is a
      // cancellation of coordinates ~1 m (the table box), where fp32 leaves ~6e-8 m of noise in
      // each component -- a normal tilted by up to ~5 degrees (tools/env_diverge.py: env 2624 of
      // the headline's t = 100 states, an arm link on the table, 0.077 of tilt and 1e-2 rad/s of
      // arm velocity per substep against the fp64 oracle's vertical normal)
      double pa[3], pb[3], pc[3], w[3];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        pa[k] = (double)p[1].v1[k] - (double)p[1].v2[k];
        pb[k] = (double)p[2].v1[k] - (double)p[2].v2[k];
        pc[k] = (double)p[3].v1[k] - (double)p[3].v2[k];
      }
      closest_tri(pa, pb, pc, w);
      const double dd = sqrt(dot3t(w, w));
      depth = (float)dd;
      if (fz(depth)) return 0;
      const double inv = 1.0 / dd;
      dir[0] = (float)(w[0] * inv), dir[1] = (float)(w[1] * inv), dir[2] = (float)(w[2] * inv);
      double ab[3], ac[3], pd[3];  // the portal's direction (its face normal), for the face fallback
#pragma unroll
      for (int k = 0; k < 3; k++) ab[k] = pb[k] - pa[k], ac[k] = pc[k] - pa[k];
      crossd(pd, ab, ac);
      const double pn = sqrt(dotd(pd, pd));
      if (pn > 0.0) pd[0] /= pn, pd[1] /= pn, pd[2] /= pn;
      portal_pos(p, pd, pos);
      return 1;
    }
    expand(p, v4);
  }
}

// ------------------------------------------------------- native GJK / EPA
// MuJoCo's nativeccd (engine_collision_gjk.c; the oracle's ccd_penetration restates the same
// algorithm in float64): GJK on the Minkowski difference from the centres' difference until a
// support plane separates the origin (apart: sep = that axis) or a tetrahedron encloses it, then
// EPA from that tetrahedron -- the polytope face closest to the origin is expanded by the support
// point along its normal until the support distance is within the tolerance of the face's.
// Depth = the closest face's distance, normal = its outward normal (geom1 -> geom2), pos = the
// midpoint of the witness points (barycentric weights of the origin's projection on that face).
// The simplex lives in registers (value selects: a lane-varying index would put it in scratch);
// the polytope, which only penetrating pairs build (a few envs per pair and substep), in private
// arrays: EPA_KV vertices (v and the geom1 support point; geom2's is v1 - v), EPA_KF faces.
constexpr int CCD_ITERS = 50;
constexpr int EPA_KV = 32, EPA_KF = 64, EPA_KE = 48;
// a face is seen from w when w lies beyond its plane by more than EPA_VIS: support points within
// rounding of a face's plane (flat sides of box-shaped Minkowski differences put them there,
// several collinear) would otherwise see it by the sign of the rounding, and the horizon stops
// being one loop.  Half the EPA tolerance: the expanded face itself is always seen
constexpr float EPA_VIS = 0.5f * MPR_TOLF;
HDI void copy3(float d[3], const float s[3]) { d[0] = s[0], d[1] = s[1], d[2] = s[2]; }
// GJK runs in fp64 on the fp32 support points: a simplex vertex is the Minkowski point
// v = s1 - s2 (exact in fp64) with geom1's support point s1 (EPA's witness).  In fp32 the
// closest-point direction resolves to ~1e-7 only; against the table box's 1.2 m Minkowski
// difference that stalled GJK a few 1e-5 m from the origin and lost sub-mm contacts the fp64
// oracle keeps (tools/ccd_mismatch.py: 2 in 4096 stress poses).  EPA stays fp32.
struct GSup {
  double v[3];
  float v1[3];
};
HDI void copyd(double d[3], const double s[3]) { d[0] = s[0], d[1] = s[1], d[2] = s[2]; }
HDI void gsel(GSup& dst, bool c, const GSup& src) {  // (value selects: see sel)
#pragma unroll
  for (int k = 0; k < 3; k++) dst.v[k] = c ? src.v[k] : dst.v[k], dst.v1[k] = c ? src.v1[k] : dst.v1[k];
}
// support point of the Minkowski difference along the fp64 direction d (queried in fp32)
HDI void gsup(const MPair& P, const double d[3], GSup& g) {
  const float df[3] = {(float)d[0], (float)d[1], (float)d[2]};
  MSup s;
  P.sup(df, s);
#pragma unroll
  for (int k = 0; k < 3; k++) g.v[k] = (double)s.v1[k] - (double)s.v2[k], g.v1[k] = s.v1[k];
}
// closest point of simplex p[0..n) (n <= 3) to the origin; the carrying sub-simplex moves to the front
HDI int gjk_reduce(GSup p[4], int n, double x[3]) {
  if (n == 1) {
    copyd(x, p[0].v);
    return 1;
  }
  if (n == 2) {
    double ab[3];
    subd(ab, p[1].v, p[0].v);
    double t = -dotd(p[0].v, ab);
    const double l2 = dotd(ab, ab);
    if (t <= 0.0 || l2 <= 0.0) {
      copyd(x, p[0].v);
      return 1;
    }
    if (t >= l2) {
      p[0] = p[1];
      copyd(x, p[0].v);
      return 1;
    }
    t /= l2;
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = p[0].v[k] + t * ab[k];
    return 2;
  }
  double ab[3], ac[3];
  subd(ab, p[1].v, p[0].v);
  subd(ac, p[2].v, p[0].v);
  const double ap[3] = {-p[0].v[0], -p[0].v[1], -p[0].v[2]};
  const double d1 = dotd(ab, ap), d2 = dotd(ac, ap);
  if (d1 <= 0.0 && d2 <= 0.0) {
    copyd(x, p[0].v);
    return 1;
  }
  const double bp[3] = {-p[1].v[0], -p[1].v[1], -p[1].v[2]};
  const double d3 = dotd(ab, bp), d4 = dotd(ac, bp);
  if (d3 >= 0.0 && d4 <= d3) {
    p[0] = p[1];
    copyd(x, p[0].v);
    return 1;
  }
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
    const double t = d1 / (d1 - d3);
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = p[0].v[k] + t * ab[k];
    return 2;
  }
  const double cp[3] = {-p[2].v[0], -p[2].v[1], -p[2].v[2]};
  const double d5 = dotd(ab, cp), d6 = dotd(ac, cp);
  if (d6 >= 0.0 && d5 <= d6) {
    p[0] = p[2];
    copyd(x, p[0].v);
    return 1;
  }
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
    const double t = d2 / (d2 - d6);
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = p[0].v[k] + t * ac[k];
    p[1] = p[2];
    return 2;
  }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
    const double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = p[1].v[k] + t * (p[2].v[k] - p[1].v[k]);
    p[0] = p[2];
    return 2;
  }
  const double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
#pragma unroll
  for (int k = 0; k < 3; k++) x[k] = p[0].v[k] + ab[k] * v + ac[k] * w;
  return 3;
}
// tetrahedron faces: face k = the vertices other than k
#if SOARM_DEVICE_PASS
__device__
#endif
constexpr int TETF[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};
// 1: origin inside tetrahedron p; 0: reduced to the face the origin lies beyond (n, x set);
// -1: flat tetrahedron
HDI int tet_contains(GSup p[4], double x[3], int& n) {
  double best = 0.0;
  int bk = -1;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double *a = p[TETF[k][0]].v, *b = p[TETF[k][1]].v, *c = p[TETF[k][2]].v;
    double ab[3], ac[3], nn[3], ak[3];
    subd(ab, b, a);
    subd(ac, c, a);
    crossd(nn, ab, ac);
    subd(ak, p[k].v, a);
    const double sg = dotd(nn, ak) > 0.0 ? -1.0 : 1.0;
    const double ln = sqrt(dotd(nn, nn));
    if (!(ln > 0.0)) return -1;
    const double sd = -sg * dotd(nn, a) / ln;
    if (sd > best) best = sd, bk = k;
  }
  if (bk < 0) return 1;
  GSup t[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    t[j] = p[TETF[0][j]];
#pragma unroll
    for (int k = 1; k < 4; k++) gsel(t[j], bk == k, p[TETF[k][j]]);
  }
  p[0] = t[0], p[1] = t[1], p[2] = t[2];
  n = gjk_reduce(p, 3, x);
  return 0;
}
// support point along d or, when the Minkowski difference reaches no further than the tolerance
// along d, along -d (d negated then); false if neither
HDI bool ccd_extend(const MPair& P, double d[3], GSup& s) {
  gsup(P, d, s);
  if (dotd(d, s.v) > (double)MPR_TOLF) return true;
  d[0] = -d[0], d[1] = -d[1], d[2] = -d[2];
  gsup(P, d, s);
  return dotd(d, s.v) > (double)MPR_TOLF;
}
// GJK ended with the origin ON the segment p[0..1] (n = 2) or the triangle p[0..2] (n = 3):
// centred symmetric shapes, whose second support point is exactly minus the first.  nativeccd
// starts EPA from such simplices (polytope2 / polytope3); here a support point off the simplex's
// span per missing dimension completes a tetrahedron with the origin on its boundary (the
// oracle's gjk_complete).  false: no extent off the span (touching).
HDI bool gjk_complete(const MPair& P, GSup p[4], int n) {
  if (n == 2) {  // a direction normal to the segment: u x (the axis of u's smallest component)
    double u[3], d[3];
    subd(u, p[1].v, p[0].v);
    const double ax = fabs(u[0]), ay = fabs(u[1]), az = fabs(u[2]);
    const int k = ax <= ay && ax <= az ? 0 : ay <= az ? 1 : 2;
    const double e[3] = {k == 0 ? 1.0 : 0.0, k == 1 ? 1.0 : 0.0, k == 2 ? 1.0 : 0.0};
    crossd(d, u, e);
    const double l = sqrt(dotd(d, d));
    if (!(l > 0.0)) return false;
    d[0] /= l, d[1] /= l, d[2] /= l;
    if (!ccd_extend(P, d, p[2])) return false;
  }
  double ab[3], ac[3], nn[3];
  subd(ab, p[1].v, p[0].v);
  subd(ac, p[2].v, p[0].v);
  crossd(nn, ab, ac);
  const double l = sqrt(dotd(nn, nn));
  if (!(l > 0.0)) return false;
  nn[0] /= l, nn[1] /= l, nn[2] /= l;
  return ccd_extend(P, nn, p[3]);
}
// GJK: true with p a tetrahedron enclosing the origin (possibly on its boundary: gjk_complete);
// false apart (sep = a separating axis when a support plane proved it) or touching.  The
// thresholds are the oracle's (oracle_collision.c gjk_enclose), both in fp64.
HDI bool gjk_enclose(const MPair& P, MSup q[4], float sep[3]) {
  float c1[3], c2[3];
  geom_center(P.m, P.g1, P.P1, c1);
  geom_center(P.m, P.g2, P.P2, c2);
  double x[3] = {(double)c1[0] - c2[0], (double)c1[1] - c2[1], (double)c1[2] - c2[2]};
  if (dotd(x, x) == 0.0) x[0] = 1e-9;
  GSup p[4];
  int n = 0;
  double xx_prev = 1e300;
  bool in = false;
  for (int it = 0; it < CCD_ITERS; it++) {
    const double d[3] = {-x[0], -x[1], -x[2]};
    GSup s;
    gsup(P, d, s);
    const double xs = dotd(x, s.v);
    if (xs > 0.0) {  // every point of A - B has x.p >= x.s > 0: -x separates
      float a[3] = {(float)-x[0], (float)-x[1], (float)-x[2]};
      nrm(a);
      setsep(sep, a);
      return false;
    }
    if (dotd(x, x) - xs <= 1e-12) return false;  // no progress: the origin is on the boundary
#pragma unroll
    for (int k = 0; k < 4; k++) gsel(p[k], k == n, s);
    n++;
    if (n == 4) {
      const GSup t0 = p[0], t1 = p[1], t2 = p[2], t3 = p[3];
      const int r = tet_contains(p, x, n);
      if (r == 1) {
        in = true;
        break;
      }
      if (r < 0) {  // flat: the previous triangle p[0..2], completed if it carries the origin
        n = gjk_reduce(p, 3, x);
        if (!(dotd(x, x) < 1e-12 * dotd(s.v, s.v))) return false;
      } else if (!(dotd(x, x) < xx_prev)) {
        // no progress (the support along x returns a vertex already held): EPA from this
        // tetrahedron decides (a face with d < 0 at the end: apart)
        p[0] = t0, p[1] = t1, p[2] = t2, p[3] = t3;
        in = true;
        break;
      }
    } else {
      n = gjk_reduce(p, n, x);
    }
    xx_prev = dotd(x, x);
    // the origin on the simplex up to rounding (|x| < 1e-6 of the support point's scale)
    if (dotd(x, x) < 1e-12 * dotd(s.v, s.v)) {
      in = n >= 2 && gjk_complete(P, p, n);
      break;
    }
  }
  if (!in) return false;
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int c = 0; c < 3; c++)
      q[k].v[c] = (float)p[k].v[c], q[k].v1[c] = p[k].v1[c], q[k].v2[c] = p[k].v1[c] - q[k].v[c];
  return true;
}
// a face of the EPA polytope: unit outward normal and plane offset (one 16-byte load)
struct alignas(16) EpaPlane {
  float n[3], d;
};
HDI EpaPlane epa_plane(const float (*V)[6], int a, int b, int c) {
  EpaPlane f;
  float ab[3], ac[3];
  sub(ab, V[b], V[a]);
  sub(ac, V[c], V[a]);
  cross(f.n, ab, ac);
  nrm(f.n);
  f.d = dot3(f.n, V[a]);
  return f;
}
HDI uint32_t epa_abc(int a, int b, int c) { return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16); }
// the polytope of one EPA run (2.1 KB): faces as planes F and vertex ids A (8 bits each)
struct EpaPoly {
  float V[EPA_KV][6];  // v (3), geom1 support point (3)
  EpaPlane F[EPA_KF];
  uint32_t A[EPA_KF];
  uint8_t E[EPA_KE][2];
};
// k_collide<native>'s per-workgroup LDS slots for EPA polytopes (null on the host): an EPA run takes
// the next free slot and keeps its polytope in LDS instead of private (scratch) memory, whose every
// access is a round trip to the memory hierarchy; runs beyond the slots use private memory
struct EpaPool {
  EpaPoly* slot;
  int* used;
  int nslot;
};
// EPA from the enclosing tetrahedron p: 1 with depth / dir / pos.  Per expansion: the faces w sees
// as a bit mask from one pass of independent loads (unrolled, so the face / vertex loads of
// several faces are in flight together -- a face-by-face walk waited on two dependent LDS loads
// per face), the horizon from the seen faces in face order, then compaction with the running
// minimum, so the next closest face needs no scan of its own (same faces, same order and the same
// first-minimum rule as a scan: bit-identical)
HDI int epa(const MPair& P, const MSup p[4], float& depth, float dir[3], float pos[3], const EpaPool* pool = nullptr) {
  EpaPoly own;
  EpaPoly* Q = &own;
#if SOARM_DEVICE_PASS
  if (pool) {
    const int k = atomicAdd(pool->used, 1);
    if (k < pool->nslot) Q = pool->slot + k;
  }
#else
  (void)pool;
#endif
  float (*V)[6] = Q->V;
  EpaPlane* F = Q->F;
  uint32_t* A = Q->A;
  uint8_t (*E)[2] = Q->E;
#pragma unroll
  for (int k = 0; k < 4; k++) copy3(V[k], p[k].v), copy3(V[k] + 3, p[k].v1);
  int nv = 4, nf = 0, best = 0;
  float bd = 0.f;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int a = TETF[k][0], b = TETF[k][1], c = TETF[k][2];
    EpaPlane f = epa_plane(V, a, b, c);
    float ak[3];
    sub(ak, p[k].v, V[a]);
    if (dot3(f.n, ak) > 0.f) f = epa_plane(V, a, c, b), b = TETF[k][2], c = TETF[k][1];
    F[nf] = f, A[nf] = epa_abc(a, b, c);
    if (k == 0 || f.d < bd) bd = f.d, best = nf;
    nf++;
  }
  float upper = 3.0e38f;
  for (int it = 0; it < CCD_ITERS; it++) {
    const EpaPlane fb = F[best];
    MSup w;
    P.sup(fb.n, w);
    upper = fminf(upper, dot3(fb.n, w.v));
    if (upper - fb.d < MPR_TOLF || nv == EPA_KV) break;
    // faces seen from w go; the edges they do not share bound the hole (the horizon).  The
    // polytope is left untouched until the expansion is known to fit (a budget exit keeps it and
    // its closest face intact).
    uint64_t vis = 0ull;
#pragma unroll 8
    for (int i = 0; i < nf; i++) {
      const EpaPlane f = F[i];
      float aw[3];
      sub(aw, w.v, V[A[i] & 255]);
      if (dot3(f.n, aw) > EPA_VIS) vis |= 1ull << i;  // (w on a face's plane does not see it)
    }
    const int nvis = __builtin_popcountll(vis);
    int ne = 0;
    bool full = false;
    for (uint64_t r = vis; r; r &= r - 1) {
      const uint32_t abc = A[__builtin_ctzll(r)];
      const int a = abc & 255, b = (abc >> 8) & 255, c = (abc >> 16) & 255;
      const int ed[3][2] = {{a, b}, {b, c}, {c, a}};
#pragma unroll
      for (int q = 0; q < 3; q++) {
        int dup = -1;
        for (int k = 0; k < ne; k++)
          if (E[k][0] == ed[q][1] && E[k][1] == ed[q][0]) dup = k;
        if (dup >= 0) {
          E[dup][0] = E[ne - 1][0], E[dup][1] = E[ne - 1][1];
          ne--;
        } else if (ne < EPA_KE) {
          E[ne][0] = (uint8_t)ed[q][0], E[ne][1] = (uint8_t)ed[q][1];
          ne++;
        } else {
          full = true;
        }
      }
    }
    if (ne == 0 || full || nf - nvis + ne > EPA_KF) break;  // (budget exhausted: the best face so far)
    int m = 0;
    best = -1;
    for (int i = 0; i < nf; i++) {
      if ((vis >> i) & 1ull) continue;
      const EpaPlane f = F[i];
      if (m != i) F[m] = f, A[m] = A[i];
      if (best < 0 || f.d < bd) bd = f.d, best = m;
      m++;
    }
    nf = m;
    copy3(V[nv], w.v), copy3(V[nv] + 3, w.v1);
    for (int r = 0; r < ne; r++) {
      const EpaPlane f = epa_plane(V, E[r][0], E[r][1], nv);
      F[nf] = f, A[nf] = epa_abc(E[r][0], E[r][1], nv);
      if (best < 0 || f.d < bd) bd = f.d, best = nf;
      nf++;
    }
    nv++;
  }
  const EpaPlane f = F[best];
  const uint32_t abc = A[best];
  const int a = abc & 255, b = (abc >> 8) & 255, c = (abc >> 16) & 255;
  const float pr[3] = {f.d * f.n[0], f.d * f.n[1], f.d * f.n[2]};
  float v0[3], v1[3], v2[3];
  sub(v0, V[b], V[a]);
  sub(v1, V[c], V[a]);
  sub(v2, pr, V[a]);
  const float d00 = dot3(v0, v0), d01 = dot3(v0, v1), d11 = dot3(v1, v1), d20 = dot3(v2, v0), d21 = dot3(v2, v1);
  const float den = d00 * d11 - d01 * d01;
  if (!(den > 0.f)) return 0;
  const float lb = (d11 * d20 - d01 * d21) / den, lc = (d00 * d21 - d01 * d20) / den, la = 1.f - lb - lc;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float x1 = la * V[a][3 + k] + lb * V[b][3 + k] + lc * V[c][3 + k];
    pos[k] = x1 - 0.5f * pr[k];  // (x1 + x2) / 2 with x2 = x1 - pr
    dir[k] = f.n[k];
  }
  depth = f.d;
  return f.d > 0.f;
}
HDI int ccd_native(const MPair& P, float& depth, float dir[3], float pos[3], float sep[3], const EpaPool* pool = nullptr) {
  MSup p[4];
  if (!gjk_enclose(P, p, sep)) return 0;
#if defined(SOARM_DIAG_NO_EPA) && SOARM_DEVICE_PASS
  if (SOARM_DIAG_NO_EPA) return 0;  // (diagnostic build: GJK's cost alone)
#endif
  return epa(P, p, depth, dir, pos, pool);
}

// ------------------------------------------------------------- primitives
// append one contact (dropped past the pair's slot count)
HDI void emit(PairOut& o, float dist, const float pos[3], const float n[3]) {
  if (o.n >= o.cap) return;
  const int r = (o.s0 + o.n) * 7;
  soa(o.cbuf, r, o.nenv, o.e) = dist;
#pragma unroll
  for (int k = 0; k < 3; k++) soa(o.cbuf, r + 1 + k, o.nenv, o.e) = pos[k], soa(o.cbuf, r + 4 + k, o.nenv, o.e) = n[k];
  o.n++;
}

HDI void plane_box(const DModel& m, int gp, int gb, const GeomPose& Pp, const GeomPose& Pb, PairOut& o) {
  const float n[3] = {Pp.R[2], Pp.R[5], Pp.R[8]};
  int cnt = 0;
  for (int i = 0; i < 8 && cnt < 4; i++) {
    const float l[3] = {(i & 1 ? 1.f : -1.f) * m.geom_size[gb][0], (i & 2 ? 1.f : -1.f) * m.geom_size[gb][1],
                        (i & 4 ? 1.f : -1.f) * m.geom_size[gb][2]};
    float w[3], rel[3];
    mv(w, Pb.R, l);
    const float p[3] = {Pb.p[0] + w[0], Pb.p[1] + w[1], Pb.p[2] + w[2]};
    sub(rel, p, Pp.p);
    const float dist = dot3(rel, n);
    if (dist < 0.f) {
      const float pos[3] = {p[0] - 0.5f * dist * n[0], p[1] - 0.5f * dist * n[1], p[2] - 0.5f * dist * n[2]};
      emit(o, dist, pos, n);
      cnt++;
    }
  }
}

HDI void plane_convex(const DModel& m, int gp, int g, const GeomPose& Pp, const GeomPose& Pg, PairOut& o) {
  const float n[3] = {Pp.R[2], Pp.R[5], Pp.R[8]};
  const float nn[3] = {-n[0], -n[1], -n[2]};
  float p[3], rel[3];
  support(m, g, Pg, nn, p);
  sub(rel, p, Pp.p);
  const float dist = dot3(rel, n);
  if (dist >= 0.f) return;
  const float pos[3] = {p[0] - 0.5f * dist * n[0], p[1] - 0.5f * dist * n[1], p[2] - 0.5f * dist * n[2]};
  emit(o, dist, pos, n);
}

// Polygon clipping and box-box face selection keep every array in registers: loops over the
// (at most 8) polygon slots are unrolled, and lane-varying indices (the polygon size, the
// wrap-around neighbour, the next output slot, the reference face / incident axis) pick their
// element by selects over compile-time indices.  A dynamically indexed private array would
// live in scratch memory (k_collide had 656 B of scratch per lane).
// (value selects, v_cndmask: a conditional store `if (j == k) out[j] = x` is merged by the
// optimizer into one store through a computed index, which sends the array to scratch)
HDI void put8(float out[8][3], int k, const float x[3]) {
#pragma unroll
  for (int j = 0; j < 8; j++)
#pragma unroll
    for (int c = 0; c < 3; c++) out[j][c] = j == k ? x[c] : out[j][c];
}
template <int R>
HDI void row3(const float M[R][3], int i, float out[3]) {
#pragma unroll
  for (int c = 0; c < 3; c++) out[c] = M[0][c];
#pragma unroll
  for (int j = 1; j < R; j++)
#pragma unroll
    for (int c = 0; c < 3; c++) out[c] = j == i ? M[j][c] : out[c];
}
HDI float pick3(const float* h, int i) { return i == 0 ? h[0] : (i == 1 ? h[1] : h[2]); }

// one Sutherland-Hodgman step: keep the part of polygon in[0..n) with (x - o).a <= lim
HDI int clip_poly8(const float in[8][3], int n, float out[8][3], const float o[3], const float a[3], float lim) {
  float sd[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    float r[3];
    sub(r, in[i], o);
    sd[i] = dot3(r, a) - lim;
  }
  int k = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (i < n) {
      const bool wrap = i + 1 >= n;
      const float sp = sd[i], sq = wrap ? sd[0] : sd[(i + 1) & 7];
      const float Q[3] = {wrap ? in[0][0] : in[(i + 1) & 7][0], wrap ? in[0][1] : in[(i + 1) & 7][1],
                          wrap ? in[0][2] : in[(i + 1) & 7][2]};
      if (sp <= 0.f) {
        put8(out, k, in[i]);
        k++;
      }
      if ((sp < 0.f && sq > 0.f) || (sp > 0.f && sq < 0.f)) {
        const float t = sp / (sp - sq);
        const float X[3] = {in[i][0] + t * (Q[0] - in[i][0]), in[i][1] + t * (Q[1] - in[i][1]),
                            in[i][2] + t * (Q[2] - in[i][2])};
        put8(out, k, X);
        k++;
      }
    }
  }
  return k < 8 ? k : 8;
}

HDI void box_box(const DModel& m, int g1, int g2, const GeomPose& P1, const GeomPose& P2, PairOut& o) {
  const float *h1 = m.geom_size[g1], *h2 = m.geom_size[g2];
  float A[3][3], B[3][3], t[3];
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int e = 0; e < 3; e++) A[k][e] = P1.R[3 * e + k], B[k][e] = P2.R[3 * e + k];
  sub(t, P2.p, P1.p);
  float best = 3.0e38f, bn[3] = {0, 0, 0};
  int bcode = -1;
  bool sep = false;
#pragma unroll
  for (int code = 0; code < 15; code++) {  // unrolled: A / B rows by compile-time index
    float L[3];
    if (code < 3)
      L[0] = A[code][0], L[1] = A[code][1], L[2] = A[code][2];
    else if (code < 6)
      L[0] = B[code - 3][0], L[1] = B[code - 3][1], L[2] = B[code - 3][2];
    else
      cross(L, A[(code - 6) / 3], B[(code - 6) % 3]);
    const float ln = sqrtf(dot3(L, L));
    if (ln < 1e-6f) continue;  // parallel edges: no axis
    L[0] /= ln, L[1] /= ln, L[2] /= ln;
    float r1 = 0.f, r2 = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) r1 += h1[k] * fabsf(dot3(A[k], L)), r2 += h2[k] * fabsf(dot3(B[k], L));
    const float tl = dot3(t, L);
    const float ov = r1 + r2 - fabsf(tl);
    sep = sep || ov < 0.f;
    const float score = code < 6 ? ov : ov * 1.05f + 1e-9f;
    if (score < best) {
      best = score;
      bcode = code;
      const float sg = tl < 0.f ? -1.f : 1.f;
      bn[0] = sg * L[0], bn[1] = sg * L[1], bn[2] = sg * L[2];
    }
  }
  if (sep || bcode < 0) return;
  if (bcode < 6) {
    const bool ref1 = bcode < 3;
    const int fa = ref1 ? bcode : bcode - 3;
    float Ar[3][3], Ai[3][3], cr[3], ci[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      cr[k] = ref1 ? P1.p[k] : P2.p[k], ci[k] = ref1 ? P2.p[k] : P1.p[k];
#pragma unroll
      for (int e = 0; e < 3; e++) Ar[k][e] = ref1 ? A[k][e] : B[k][e], Ai[k][e] = ref1 ? B[k][e] : A[k][e];
    }
    const float* hr = ref1 ? h1 : h2;
    const float* hi = ref1 ? h2 : h1;
    float nr[3];
#pragma unroll
    for (int k = 0; k < 3; k++) nr[k] = ref1 ? bn[k] : -bn[k];
    const float hfa = pick3(hr, fa);
    float fc[3];
#pragma unroll
    for (int k = 0; k < 3; k++) fc[k] = cr[k] + nr[k] * hfa;
    int ia = 0;
    float bd = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float dd = fabsf(dot3(Ai[k], nr));
      if (dd > bd) bd = dd, ia = k;
    }
    float aia[3], au[3], av[3];
    const int u = (ia + 1) % 3, v = (ia + 2) % 3;
    row3<3>(Ai, ia, aia);
    row3<3>(Ai, u, au);
    row3<3>(Ai, v, av);
    const float s = dot3(aia, nr) > 0.f ? -1.f : 1.f;
    const float hia = pick3(hi, ia), hu = pick3(hi, u), hv = pick3(hi, v);
    float poly[8][3], tmp[8][3] = {};
    const float su[4] = {1, -1, -1, 1}, sv[4] = {1, 1, -1, -1};
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int k = 0; k < 3; k++) poly[q][k] = ci[k] + s * hia * aia[k] + su[q] * hu * au[k] + sv[q] * hv * av[k];
#pragma unroll
    for (int q = 4; q < 8; q++) poly[q][0] = poly[q][1] = poly[q][2] = 0.f;
    const int ra = (fa + 1) % 3, rb = (fa + 2) % 3;
    float ara[3], arb[3];
    row3<3>(Ar, ra, ara);
    row3<3>(Ar, rb, arb);
    const float hra = pick3(hr, ra), hrb = pick3(hr, rb);
    {
      // fast path (cube resting on the table): the incident face lies inside the reference
      // face's side slabs, so clipping is the identity; emit penetrating corners deepest first
      // (the same stable order as the general path), all with compile-time indices.
      bool inside = true;
      float dep[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        float rel[3];
        sub(rel, poly[q], fc);
        inside = inside && fabsf(dot3(rel, ara)) <= hra && fabsf(dot3(rel, arb)) <= hrb;
        dep[q] = dot3(rel, nr);
      }
      if (inside) {
        unsigned used = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          int best = -1;
          float bdep = 0.f;
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (!((used >> q) & 1u) && dep[q] < bdep) bdep = dep[q], best = q;
          if (best < 0) break;
          used |= 1u << best;
          float pos[3] = {0, 0, 0};
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (q == best)
#pragma unroll
              for (int k = 0; k < 3; k++) pos[k] = poly[q][k] - 0.5f * bdep * nr[k];
          emit(o, bdep, pos, bn);
        }
        return;
      }
    }
    int n = 4;
    float na[3];
    n = clip_poly8(poly, n, tmp, fc, ara, hra);
    na[0] = -ara[0], na[1] = -ara[1], na[2] = -ara[2];
    n = clip_poly8(tmp, n, poly, fc, na, hra);
    n = clip_poly8(poly, n, tmp, fc, arb, hrb);
    na[0] = -arb[0], na[1] = -arb[1], na[2] = -arb[2];
    n = clip_poly8(tmp, n, poly, fc, na, hrb);
    // penetrating vertices, deepest first (stable: ties keep polygon order), at most 4
    float dep[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      float rel[3];
      sub(rel, poly[q], fc);
      const float sd = dot3(rel, nr);
      dep[q] = (q < n && sd < 0.f) ? sd : 0.f;
    }
    unsigned used = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      int best = -1;
      float bdep = 0.f;
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (!((used >> q) & 1u) && dep[q] < bdep) bdep = dep[q], best = q;
      if (best < 0) break;
      used |= 1u << best;
      float pos[3] = {0, 0, 0};
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (q == best)
#pragma unroll
          for (int k = 0; k < 3; k++) pos[k] = poly[q][k] - 0.5f * bdep * nr[k];
      emit(o, bdep, pos, bn);
    }
    return;
  }
  // edge-edge (the edge rows picked by selects: a computed index into A / B would put them in scratch)
  const int ea = (bcode - 6) / 3, eb = (bcode - 6) % 3;
  float aea[3], beb[3];
  row3<3>(A, ea, aea);
  row3<3>(B, eb, beb);
  const float h1a = pick3(h1, ea), h2b = pick3(h2, eb);
  float p1[3] = {P1.p[0], P1.p[1], P1.p[2]}, p2[3] = {P2.p[0], P2.p[1], P2.p[2]};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (k != ea) {
      const float sg = dot3(A[k], bn) > 0.f ? 1.f : -1.f;
#pragma unroll
      for (int e = 0; e < 3; e++) p1[e] += sg * h1[k] * A[k][e];
    }
    if (k != eb) {
      const float sg = dot3(B[k], bn) > 0.f ? -1.f : 1.f;
#pragma unroll
      for (int e = 0; e < 3; e++) p2[e] += sg * h2[k] * B[k][e];
    }
  }
  float r[3];
  sub(r, p1, p2);
  const float b = dot3(aea, beb), c = dot3(aea, r), f = dot3(beb, r);
  const float den = 1.f - b * b;
  float sp = den > 1e-12f ? (b * f - c) / den : 0.f;
  float tp = b * sp + f;
  sp = fminf(fmaxf(sp, -h1a), h1a);
  tp = fminf(fmaxf(tp, -h2b), h2b);
  float pos[3];
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = 0.5f * (p1[k] + sp * aea[k] + p2[k] + tp * beb[k]);
  emit(o, -best / 1.05f, pos, bn);
}

// the env's body world frames (BREC floats each, bodies 1 .. NB-1); lane g0 of gstep writes the
// floats f = g0, g0 + gstep, ... of the env's record (f = (b - 1) * BREC + k, compile-time body and
// component: the frame is read with constant register indices)
template <int NA, int NF>
HDI void write_body_frames(const Sim<NA, NF>& S, float* __restrict__ gpose, int n, int e, int g0 = 0,
                           int gstep = 1) {
  constexpr int NB = Sim<NA, NF>::NB;
#pragma unroll
  for (int b = 1; b < NB; b++) {
#pragma unroll
    for (int k = 0; k < BREC; k++) {
      const int f = (b - 1) * BREC + k;
      if (f % gstep == g0) soa(gpose, b * BREC + k, n, e) = k < 3 ? S.xpos[b][k] : S.xmat[b][k - 3];
    }
  }
}
// the same from the env's 16 lanes via LDS (fr: 12 * NB floats of this env, free at this point): the
// frames are staged once, then lane g0 of gstep stores floats g0, g0 + gstep, ... -- one store
// instruction covers 16 consecutive floats of each of the wave's 4 envs
template <int NA, int NF>
__device__ __forceinline__ void write_body_frames_lds(const Sim<NA, NF>& S, float* __restrict__ gpose, int n,
                                                      int e, int g0, int gstep, float* fr) {
  constexpr int NB = Sim<NA, NF>::NB;
  // (every lane of the env writes the same values: one LDS store per float per env)
#pragma unroll
  for (int b = 1; b < NB; b++) {
#pragma unroll
    for (int c = 0; c < 3; c++) fr[b * BREC + c] = S.xpos[b][c];
#pragma unroll
    for (int c = 0; c < 9; c++) fr[b * BREC + 3 + c] = S.xmat[b][c];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  for (int f = BREC + g0; f < NB * BREC; f += gstep) soa(gpose, f, n, e) = fr[f];
}

// a body-frame point x in world coordinates from the env's frame of body b (b = 0: the world)
HDI void body_point(const DModel& m, const float* __restrict__ gpose, int n, int e, int b, const float x[3],
                    float w[3]) {
  if (b == 0) {
    w[0] = x[0], w[1] = x[1], w[2] = x[2];
    return;
  }
  float bR[9];
#pragma unroll
  for (int k = 0; k < 9; k++) bR[k] = soa(gpose, b * BREC + 3 + k, n, e);
  mv(w, bR, x);
#pragma unroll
  for (int k = 0; k < 3; k++) w[k] += soa(gpose, b * BREC + k, n, e);
}
// geom g's world pose from its body's frame (the world body: the geom's own placement)
HDI void load_pose(const DModel& m, const float* __restrict__ gpose, int n, int e, int g, GeomPose& o) {
  const int b = m.geom_bodyid[g];
  float bp[3] = {0.f, 0.f, 0.f}, bR[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f};
  if (b > 0) {
#pragma unroll
    for (int k = 0; k < 3; k++) bp[k] = soa(gpose, b * BREC + k, n, e);
#pragma unroll
    for (int k = 0; k < 9; k++) bR[k] = soa(gpose, b * BREC + 3 + k, n, e);
  }
  const float gp[3] = {m.geom_pos[g][0], m.geom_pos[g][1], m.geom_pos[g][2]};
  float w[3];
  mv(w, bR, gp);
  mm(o.R, bR, m.geom_mat[g]);
#pragma unroll
  for (int c = 0; c < 3; c++) o.p[c] = bp[c] + w[c];
}
// the midphase bound of geom g at pose P: the world centre of its collision box and that box's
// world-axis half-extents |R| h
HDI void geom_bound(const DModel& m, int g, const GeomPose& P, float c[3], float h[3]) {
  geom_center(m, g, P, c);
#pragma unroll
  for (int k = 0; k < 3; k++)
    h[k] = fabsf(P.R[3 * k]) * m.geom_half[g][0] + fabsf(P.R[3 * k + 1]) * m.geom_half[g][1] +
           fabsf(P.R[3 * k + 2]) * m.geom_half[g][2];
}

// midphase of candidate pair p from the env's body frames: bounding spheres and, for a plane, the
// other geom's bounding sphere above it (from the body frames alone), then world-aligned boxes of
// the composed poses.  false: no contact is possible; P1 / P2 are set when it returns true.
HDI bool midphase(const DModel& m, int p, const float* __restrict__ gpose, int n, int e, GeomPose& P1,
                   GeomPose& P2) {
  const int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
  if (m.geom_rbound[g1] > 0.f && m.geom_rbound[g2] > 0.f) {
    // bounding spheres first, from the body frames and the centres' body-frame offsets (no geom
    // pose composed for the ~80 of 86 pairs this rejects)
    float c1[3], c2[3], r[3];
    body_point(m, gpose, n, e, m.geom_bodyid[g1], m.geom_cbody[g1], c1);
    body_point(m, gpose, n, e, m.geom_bodyid[g2], m.geom_cbody[g2], c2);
    sub(r, c1, c2);
    const float rr = m.geom_rbound[g1] + m.geom_rbound[g2] + m.pair_margin[p];
    if (dot3(r, r) > rr * rr) return false;
  }
  if (m.geom_type[g1] == SIM_GEOM_PLANE && m.geom_rbound[g2] > 0.f) {
    // bounding sphere of geom2 entirely above the plane (beyond the margin): no contact
    float c2[3];
    body_point(m, gpose, n, e, m.geom_bodyid[g2], m.geom_cbody[g2], c2);
    load_pose(m, gpose, n, e, g1, P1);
    const float h = (c2[0] - P1.p[0]) * P1.R[2] + (c2[1] - P1.p[1]) * P1.R[5] + (c2[2] - P1.p[2]) * P1.R[8];
    if (h > m.geom_rbound[g2] + m.pair_margin[p]) return false;
  }
  load_pose(m, gpose, n, e, g1, P1);
  load_pose(m, gpose, n, e, g2, P2);
  if (m.geom_rbound[g1] > 0.f && m.geom_rbound[g2] > 0.f) {  // world-aligned boxes
    float c1[3], h1[3], c2[3], h2[3], r[3];
    geom_bound(m, g1, P1, c1, h1);
    geom_bound(m, g2, P2, c2, h2);
    sub(r, c1, c2);
    const float mg = m.pair_margin[p];
    bool sep = false;
#pragma unroll
    for (int k = 0; k < 3; k++) sep |= fabsf(r[k]) > h1[k] + h2[k] + mg;
    if (sep) return false;
  }
  return true;
}

// Separating-axis cache of one env's candidate pairs, [pair*3 + k][env]: the axis of the last
// MPR run that proved the pair apart (zero: none).  A pair whose cached axis still separates it
// (the support bounds along it leave a gap > SEP_MARGIN) is apart, exactly as MPR would find --
// any separating axis is a proof -- so the cache changes which pairs skip MPR, never a contact.
// Between substeps the geoms move by millimetres: a persistently separated near pair (the
// wrist/jaw meshes, the jaw above the cube) skips its MPR run on nearly every substep.
struct SepCache {
  float* a;  // null: no cache (the fused-collide build)
  int n, e;
  HDI void load(int p, float d[3]) const {
#pragma unroll
    for (int k = 0; k < 3; k++) d[k] = a ? soa(a, 3 * p + k, n, e) : 0.f;
  }
  HDI void store(int p, const float d[3]) const {
    if (!a) return;
#pragma unroll
    for (int k = 0; k < 3; k++) soa(a, 3 * p + k, n, e) = d[k];
  }
};
// upper bound on geom g's support value along the local direction l (box: exact)
HDI float support_ub_any(const DModel& m, int g, const float l[3]) {
  if (m.geom_type[g] == SIM_GEOM_BOX)
    return fabsf(l[0]) * m.geom_size[g][0] + fabsf(l[1]) * m.geom_size[g][1] + fabsf(l[2]) * m.geom_size[g][2];
  return support_ub(m, g, l);
}
// upper bound on max over (geom1 - geom2) of x.d: below zero proves the pair apart along d
HDI float minkowski_ub(const DModel& m, int g1, int g2, const GeomPose& P1, const GeomPose& P2, const float d[3]) {
  float l1[3], l2[3];
  mtv(l1, P1.R, d);
  mtv(l2, P2.R, d);
  l2[0] = -l2[0], l2[1] = -l2[1], l2[2] = -l2[2];
  return (P1.p[0] - P2.p[0]) * d[0] + (P1.p[1] - P2.p[1]) * d[1] + (P1.p[2] - P2.p[2]) * d[2] +
         support_ub_any(m, g1, l1) + support_ub_any(m, g2, l2);
}
// the cached axis of pair p still separates it
HDI bool cached_apart(const DModel& m, int p, int g1, int g2, const GeomPose& P1, const GeomPose& P2,
                       const SepCache& sc) {
  float d[3];
  sc.load(p, d);
  if (d[0] == 0.f && d[1] == 0.f && d[2] == 0.f) return false;
  return minkowski_ub(m, g1, g2, P1, P2, d) < -(m.pair_margin[p] + SEP_MARGIN);
}

// narrowphase of a pair that passed the midphase (geom types are uniform over a pair); CCD: the
// convex-convex narrowphase fixed at compile time (SIM_CCD_*), or -1 to read it from the model
template <int CCD = -1>
HDI void narrowphase(const DModel& m, int p, const GeomPose& P1, const GeomPose& P2, PairOut& o,
                      const SepCache& sc, const EpaPool* pool = nullptr) {
  o.n = 0;
  o.xc = 6;
  const int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
  const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  if (t1 == SIM_GEOM_PLANE) {
    if (t2 == SIM_GEOM_BOX)
      plane_box(m, g1, g2, P1, P2, o);
    else if (t2 == SIM_GEOM_MESH)
      plane_convex(m, g1, g2, P1, P2, o);
    return;
  }
  if (t1 == SIM_GEOM_BOX && t2 == SIM_GEOM_BOX) {
    box_box(m, g1, g2, P1, P2, o);
    return;
  }
  if (t1 == SIM_GEOM_BOX && t2 == SIM_GEOM_MESH) {
    // separating-axis pre-test on the box face that faces the hull's centre most: if
    // the hull's extreme point toward the box lies beyond that face, they are apart
    // (exact; MPR would find no contact).  One support query instead of an MPR run.
    float c2[3];
    geom_center(m, g2, P2, c2);
    const float r[3] = {c2[0] - P1.p[0], c2[1] - P1.p[1], c2[2] - P1.p[2]};
    float best = -3.0e38f, ax[3] = {0.f, 0.f, 1.f}, h = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float a[3] = {P1.R[k], P1.R[3 + k], P1.R[6 + k]};
      const float dk = dot3(r, a);
      const float gap = fabsf(dk) - m.geom_size[g1][k];
      if (gap > best) {
        const float sg = dk >= 0.f ? 1.f : -1.f;
        best = gap, h = m.geom_size[g1][k];
        ax[0] = sg * a[0], ax[1] = sg * a[1], ax[2] = sg * a[2];
      }
    }
    const float nd[3] = {-ax[0], -ax[1], -ax[2]};
    {  // the same test on the support bound first: no hull data when it already separates
      const float l[3] = {P2.R[0] * nd[0] + P2.R[3] * nd[1] + P2.R[6] * nd[2],
                          P2.R[1] * nd[0] + P2.R[4] * nd[1] + P2.R[7] * nd[2],
                          P2.R[2] * nd[0] + P2.R[5] * nd[1] + P2.R[8] * nd[2]};
      const float lo = -support_ub(m, g2, l) + (P2.p[0] - P1.p[0]) * ax[0] + (P2.p[1] - P1.p[1]) * ax[1] +
                       (P2.p[2] - P1.p[2]) * ax[2] - h;  // <= the hull's distance beyond the face
      if (lo > m.pair_margin[p] + SEP_MARGIN) return (void)(o.xc = 1);
    }
    if (cached_apart(m, p, g1, g2, P1, P2, sc)) return (void)(o.xc = 2);
    float sp[3];
    support(m, g2, P2, nd, sp);
    const float dist = (sp[0] - P1.p[0]) * ax[0] + (sp[1] - P1.p[1]) * ax[1] + (sp[2] - P1.p[2]) * ax[2] - h;
    if (dist > m.pair_margin[p]) return (void)(o.xc = 1);
  }
  if (t1 == SIM_GEOM_MESH && t2 == SIM_GEOM_MESH) {
    // MPR's first test on support bounds: along d = c2 - c1 (MPR's first search direction) the
    // Minkowski difference reaches at most ub = h1(d) + h2(-d); ub < 0 proves the hulls apart,
    // exactly where MPR would stop at its first support point (discover's first `dt < 0`), but
    // without the two hull support queries (persistently separated near pairs such as the
    // wrist/jaw meshes otherwise cost the collide kernel its longest waves)
    float c1[3], c2[3];
    geom_center(m, g1, P1, c1);
    geom_center(m, g2, P2, c2);
    float d[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
    const float n2 = dot3(d, d);
    if (n2 > 1e-20f) {
      const float inv = frsqrt(n2);
      d[0] *= inv, d[1] *= inv, d[2] *= inv;
      const float l1[3] = {P1.R[0] * d[0] + P1.R[3] * d[1] + P1.R[6] * d[2],
                           P1.R[1] * d[0] + P1.R[4] * d[1] + P1.R[7] * d[2],
                           P1.R[2] * d[0] + P1.R[5] * d[1] + P1.R[8] * d[2]};
      const float l2[3] = {-(P2.R[0] * d[0] + P2.R[3] * d[1] + P2.R[6] * d[2]),
                           -(P2.R[1] * d[0] + P2.R[4] * d[1] + P2.R[7] * d[2]),
                           -(P2.R[2] * d[0] + P2.R[5] * d[1] + P2.R[8] * d[2])};
      const float ub = (P1.p[0] - P2.p[0]) * d[0] + (P1.p[1] - P2.p[1]) * d[1] + (P1.p[2] - P2.p[2]) * d[2] +
                       support_ub(m, g1, l1) + support_ub(m, g2, l2);
      if (ub < -SEP_MARGIN) return (void)(o.xc = 1);
    }
    if (cached_apart(m, p, g1, g2, P1, P2, sc)) return (void)(o.xc = 2);
  }
  MPair mp{m, g1, g2, P1, P2};
  float depth, dir[3], pos[3], sep[3] = {0.f, 0.f, 0.f};
  const bool native = CCD < 0 ? m.ccd == SIM_CCD_NATIVE : CCD == SIM_CCD_NATIVE;
  if (native ? ccd_native(mp, depth, dir, pos, sep, pool) : mpr(mp, depth, dir, pos, sep)) {
    emit(o, -depth, pos, dir);
    o.xc = 5;
  } else {
    o.xc = (sep[0] != 0.f || sep[1] != 0.f || sep[2] != 0.f) ? 3 : 4;
  }
  sc.store(p, sep);
}

}  // namespace soarm

namespace soarm {
// midphase + narrowphase of candidate pair p of env e (geom records in gpose)
template <int CCD = -1>
HDI void collide_pair(const DModel& m, int p, const float* __restrict__ gpose, int n, int e, PairOut& o,
                       const SepCache& sc = SepCache{nullptr, 0, 0}, const EpaPool* pool = nullptr) {
  o.n = 0;
#if defined(SOARM_DIAG_SUPPORT) && !SOARM_DEVICE_PASS
  g_diag_prev_host[0] = g_diag_prev_host[1] = ~0u;
#endif
  GeomPose P1, P2;
  if (midphase(m, p, gpose, n, e, P1, P2)) narrowphase<CCD>(m, p, P1, P2, o, sc, pool);
}
}  // namespace soarm
