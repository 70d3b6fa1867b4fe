/*
 * oracle_collision.c — float64 restatement of mj_collision for the hot-path
 * scenes.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * [ext] MuJoCo engine_collision_driver.c / engine_collision_convex.c /
 * engine_collision_box.c / engine_collision_primitive.c, libccd mpr.c:
 *  - candidate pairs come pre-filtered and pre-ordered from the compiler
 *    (sim_model_desc.pair_geom1/2); the midphase is MuJoCo's bounding-sphere
 *    test about the geom's collision centre (rbound + margin);
 *  - convex-convex (mesh hull / box vs mesh hull): native GJK/EPA (MuJoCo's
 *    nativeccd, sim_model_desc.ccd = SIM_CCD_NATIVE, the default of current
 *    releases; see below) or MPR (libccd, SIM_CCD_MPR) penetration with
 *    tolerance 1e-6 and 50 iterations (MuJoCo's defaults), one contact per
 *    pair, dist = -depth, normal geom1 -> geom2, pos = midpoint of the two
 *    witness points;
 *  - box-box: separating-axis test over 15 axes, reference-face clipping of
 *    the incident face (<= 4 contacts, deepest kept) or one edge-edge contact;
 *  - plane-box: penetrating corners (<= 4); plane-convex: deepest hull vertex.
 * Hull support is exact (brute-force argmax over the hull vertices; the
 * product kernel hill-climbs the hull graph to the same vertex).
 */
#include <math.h>
#include <string.h>

#include "oracle.h"

#define EPS 2.220446049250313e-16
#define MPR_TOL 1e-6
#define MPR_ITER 50

/* algorithmic flop counter for collision work (SURVEY.md §8d binding procedure) */
static __thread double g_cflops;
/* collision statistics (diagnostic): [0] pairs tested, [1] midphase passes,
   [2] MPR calls, [3] MPR hits, [4] support calls, [5] hull climb steps, [6] box-box, [7] plane */
static double g_cstat[8];
static double g_pstat[SIM_MAXPAIR][2]; /* per pair: midphase passes, support calls */
static __thread int g_curpair = -1;

static double dot3(const double a[3], const double b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void sub3(double r[3], const double a[3], const double b[3]) {
  r[0] = a[0] - b[0];
  r[1] = a[1] - b[1];
  r[2] = a[2] - b[2];
}
static double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
static void normalize3(double a[3]) {
  double n = norm3(a);
  if (n > 0) {
    a[0] /= n;
    a[1] /= n;
    a[2] /= n;
  }
}
static int is_zero(double x) { return fabs(x) < EPS; }
static int approx_eq(double a, double b) {
  double ab = fabs(a - b);
  if (ab < EPS) return 1;
  double fa = fabs(a), fb = fabs(b);
  return ab < EPS * (fa > fb ? fa : fb);
}
/* column k of a row-major rotation = local axis k in world */
static void col(double r[3], const double R[9], int k) {
  r[0] = R[k];
  r[1] = R[3 + k];
  r[2] = R[6 + k];
}

/* ------------------------------------------------------------- geometry */
static void geom_center(const orc_model* om, const orc_data* d, int g, double c[3]) {
  const double* a = om->m->geom_aabb[g];
  const double* R = d->geom_xmat[g];
  for (int k = 0; k < 3; k++)
    c[k] = d->geom_xpos[g][k] + R[3 * k] * a[0] + R[3 * k + 1] * a[1] + R[3 * k + 2] * a[2];
}

/* Support vertex of a mesh geom's hull for a LOCAL direction: steepest-ascent
   hill climbing over the hull's vertex graph from the best precomputed seed (on a convex hull a
   local maximum of a linear function is global).  With graph == NULL this is
   the brute-force argmax used to test the climber. */
int orc_hull_support_ex(const orc_model* om, int g, const double l[3], int use_graph) {
  const sim_model_desc* m = om->m;
  const float* v = om->hull_vert + 3 * (size_t)m->geom_hulladr[g];
  int nvert = m->geom_hullnum[g];
  if (!use_graph || !om->hull_adr) {
    int best = 0;
    double bd = -1e300;
    for (int i = 0; i < nvert; i++) {
      double s = l[0] * v[3 * i] + l[1] * v[3 * i + 1] + l[2] * v[3 * i + 2];
      if (s > bd) {
        bd = s;
        best = i;
      }
    }
    return best;
  }
  const int32_t* adr = om->hull_adr + m->geom_hulladr[g];
  int cur = 0;
  double cd = l[0] * v[0] + l[1] * v[1] + l[2] * v[2];
  g_cflops += 5;
  if (om->hull_seed) { /* start from the best seed (the same exact argmax is reached) */
    const int32_t* sd = om->hull_seed + g * ORC_NSEED;
    cur = sd[0];
    cd = l[0] * v[3 * cur] + l[1] * v[3 * cur + 1] + l[2] * v[3 * cur + 2];
    for (int k = 1; k < ORC_NSEED; k++) {
      int s = sd[k];
      double t = l[0] * v[3 * s] + l[1] * v[3 * s + 1] + l[2] * v[3 * s + 2];
      if (t > cd) {
        cd = t;
        cur = s;
      }
    }
    g_cflops += 5.0 * ORC_NSEED;
  }
  g_cstat[4] += 1;
  if (g_curpair >= 0) g_pstat[g_curpair][1] += 1;
  for (int guard = 0; guard < nvert; guard++) {
    int nxt = cur;
    double nd = cd;
    g_cstat[5] += 1;
    g_cflops += 5.0 * (adr[cur + 1] - adr[cur]);
    for (int a = adr[cur]; a < adr[cur + 1]; a++) {
      int u = om->hull_adj[a];
      double s = l[0] * v[3 * u] + l[1] * v[3 * u + 1] + l[2] * v[3 * u + 2];
      if (s > nd) {
        nd = s;
        nxt = u;
      }
    }
    if (nxt == cur) break;
    cur = nxt;
    cd = nd;
  }
  return cur;
}
int orc_hull_support(const orc_model* om, int g, const double l[3]) {
  return orc_hull_support_ex(om, g, l, 1);
}

/* seeds: for each of ORC_NSEED Fibonacci-sphere directions the brute-force
   argmax hull vertex (ties -> lowest index) */
void orc_hull_seeds(const sim_model_desc* m, const float* hv, int32_t* seeds) {
  for (int g = 0; g < m->ngeom; g++) {
    for (int k = 0; k < ORC_NSEED; k++) seeds[g * ORC_NSEED + k] = 0;
    if (m->geom_type[g] != SIM_GEOM_MESH) continue;
    const float* v = hv + 3 * (size_t)m->geom_hulladr[g];
    for (int k = 0; k < ORC_NSEED; k++) {
      double z = 1.0 - (2.0 * k + 1.0) / ORC_NSEED, r = sqrt(1.0 - z * z), ph = k * 2.399963229728653;
      double d[3] = {r * cos(ph), r * sin(ph), z}, bd = -1e300;
      int best = 0;
      for (int i = 0; i < m->geom_hullnum[g]; i++) {
        double s = d[0] * v[3 * i] + d[1] * v[3 * i + 1] + d[2] * v[3 * i + 2];
        if (s > bd) {
          bd = s;
          best = i;
        }
      }
      seeds[g * ORC_NSEED + k] = best;
    }
  }
}

/* world-frame support point of geom g in direction dir */
static void support(const orc_model* om, const orc_data* d, int g, const double dir[3],
                    double out[3]) {
  const sim_model_desc* m = om->m;
  const double* R = d->geom_xmat[g];
  double l[3] = {R[0] * dir[0] + R[3] * dir[1] + R[6] * dir[2],
                 R[1] * dir[0] + R[4] * dir[1] + R[7] * dir[2],
                 R[2] * dir[0] + R[5] * dir[1] + R[8] * dir[2]};
  double p[3] = {0, 0, 0};
  switch (m->geom_type[g]) {
    case SIM_GEOM_BOX:
      for (int k = 0; k < 3; k++) p[k] = (l[k] >= 0 ? 1 : -1) * m->geom_size[g][k];
      break;
    case SIM_GEOM_SPHERE: {
      double n = norm3(l);
      for (int k = 0; k < 3; k++) p[k] = n > 0 ? l[k] / n * m->geom_size[g][0] : 0;
      break;
    }
    case SIM_GEOM_MESH: {
      int best = orc_hull_support(om, g, l);
      const float* v = om->hull_vert + 3 * ((size_t)m->geom_hulladr[g] + best);
      for (int k = 0; k < 3; k++) p[k] = v[k];
      break;
    }
    default:
      break;
  }
  for (int k = 0; k < 3; k++)
    out[k] = d->geom_xpos[g][k] + R[3 * k] * p[0] + R[3 * k + 1] * p[1] + R[3 * k + 2] * p[2];
}

/* ------------------------------------------------------------------ MPR */
typedef struct {
  double v[3], v1[3], v2[3];
} msup;

typedef struct {
  const orc_model* om;
  const orc_data* d;
  int g1, g2;
} mpair;

static void msupport(const mpair* P, const double dir[3], msup* s) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  g_cflops += 2 * 36.0 + 3 + 40; /* two frame transforms, difference, portal bookkeeping */
  support(P->om, P->d, P->g1, dir, s->v1);
  support(P->om, P->d, P->g2, nd, s->v2);
  sub3(s->v, s->v1, s->v2);
}

/* normal of the portal face (v1, v2, v3), pointing away from v0 */
static void portal_dir(const msup* p, double dir[3]) {
  double a[3], b[3];
  sub3(a, p[2].v, p[1].v);
  sub3(b, p[3].v, p[1].v);
  cross3(dir, a, b);
  normalize3(dir);
}

/* returns -1 separated, 0 portal found, 1 origin on v1, 2 origin on v0-v1 */
static int discover_portal(const mpair* P, msup* p) {
  double c1[3], c2[3], dir[3], va[3], vb[3];
  geom_center(P->om, P->d, P->g1, c1);
  geom_center(P->om, P->d, P->g2, c2);
  memcpy(p[0].v1, c1, sizeof(c1));
  memcpy(p[0].v2, c2, sizeof(c2));
  sub3(p[0].v, c1, c2);
  if (is_zero(p[0].v[0]) && is_zero(p[0].v[1]) && is_zero(p[0].v[2])) p[0].v[0] += 10 * EPS;

  for (int k = 0; k < 3; k++) dir[k] = -p[0].v[k];
  normalize3(dir);
  msupport(P, dir, &p[1]);
  double dt = dot3(p[1].v, dir);
  if (is_zero(dt) || dt < 0) return -1;

  cross3(dir, p[0].v, p[1].v);
  if (is_zero(dot3(dir, dir))) {
    if (is_zero(p[1].v[0]) && is_zero(p[1].v[1]) && is_zero(p[1].v[2])) return 1;
    return 2;
  }
  normalize3(dir);
  msupport(P, dir, &p[2]);
  dt = dot3(p[2].v, dir);
  if (is_zero(dt) || dt < 0) return -1;

  sub3(va, p[1].v, p[0].v);
  sub3(vb, p[2].v, p[0].v);
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, p[0].v) > 0) {
    msup t = p[1];
    p[1] = p[2];
    p[2] = t;
    for (int k = 0; k < 3; k++) dir[k] = -dir[k];
  }
  for (int guard = 0; guard < 1000; guard++) {
    msupport(P, dir, &p[3]);
    dt = dot3(p[3].v, dir);
    if (is_zero(dt) || dt < 0) return -1;
    int cont = 0;
    cross3(va, p[1].v, p[3].v);
    dt = dot3(va, p[0].v);
    if (dt < 0 && !is_zero(dt)) {
      p[2] = p[3];
      cont = 1;
    }
    if (!cont) {
      cross3(va, p[3].v, p[2].v);
      dt = dot3(va, p[0].v);
      if (dt < 0 && !is_zero(dt)) {
        p[1] = p[3];
        cont = 1;
      }
    }
    if (!cont) return 0;
    sub3(va, p[1].v, p[0].v);
    sub3(vb, p[2].v, p[0].v);
    cross3(dir, va, vb);
    normalize3(dir);
  }
  return -1;
}

static int reach_tolerance(const msup* p, const msup* v4, const double dir[3]) {
  double d4 = dot3(v4->v, dir);
  double a = d4 - dot3(p[1].v, dir), b = d4 - dot3(p[2].v, dir), c = d4 - dot3(p[3].v, dir);
  double mn = a < b ? a : b;
  mn = mn < c ? mn : c;
  return approx_eq(mn, MPR_TOL) || mn < MPR_TOL;
}

static void expand_portal(msup* p, const msup* v4) {
  double x[3];
  cross3(x, v4->v, p[0].v);
  if (dot3(p[1].v, x) > 0) {
    if (dot3(p[2].v, x) > 0)
      p[1] = *v4;
    else
      p[3] = *v4;
  } else {
    if (dot3(p[3].v, x) > 0)
      p[2] = *v4;
    else
      p[1] = *v4;
  }
}

static int refine_portal(const mpair* P, msup* p) {
  double dir[3];
  for (int it = 0; it < 1000; it++) {
    portal_dir(p, dir);
    double dt = dot3(dir, p[1].v);
    if (is_zero(dt) || dt > 0) return 0; /* origin inside the portal */
    msup v4;
    msupport(P, dir, &v4);
    double d4 = dot3(v4.v, dir);
    if (!(is_zero(d4) || d4 > 0) || reach_tolerance(p, &v4, dir)) return -1;
    expand_portal(p, &v4);
  }
  return -1;
}

/* closest point to the origin on triangle (a, b, c) */
static void closest_on_triangle(const double a[3], const double b[3], const double c[3],
                                double out[3]) {
  double ab[3], ac[3], ap[3];
  sub3(ab, b, a);
  sub3(ac, c, a);
  for (int k = 0; k < 3; k++) ap[k] = -a[k];
  double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) {
    memcpy(out, a, 3 * sizeof(double));
    return;
  }
  double bp[3] = {-b[0], -b[1], -b[2]};
  double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) {
    memcpy(out, b, 3 * sizeof(double));
    return;
  }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    double v = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) out[k] = a[k] + v * ab[k];
    return;
  }
  double cp[3] = {-c[0], -c[1], -c[2]};
  double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) {
    memcpy(out, c, 3 * sizeof(double));
    return;
  }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    double w = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) out[k] = a[k] + w * ac[k];
    return;
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) out[k] = b[k] + w * (c[k] - b[k]);
    return;
  }
  double den = 1.0 / (va + vb + vc);
  double v = vb * den, w = vc * den;
  for (int k = 0; k < 3; k++) out[k] = a[k] + ab[k] * v + ac[k] * w;
}

/* contact position: barycentric weights of the origin in the final portal
   tetrahedron (or its face), applied to the witness points of both shapes */
static void portal_pos(const msup* p, double pos[3]) {
  double dir[3], x[3], b[4];
  portal_dir(p, dir);
  cross3(x, p[1].v, p[2].v);
  b[0] = dot3(x, p[3].v);
  cross3(x, p[3].v, p[2].v);
  b[1] = dot3(x, p[0].v);
  cross3(x, p[0].v, p[1].v);
  b[2] = dot3(x, p[3].v);
  cross3(x, p[2].v, p[1].v);
  b[3] = dot3(x, p[0].v);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (is_zero(sum) || sum < 0) {
    b[0] = 0;
    cross3(x, p[2].v, p[3].v);
    b[1] = dot3(x, dir);
    cross3(x, p[3].v, p[1].v);
    b[2] = dot3(x, dir);
    cross3(x, p[1].v, p[2].v);
    b[3] = dot3(x, dir);
    sum = b[1] + b[2] + b[3];
  }
  double inv = 1.0 / sum, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) {
      p1[k] += b[i] * p[i].v1[k];
      p2[k] += b[i] * p[i].v2[k];
    }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] + p2[k]) * inv;
}

/* MPR penetration: returns 1 with depth >= 0, dir (geom1 -> geom2), pos */
static int mpr_penetration(const mpair* P, double* depth, double dir[3], double pos[3]) {
  msup p[4];
  int res = discover_portal(P, p);
  if (res < 0 || res == 1) return 0;
  if (res == 2) {
    /* origin on segment v0-v1 */
    *depth = norm3(p[1].v);
    memcpy(dir, p[1].v, 3 * sizeof(double));
    normalize3(dir);
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].v1[k] + p[1].v2[k]);
    return *depth > 0;
  }
  if (refine_portal(P, p) < 0) return 0;
  for (int it = 0;; it++) {
    double pd[3];
    portal_dir(p, pd);
    msup v4;
    msupport(P, pd, &v4);
    if (reach_tolerance(p, &v4, pd) || it > MPR_ITER) {
      double w[3];
      closest_on_triangle(p[1].v, p[2].v, p[3].v, w);
      *depth = norm3(w);
      if (is_zero(*depth)) return 0;
      for (int k = 0; k < 3; k++) dir[k] = w[k] / *depth;
      portal_pos(p, pos);
      return 1;
    }
    expand_portal(p, &v4);
  }
}

/* ----------------------------------------------------- native GJK / EPA */
/* [ext] MuJoCo engine_collision_gjk.c (mjc_ccd, "nativeccd": the convex-convex default of
   current MuJoCo releases; opt.ccd_tolerance 1e-6, opt.ccd_iterations 50), restated by
   algorithm: GJK on the Minkowski difference A - B (support s = sA(d) - sB(-d)) from the
   difference of the shapes' centres, stopping as soon as a support plane separates the
   origin (no contact: margin 0) or a tetrahedron encloses it; then EPA (expanding polytope)
   from that tetrahedron: per iteration the face closest to the origin (a lower bound of the
   penetration depth) is expanded by the support point along its normal (an upper bound),
   until upper - lower < tolerance.  Contact: depth = the closest face's distance, normal = its
   outward normal (geom1 -> geom2), witness points x1, x2 = the barycentric weights of the
   origin's projection on that face applied to the two shapes' support points, pos = (x1+x2)/2.
   GJK may end with the origin ON a segment or triangle of its simplex (centred symmetric
   shapes: the second support point is exactly minus the first).  nativeccd then builds EPA's
   start from that simplex (polytope2 / polytope3); gjk_complete restates it as adding a support
   point off the simplex's span per missing dimension, giving a tetrahedron with the origin on
   its boundary, from which EPA expands as usual.  A lone vertex at the origin, or no extent off
   the span in either direction, is a touching configuration: no contact. */
#define CCD_TOL 1e-6
#define CCD_ITER 50
#define EPA_MAXV (4 + CCD_ITER)
#define EPA_MAXF (2 * EPA_MAXV)

typedef struct {
  int a, b, c, live;
  double n[3], d;
} epa_face;

/* closest point to the origin on the simplex p[0..n-1] (n <= 3); keeps in p only the vertices
   of the sub-simplex that carries it (Ericson's Voronoi-region tests).  Returns its size. */
static int gjk_reduce(msup* p, int n, double x[3]) {
  if (n == 1) {
    memcpy(x, p[0].v, sizeof(double) * 3);
    return 1;
  }
  if (n == 2) {
    double ab[3], t;
    sub3(ab, p[1].v, p[0].v);
    t = -dot3(p[0].v, ab);
    double l2 = dot3(ab, ab);
    if (t <= 0 || l2 <= 0) {
      memcpy(x, p[0].v, sizeof(double) * 3);
      return 1;
    }
    if (t >= l2) {
      p[0] = p[1];
      memcpy(x, p[0].v, sizeof(double) * 3);
      return 1;
    }
    t /= l2;
    for (int k = 0; k < 3; k++) x[k] = p[0].v[k] + t * ab[k];
    return 2;
  }
  /* triangle: regions of a, b, c, edges, face */
  const double *a = p[0].v, *b = p[1].v, *c = p[2].v;
  double ab[3], ac[3], ap[3] = {-a[0], -a[1], -a[2]};
  sub3(ab, b, a);
  sub3(ac, c, a);
  double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) {
    memcpy(x, a, sizeof(double) * 3);
    return 1;
  }
  double bp[3] = {-b[0], -b[1], -b[2]};
  double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) {
    p[0] = p[1];
    memcpy(x, b, sizeof(double) * 3);
    return 1;
  }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    double t = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) x[k] = a[k] + t * ab[k];
    return 2; /* a, b */
  }
  double cp[3] = {-c[0], -c[1], -c[2]};
  double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) {
    p[0] = p[2];
    memcpy(x, c, sizeof(double) * 3);
    return 1;
  }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    double t = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) x[k] = a[k] + t * ac[k];
    p[1] = p[2];
    return 2; /* a, c */
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) x[k] = b[k] + t * (c[k] - b[k]);
    p[0] = p[2]; /* b, c */
    return 2;
  }
  double den = 1.0 / (va + vb + vc), v = vb * den, w = vc * den;
  for (int k = 0; k < 3; k++) x[k] = a[k] + ab[k] * v + ac[k] * w;
  return 3;
}

/* 1 if the origin lies inside tetrahedron p[0..3] (strictly, up to rounding); else the index
   of a face whose plane separates it: the simplex is reduced to that face (returned 3-simplex
   with the origin on its outer side) */
static int tet_contains(msup* p, double x[3], int* nout) {
  /* face k = the three vertices other than k; outward = away from vertex k */
  static const int F[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};
  double best = 0;
  int bk = -1;
  for (int k = 0; k < 4; k++) {
    const double *a = p[F[k][0]].v, *b = p[F[k][1]].v, *c = p[F[k][2]].v;
    double ab[3], ac[3], n[3];
    sub3(ab, b, a);
    sub3(ac, c, a);
    cross3(n, ab, ac);
    double ak[3];
    sub3(ak, p[k].v, a);
    if (dot3(n, ak) > 0) for (int q = 0; q < 3; q++) n[q] = -n[q];
    double ln = norm3(n);
    if (ln <= 0) return -1; /* flat */
    double s = -dot3(n, a) / ln; /* > 0: origin outside this face */
    if (s > best) {
      best = s;
      bk = k;
    }
  }
  if (bk < 0) return 1;
  msup t[3] = {p[F[bk][0]], p[F[bk][1]], p[F[bk][2]]};
  p[0] = t[0], p[1] = t[1], p[2] = t[2];
  *nout = gjk_reduce(p, 3, x);
  return 0;
}

/* support point along d or, when the Minkowski difference has no extent along d beyond the
   tolerance, along -d (d is negated then); 0 if neither */
static int ccd_extend(const mpair* P, double d[3], msup* s) {
  msupport(P, d, s);
  if (dot3(d, s->v) > CCD_TOL) return 1;
  for (int k = 0; k < 3; k++) d[k] = -d[k];
  msupport(P, d, s);
  return dot3(d, s->v) > CCD_TOL;
}

/* the origin lies on the segment p[0..1] (n = 2) or the triangle p[0..2] (n = 3): complete a
   tetrahedron p[0..3] around it (the origin on its boundary); 0 when touching */
static int gjk_complete(const mpair* P, msup* p, int n) {
  if (n == 2) { /* a direction normal to the segment: u x (the axis of u's smallest component) */
    double u[3], e[3] = {0, 0, 0}, d[3];
    sub3(u, p[1].v, p[0].v);
    const double ax = fabs(u[0]), ay = fabs(u[1]), az = fabs(u[2]);
    e[ax <= ay && ax <= az ? 0 : ay <= az ? 1 : 2] = 1;
    cross3(d, u, e);
    if (!(norm3(d) > 0)) return 0;
    normalize3(d);
    if (!ccd_extend(P, d, &p[2])) return 0;
  }
  double ab[3], ac[3], nn[3];
  sub3(ab, p[1].v, p[0].v);
  sub3(ac, p[2].v, p[0].v);
  cross3(nn, ab, ac);
  if (!(norm3(nn) > 0)) return 0;
  normalize3(nn);
  return ccd_extend(P, nn, &p[3]);
}

/* GJK: 1 with p[0..3] a tetrahedron enclosing the origin (possibly on its boundary, see
   gjk_complete), 0 if apart or touching */
static int gjk_enclose(const mpair* P, msup* p) {
  double c1[3], c2[3], x[3];
  geom_center(P->om, P->d, P->g1, c1);
  geom_center(P->om, P->d, P->g2, c2);
  sub3(x, c1, c2);
  if (dot3(x, x) == 0) x[0] = 1e-9;
  int n = 0;
  double xx_prev = 1e300;
  for (int it = 0; it < CCD_ITER; it++) {
    double dir[3] = {-x[0], -x[1], -x[2]};
    msup s;
    msupport(P, dir, &s);
    if (dot3(x, s.v) > 0) return 0; /* the plane x.p = x.s separates the origin: apart */
    /* no progress toward the origin: it lies (within tolerance) on the boundary */
    double xx = dot3(x, x);
    if (xx - dot3(x, s.v) <= CCD_TOL * CCD_TOL) return 0;
    p[n++] = s;
    if (n == 4) {
      msup q[4] = {p[0], p[1], p[2], p[3]};
      int r = tet_contains(p, x, &n);
      if (r == 1) return 1;
      if (r < 0) { /* flat: the previous triangle p[0..2], completed if it carries the origin */
        n = gjk_reduce(p, 3, x);
        if (!(dot3(x, x) < 1e-12 * dot3(s.v, s.v))) return 0;
      } else if (!(dot3(x, x) < xx_prev)) {
        /* no progress (the support along x returns a vertex already held): the origin is within
           rounding of this tetrahedron, EPA from it decides (the kernel's fp32 GJK stalls so on
           the table box's large flat Minkowski difference) */
        memcpy(p, q, sizeof(q));
        return 1;
      }
    } else {
      n = gjk_reduce(p, n, x);
    }
    xx_prev = dot3(x, x);
    /* the origin on the simplex up to rounding (|x| < 1e-6 of the support point's scale) */
    if (dot3(x, x) < 1e-12 * dot3(s.v, s.v)) return n >= 2 && gjk_complete(P, p, n);
  }
  return 0;
}

static void epa_face_set(epa_face* f, const msup* V, int a, int b, int c) {
  double ab[3], ac[3];
  sub3(ab, V[b].v, V[a].v);
  sub3(ac, V[c].v, V[a].v);
  cross3(f->n, ab, ac);
  normalize3(f->n);
  f->a = a, f->b = b, f->c = c, f->live = 1;
  f->d = dot3(f->n, V[a].v);
}

/* EPA from the enclosing tetrahedron V[0..3]: 1 with depth, normal, pos */
static int epa(const mpair* P, msup* V, double* depth, double dir[3], double pos[3]) {
  epa_face F[EPA_MAXF];
  int nv = 4, nf = 0;
  static const int T[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};
  for (int k = 0; k < 4; k++) {
    epa_face_set(&F[nf], V, T[k][0], T[k][1], T[k][2]);
    double ak[3];
    sub3(ak, V[k].v, V[T[k][0]].v);
    if (dot3(F[nf].n, ak) > 0) epa_face_set(&F[nf], V, T[k][0], T[k][2], T[k][1]); /* outward */
    nf++;
  }
  int best = -1;
  double upper = 1e300;
  for (int it = 0; it < CCD_ITER; it++) {
    best = -1;
    for (int i = 0; i < nf; i++)
      if (F[i].live && (best < 0 || F[i].d < F[best].d)) best = i;
    if (best < 0) return 0;
    msup w;
    msupport(P, F[best].n, &w);
    double dw = dot3(F[best].n, w.v);
    if (dw < upper) upper = dw;
    if (upper - F[best].d < CCD_TOL || nv == EPA_MAXV) break;
    /* faces seen from w go; their boundary (edges not shared by two of them) is the horizon.
       The polytope is untouched until the expansion is known to fit. */
    int E[3 * EPA_MAXF][2], ne = 0, nvis = 0;
    unsigned char vis[EPA_MAXF];
    for (int i = 0; i < nf; i++) {
      vis[i] = 0;
      if (!F[i].live) continue;
      double aw[3];
      sub3(aw, w.v, V[F[i].a].v);
      if (dot3(F[i].n, aw) <= 0.5 * CCD_TOL) continue; /* (on its plane: not seen, as the kernel) */
      vis[i] = 1;
      nvis++;
      const int ed[3][2] = {{F[i].a, F[i].b}, {F[i].b, F[i].c}, {F[i].c, F[i].a}};
      for (int q = 0; q < 3; q++) {
        int dup = -1;
        for (int r = 0; r < ne; r++)
          if (E[r][0] == ed[q][1] && E[r][1] == ed[q][0]) dup = r;
        if (dup >= 0) {
          E[dup][0] = E[ne - 1][0], E[dup][1] = E[ne - 1][1];
          ne--;
        } else {
          E[ne][0] = ed[q][0], E[ne][1] = ed[q][1];
          ne++;
        }
      }
    }
    if (ne == 0 || nf - nvis + ne > EPA_MAXF) break; /* (budget: keep the best face so far) */
    int m = 0;
    for (int i = 0; i < nf; i++)
      if (F[i].live && !vis[i]) F[m++] = F[i];
    nf = m;
    V[nv] = w;
    for (int r = 0; r < ne; r++) epa_face_set(&F[nf++], V, E[r][0], E[r][1], nv);
    nv++;
    best = -1;
  }
  if (best < 0) {
    best = 0;
    for (int i = 1; i < nf; i++)
      if (F[i].d < F[best].d) best = i;
  }
  /* witness points of the closest face */
  const epa_face* f = &F[best];
  double pr[3] = {f->d * f->n[0], f->d * f->n[1], f->d * f->n[2]};
  const double *a = V[f->a].v, *b = V[f->b].v, *c = V[f->c].v;
  double v0[3], v1[3], v2[3];
  sub3(v0, b, a);
  sub3(v1, c, a);
  sub3(v2, pr, a);
  double d00 = dot3(v0, v0), d01 = dot3(v0, v1), d11 = dot3(v1, v1), d20 = dot3(v2, v0), d21 = dot3(v2, v1);
  double den = d00 * d11 - d01 * d01;
  if (den <= 0) return 0;
  double lb = (d11 * d20 - d01 * d21) / den, lc = (d00 * d21 - d01 * d20) / den, la = 1 - lb - lc;
  for (int k = 0; k < 3; k++) {
    double x1 = la * V[f->a].v1[k] + lb * V[f->b].v1[k] + lc * V[f->c].v1[k];
    double x2 = la * V[f->a].v2[k] + lb * V[f->b].v2[k] + lc * V[f->c].v2[k];
    pos[k] = 0.5 * (x1 + x2);
    dir[k] = f->n[k];
  }
  *depth = f->d;
  g_cflops += 0; /* (counted by msupport) */
  return f->d > 0;
}

static int ccd_penetration(const mpair* P, double* depth, double dir[3], double pos[3]) {
  msup V[EPA_MAXV];
  if (!gjk_enclose(P, V)) return 0;
  return epa(P, V, depth, dir, pos);
}

/* ----------------------------------------------------------- primitives */
static void make_frame(double f[9]) {
  normalize3(f);
  double y[3];
  if (fabs(f[1]) < 0.5) {
    y[0] = 0;
    y[1] = 1;
    y[2] = 0;
  } else {
    y[0] = 0;
    y[1] = 0;
    y[2] = 1;
  }
  double dd = dot3(f, y);
  for (int k = 0; k < 3; k++) y[k] -= dd * f[k];
  normalize3(y);
  memcpy(f + 3, y, sizeof(y));
  cross3(f + 6, f, f + 3);
}

static int plane_box(const orc_model* om, const orc_data* d, int gp, int gb, orc_contact* out,
                     int maxout) {
  const double* Rp = d->geom_xmat[gp];
  double n[3];
  col(n, Rp, 2);
  const double* R = d->geom_xmat[gb];
  const double* h = om->m->geom_size[gb];
  int cnt = 0;
  for (int i = 0; i < 8 && cnt < maxout && cnt < 4; i++) {
    double l[3] = {(i & 1 ? 1 : -1) * h[0], (i & 2 ? 1 : -1) * h[1], (i & 4 ? 1 : -1) * h[2]};
    double p[3], rel[3];
    for (int k = 0; k < 3; k++)
      p[k] = d->geom_xpos[gb][k] + R[3 * k] * l[0] + R[3 * k + 1] * l[1] + R[3 * k + 2] * l[2];
    sub3(rel, p, d->geom_xpos[gp]);
    double dist = dot3(rel, n);
    if (dist < 0) {
      orc_contact* c = &out[cnt++];
      c->dist = dist;
      for (int k = 0; k < 3; k++) c->pos[k] = p[k] - 0.5 * dist * n[k];
      memcpy(c->frame, n, sizeof(n));
    }
  }
  return cnt;
}

static int plane_convex(const orc_model* om, const orc_data* d, int gp, int g, orc_contact* out) {
  double n[3], nn[3], p[3], rel[3];
  col(n, d->geom_xmat[gp], 2);
  for (int k = 0; k < 3; k++) nn[k] = -n[k];
  support(om, d, g, nn, p);
  sub3(rel, p, d->geom_xpos[gp]);
  double dist = dot3(rel, n);
  if (dist >= 0) return 0;
  out->dist = dist;
  for (int k = 0; k < 3; k++) out->pos[k] = p[k] - 0.5 * dist * n[k];
  memcpy(out->frame, n, sizeof(n));
  return 1;
}

/* Sutherland-Hodgman clip of a polygon against  (p - o).a <= lim */
static int clip_poly(double in[][3], int n, double out[][3], const double o[3], const double a[3],
                     double lim) {
  int m = 0;
  for (int i = 0; i < n; i++) {
    const double* P = in[i];
    const double* Q = in[(i + 1) % n];
    double rp[3], rq[3];
    sub3(rp, P, o);
    sub3(rq, Q, o);
    double sp = dot3(rp, a) - lim, sq = dot3(rq, a) - lim;
    if (sp <= 0) memcpy(out[m++], P, 3 * sizeof(double));
    if ((sp < 0 && sq > 0) || (sp > 0 && sq < 0)) {
      double t = sp / (sp - sq);
      for (int k = 0; k < 3; k++) out[m][k] = P[k] + t * (Q[k] - P[k]);
      m++;
    }
  }
  return m;
}

static int box_box(const orc_model* om, const orc_data* d, int g1, int g2, orc_contact* out,
                   int maxout) {
  const double *c1 = d->geom_xpos[g1], *c2 = d->geom_xpos[g2];
  const double *R1 = d->geom_xmat[g1], *R2 = d->geom_xmat[g2];
  const double *h1 = om->m->geom_size[g1], *h2 = om->m->geom_size[g2];
  double A[3][3], B[3][3], t[3];
  for (int k = 0; k < 3; k++) {
    col(A[k], R1, k);
    col(B[k], R2, k);
  }
  sub3(t, c2, c1);
  double best = 1e300, bn[3] = {0, 0, 0};
  int bcode = -1;
  for (int code = 0; code < 15; code++) {
    double L[3];
    if (code < 3)
      memcpy(L, A[code], sizeof(L));
    else if (code < 6)
      memcpy(L, B[code - 3], sizeof(L));
    else
      cross3(L, A[(code - 6) / 3], B[(code - 6) % 3]);
    double ln = norm3(L);
    if (ln < 1e-6) continue;
    for (int k = 0; k < 3; k++) L[k] /= ln;
    double r1 = 0, r2 = 0;
    for (int k = 0; k < 3; k++) {
      r1 += h1[k] * fabs(dot3(A[k], L));
      r2 += h2[k] * fabs(dot3(B[k], L));
    }
    double tl = dot3(t, L);
    double ov = r1 + r2 - fabs(tl);
    if (ov < 0) return 0;
    double score = code < 6 ? ov : ov * 1.05 + 1e-9;
    if (score < best) {
      best = score;
      bcode = code;
      for (int k = 0; k < 3; k++) bn[k] = tl < 0 ? -L[k] : L[k];
    }
  }
  if (bcode < 0) return 0;
  if (bcode < 6) {
    /* face contact: reference box r, incident box i; nr = outward ref normal towards i */
    int ref1 = bcode < 3;
    int fa = ref1 ? bcode : bcode - 3;
    const double* cr = ref1 ? c1 : c2;
    const double* ci = ref1 ? c2 : c1;
    double(*Ar)[3] = ref1 ? A : B;
    double(*Ai)[3] = ref1 ? B : A;
    const double* hr = ref1 ? h1 : h2;
    const double* hi = ref1 ? h2 : h1;
    double nr[3];
    for (int k = 0; k < 3; k++) nr[k] = ref1 ? bn[k] : -bn[k];
    double fc[3];
    for (int k = 0; k < 3; k++) fc[k] = cr[k] + nr[k] * hr[fa];
    /* incident face: most anti-parallel to nr */
    int ia = 0;
    double bd = 0;
    for (int k = 0; k < 3; k++) {
      double dd = fabs(dot3(Ai[k], nr));
      if (dd > bd) {
        bd = dd;
        ia = k;
      }
    }
    double s = dot3(Ai[ia], nr) > 0 ? -1.0 : 1.0;
    int u = (ia + 1) % 3, v = (ia + 2) % 3;
    double poly[16][3], tmp[16][3];
    static const double su[4] = {1, -1, -1, 1}, sv[4] = {1, 1, -1, -1};
    for (int q = 0; q < 4; q++)
      for (int k = 0; k < 3; k++)
        poly[q][k] = ci[k] + s * hi[ia] * Ai[ia][k] + su[q] * hi[u] * Ai[u][k] +
                     sv[q] * hi[v] * Ai[v][k];
    int n = 4;
    int ra = (fa + 1) % 3, rb = (fa + 2) % 3;
    double na[3];
    n = clip_poly(poly, n, tmp, fc, Ar[ra], hr[ra]);
    for (int k = 0; k < 3; k++) na[k] = -Ar[ra][k];
    n = clip_poly(tmp, n, poly, fc, na, hr[ra]);
    n = clip_poly(poly, n, tmp, fc, Ar[rb], hr[rb]);
    for (int k = 0; k < 3; k++) na[k] = -Ar[rb][k];
    n = clip_poly(tmp, n, poly, fc, na, hr[rb]);
    /* penetrating points, deepest first (stable) */
    double dep[16];
    int idx[16], m = 0;
    for (int q = 0; q < n; q++) {
      double rel[3];
      sub3(rel, poly[q], fc);
      double sd = dot3(rel, nr);
      if (sd < 0) {
        dep[m] = sd;
        idx[m++] = q;
      }
    }
    for (int a = 1; a < m; a++)
      for (int b = a; b > 0 && dep[b] < dep[b - 1]; b--) {
        double td = dep[b];
        dep[b] = dep[b - 1];
        dep[b - 1] = td;
        int ti = idx[b];
        idx[b] = idx[b - 1];
        idx[b - 1] = ti;
      }
    int cnt = 0;
    for (int q = 0; q < m && cnt < 4 && cnt < maxout; q++) {
      orc_contact* c = &out[cnt++];
      c->dist = dep[q];
      for (int k = 0; k < 3; k++) c->pos[k] = poly[idx[q]][k] - 0.5 * dep[q] * nr[k];
      memcpy(c->frame, bn, sizeof(bn));
    }
    return cnt;
  }
  /* edge-edge */
  int ea = (bcode - 6) / 3, eb = (bcode - 6) % 3;
  double p1[3], p2[3];
  memcpy(p1, c1, sizeof(p1));
  memcpy(p2, c2, sizeof(p2));
  for (int k = 0; k < 3; k++) {
    if (k != ea) {
      double sg = dot3(A[k], bn) > 0 ? 1.0 : -1.0;
      for (int e = 0; e < 3; e++) p1[e] += sg * h1[k] * A[k][e];
    }
    if (k != eb) {
      double sg = dot3(B[k], bn) > 0 ? -1.0 : 1.0;
      for (int e = 0; e < 3; e++) p2[e] += sg * h2[k] * B[k][e];
    }
  }
  /* closest points of lines p1 + s A[ea], p2 + t B[eb] */
  double r[3];
  sub3(r, p1, p2);
  double a = 1, e = 1, b = dot3(A[ea], B[eb]), c = dot3(A[ea], r), f = dot3(B[eb], r);
  double den = a * e - b * b;
  double sp = den > 1e-12 ? (b * f - c * e) / den : 0;
  double tp = (b * sp + f) / e;
  if (sp > h1[ea]) sp = h1[ea];
  if (sp < -h1[ea]) sp = -h1[ea];
  if (tp > h2[eb]) tp = h2[eb];
  if (tp < -h2[eb]) tp = -h2[eb];
  orc_contact* cc = &out[0];
  cc->dist = -best / 1.05;
  for (int k = 0; k < 3; k++) cc->pos[k] = 0.5 * (p1[k] + sp * A[ea][k] + p2[k] + tp * B[eb][k]);
  memcpy(cc->frame, bn, sizeof(bn));
  return maxout > 0;
}

/* narrowphase dispatch for one candidate pair; fills pos/dist/normal */
int orc_collide_pair(const orc_model* om, const orc_data* d, int g1, int g2, orc_contact* out,
                     int maxout) {
  const sim_model_desc* m = om->m;
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  if (maxout <= 0) return 0;
  g_cstat[0] += 1;
  /* bounding-sphere midphase (planes have rbound 0 and skip it) */
  if (m->geom_rbound[g1] > 0 && m->geom_rbound[g2] > 0) {
    double a[3], b[3], r[3];
    geom_center(om, d, g1, a);
    geom_center(om, d, g2, b);
    sub3(r, a, b);
    double mg = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
    if (norm3(r) > m->geom_rbound[g1] + m->geom_rbound[g2] + mg) return 0;
    /* world-axis-aligned boxes around the local boxes (MuJoCo's broadphase AABBs) */
    const double *R1 = d->geom_xmat[g1], *R2 = d->geom_xmat[g2];
    const double *h1 = m->geom_aabb[g1] + 3, *h2 = m->geom_aabb[g2] + 3;
    for (int k = 0; k < 3; k++) {
      double e1 = fabs(R1[3 * k]) * h1[0] + fabs(R1[3 * k + 1]) * h1[1] + fabs(R1[3 * k + 2]) * h1[2];
      double e2 = fabs(R2[3 * k]) * h2[0] + fabs(R2[3 * k + 1]) * h2[1] + fabs(R2[3 * k + 2]) * h2[2];
      if (fabs(r[k]) > e1 + e2 + mg) return 0;
    }
  }
  g_cflops += 60; /* midphase sphere + AABB */
  g_cstat[1] += 1;
  if (g_curpair >= 0) g_pstat[g_curpair][0] += 1;
  if (t1 == SIM_GEOM_PLANE) {
    /* bounding sphere of geom2 entirely above the plane (beyond the margin): no contact */
    if (m->geom_rbound[g2] > 0) {
      double c[3], h = 0;
      const double* R = d->geom_xmat[g1];
      geom_center(om, d, g2, c);
      for (int k = 0; k < 3; k++) h += (c[k] - d->geom_xpos[g1][k]) * R[3 * k + 2];
      double mg = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
      if (h > m->geom_rbound[g2] + mg) return 0;
    }
    g_cstat[7] += 1;
    g_cflops += 150;
    if (t2 == SIM_GEOM_BOX) return plane_box(om, d, g1, g2, out, maxout);
    if (t2 == SIM_GEOM_MESH) return plane_convex(om, d, g1, g2, out);
    return 0;
  }
  if (t1 == SIM_GEOM_BOX && t2 == SIM_GEOM_BOX) {
    g_cstat[6] += 1;
    g_cflops += 700; /* 15-axis SAT + face clipping */
    return box_box(om, d, g1, g2, out, maxout);
  }
  if (t1 == SIM_GEOM_BOX && t2 == SIM_GEOM_MESH) {
    /* separating-axis pre-test on the box face that faces the hull's centre most:
       the hull's extreme point toward the box beyond that face -> apart (exact) */
    double c[3], r[3], best = -1e300, ax[3] = {0, 0, 1}, h = 0;
    const double* R = d->geom_xmat[g1];
    geom_center(om, d, g2, c);
    sub3(r, c, d->geom_xpos[g1]);
    for (int k = 0; k < 3; k++) {
      double a[3] = {R[k], R[3 + k], R[6 + k]};
      double dk = dot3(r, a), gap = fabs(dk) - m->geom_size[g1][k];
      if (gap > best) {
        double sg = dk >= 0 ? 1 : -1;
        best = gap, h = m->geom_size[g1][k];
        for (int q = 0; q < 3; q++) ax[q] = sg * a[q];
      }
    }
    double nd[3] = {-ax[0], -ax[1], -ax[2]}, sp[3], dist = -h;
    support(om, d, g2, nd, sp);
    for (int q = 0; q < 3; q++) dist += (sp[q] - d->geom_xpos[g1][q]) * ax[q];
    g_cflops += 60 + 36 + 10;
    double mg = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
    if (dist > mg) return 0;
  }
  mpair P = {om, d, g1, g2};
  double depth, dir[3], pos[3];
  g_cstat[2] += 1;
  if (m->ccd == SIM_CCD_NATIVE ? !ccd_penetration(&P, &depth, dir, pos) : !mpr_penetration(&P, &depth, dir, pos))
    return 0;
  g_cstat[3] += 1;
  out->dist = -depth;
  memcpy(out->pos, pos, sizeof(pos));
  memcpy(out->frame, dir, sizeof(dir));
  return 1;
}

/* mj_collision: all candidate pairs in order, contacts appended in pair order */
void orc_collision(const orc_model* om, orc_data* d) {
  const sim_model_desc* m = om->m;
  d->ncon = 0;
  g_cflops = 0;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    orc_contact tmp[8];
    g_curpair = p;
    int n = orc_collide_pair(om, d, g1, g2, tmp, 8);
    g_curpair = -1;
    for (int i = 0; i < n; i++) {
      if (d->ncon >= SIM_MAXCON) {
        d->status |= SIM_ST_CONOVERFLOW;
        break;
      }
      orc_contact* c = &d->contact[d->ncon++];
      *c = tmp[i];
      c->geom1 = g1;
      c->geom2 = g2;
      c->pair = p;
      make_frame(c->frame);
      for (int k = 0; k < 3; k++) {
        double f1 = m->geom_friction[g1][k], f2 = m->geom_friction[g2][k];
        double f = f1 > f2 ? f1 : f2;
        if (k == 0 && om->friction >= 0) f = om->friction;
        if (k == 0) c->friction[0] = c->friction[1] = f;
        if (k == 1) c->friction[2] = f;
        if (k == 2) c->friction[3] = c->friction[4] = f;
      }
      c->mu = c->friction[0];
    }
  }
  d->flops += g_cflops;
  d->cflops += g_cflops;
}

int orc_collide_geoms(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                      const int32_t* hadj, const double* qpos, int g1, int g2, double* out,
                      int maxout) {
  int32_t seeds[SIM_MAXGEOM * ORC_NSEED];
  if (hv) orc_hull_seeds(m, hv, seeds);
  orc_model om = {m, hv, hadr, hadj, hv ? seeds : NULL, 1.0, -1.0, 1.0};
  static __thread orc_data d;
  orc_reset_data(&om, &d);
  for (int i = 0; i < m->nq; i++) d.qpos[i] = qpos[i];
  orc_kinematics(&om, &d);
  orc_contact c[8];
  int n = orc_collide_pair(&om, &d, g1, g2, c, maxout < 8 ? maxout : 8);
  for (int i = 0; i < n; i++) {
    out[7 * i] = c[i].dist;
    for (int k = 0; k < 3; k++) out[7 * i + 1 + k] = c[i].pos[k];
    for (int k = 0; k < 3; k++) out[7 * i + 4 + k] = c[i].frame[k];
  }
  return n;
}

/* world frames of every geom at qpos (kinematics only): xpos [ngeom][3], xmat [ngeom][9] */
void orc_geom_frames(const sim_model_desc* m, const double* qpos, double* xpos, double* xmat) {
  orc_model om = {m, NULL, NULL, NULL, NULL, 1.0, -1.0, 1.0};
  static __thread orc_data d;
  orc_reset_data(&om, &d);
  for (int i = 0; i < m->nq; i++) d.qpos[i] = qpos[i];
  orc_kinematics(&om, &d);
  for (int g = 0; g < m->ngeom; g++) {
    for (int k = 0; k < 3; k++) xpos[3 * g + k] = d.geom_xpos[g][k];
    for (int k = 0; k < 9; k++) xmat[9 * g + k] = d.geom_xmat[g][k];
  }
}

int orc_hull_support_flat(const sim_model_desc* m, const float* hv, const int32_t* hadr,
                          const int32_t* hadj, int g, const double* dirs, int n, int use_graph,
                          int32_t* out) {
  int32_t seeds[SIM_MAXGEOM * ORC_NSEED];
  if (hv) orc_hull_seeds(m, hv, seeds);
  orc_model om = {m, hv, hadr, hadj, hv ? seeds : NULL, 1.0, -1.0, 1.0};
  for (int i = 0; i < n; i++) out[i] = orc_hull_support_ex(&om, g, dirs + 3 * i, use_graph);
  return 0;
}

/* diagnostic counters (single-threaded use) */
void orc_collision_stats(double* out, int reset) {
  for (int k = 0; k < 8; k++) {
    out[k] = g_cstat[k];
    if (reset) g_cstat[k] = 0;
  }
  for (int p = 0; p < SIM_MAXPAIR; p++)
    for (int k = 0; k < 2; k++) {
      out[8 + 2 * p + k] = g_pstat[p][k];
      if (reset) g_pstat[p][k] = 0;
    }
}
