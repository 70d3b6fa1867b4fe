/*
 * selftest.c — drives the float64 oracle end to end from a compiled model file, for the
 * AddressSanitizer / UndefinedBehaviorSanitizer build (make -C oracle selftest_asan;
 * tests/test_oracle_sanitize.py).  TEST INFRASTRUCTURE ONLY.
 *
 * Model file (written by tests/test_oracle_sanitize.py from mjcf.compile_mjcf):
 *   sim_model_desc (raw bytes) | int32 nhv | float hv[3 nhv] | int32 hadr[nhv + 1] |
 *   int32 nadj | int32 hadj[nadj]
 * Runs: reset, 20 env-steps of random actions with PGS, the same with Newton (MuJoCo's
 * tolerance and exact), qfrc_bias, a diagnostic forward, pose and position IK; every state
 * must stay finite.  Exit status 0 on success.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static void* rd(FILE* f, size_t n) {
  void* p = malloc(n ? n : 1);
  if (n && fread(p, 1, n, f) != n) {
    fprintf(stderr, "short model file\n");
    exit(2);
  }
  return p;
}

static double urand(unsigned* s) {
  *s = *s * 1664525u + 1013904223u;
  return (*s >> 8) * (1.0 / 16777216.0);
}

static int finite_all(const double* x, int n) {
  for (int i = 0; i < n; i++)
    if (!isfinite(x[i])) return 0;
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s model.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  sim_model_desc* m = (sim_model_desc*)rd(f, sizeof(sim_model_desc));
  int32_t nhv, nadj;
  if (fread(&nhv, 4, 1, f) != 1) return 2;
  float* hv = (float*)rd(f, sizeof(float) * 3 * (size_t)nhv);
  int32_t* hadr = (int32_t*)rd(f, sizeof(int32_t) * ((size_t)nhv + 1));
  if (fread(&nadj, 4, 1, f) != 1) return 2;
  int32_t* hadj = (int32_t*)rd(f, sizeof(int32_t) * (size_t)nadj);
  fclose(f);

  const int n = 16, T = 20;
  unsigned seed = 12345u;
  int bad = 0;
  for (int solver = 0; solver < 3; solver++) {
    sim_model_desc mm = *m;
    mm.solver = solver == 0 ? SIM_SOL_PGS : SIM_SOL_NEWTON;
    if (solver == 2) mm.tolerance = 0.0;
    double *qpos = calloc((size_t)n * mm.nq, 8), *qvel = calloc((size_t)n * mm.nv, 8),
           *warm = calloc((size_t)n * mm.nv, 8), *ctrl = calloc((size_t)n * mm.nu, 8),
           *iq = calloc((size_t)n * mm.obs_nq, 8), *ex = calloc((size_t)n * mm.nq, 8),
           *obs = calloc((size_t)n * (3 + mm.obs_nq), 8), *act = calloc((size_t)n * mm.nact, 8),
           *ncon = calloc(n, 8), *bias = calloc((size_t)n * mm.nv, 8);
    int32_t* status = calloc(n, 4);
    for (int e = 0; e < n; e++) {
      for (int i = 0; i < mm.nq; i++) ex[e * mm.nq + i] = mm.qpos0[i];
      if (mm.nq > 6) ex[e * mm.nq + 8] = -0.0009 + 0.015, ex[e * mm.nq + 6] = 0.25;
      for (int k = 0; k < mm.obs_nq; k++) iq[e * mm.obs_nq + k] = -1.0 + 2.0 * urand(&seed);
    }
    orc_batch_reset(&mm, n, qpos, qvel, warm, ctrl, iq, NULL, ex, obs);
    double fl[2];
    for (int t = 0; t < T; t++) {
      for (int i = 0; i < n * mm.nact; i++) act[i] = urand(&seed) - 0.5;
      orc_batch_step(&mm, hv, hadr, hadj, n, qpos, qvel, warm, ctrl, act, 10, obs, status, ncon, NULL, 2, fl,
                     NULL);
    }
    orc_batch_bias(&mm, n, qpos, qvel, NULL, bias);
    bad |= !finite_all(qpos, n * mm.nq) || !finite_all(qvel, n * mm.nv) || !finite_all(bias, n * mm.nv);
    double M[SIM_MAXDOF * SIM_MAXDOF], b[SIM_MAXDOF], qa[SIM_MAXDOF], con[9 * SIM_MAXCON], site[3 * SIM_MAXSITE],
        gx[3 * SIM_MAXGEOM], efc[ORC_MAXEFC];
    int nefc = 0;
    orc_debug_forward(&mm, hv, hadr, hadj, qpos, qvel, ctrl, warm, M, b, qa, con, site, gx, efc, &nefc);
    bad |= !finite_all(qa, mm.nv);
    printf("solver %d: ncon/env/substep %.3f, finite %d\n", solver, 0.0, !bad);
    free(qpos), free(qvel), free(warm), free(ctrl), free(iq), free(ex), free(obs), free(act), free(ncon);
    free(bias), free(status);
  }
  /* IK: position only and pose toward the reachable pose of a known configuration */
  {
    double tgt[3 * 8], tq[4 * 8], q[SIM_MAXQ * 8];
    int32_t ok[8], it[8];
    for (int e = 0; e < 8; e++) {
      tgt[3 * e] = 0.3, tgt[3 * e + 1] = 0.05 * (e - 4), tgt[3 * e + 2] = 0.2;
      tq[4 * e] = 1, tq[4 * e + 1] = tq[4 * e + 2] = tq[4 * e + 3] = 0;
      for (int i = 0; i < m->nq; i++) q[e * m->nq + i] = m->qpos0[i];
    }
    orc_ik_dls(m, 8, tgt, NULL, q, ok, it, 1e-6, 0.5, 0.1, 1e-2, 2.0, 20.0, 100, m->obs_site, 5);
    bad |= !finite_all(q, 8 * m->nq);
    orc_ik_dls(m, 8, tgt, tq, q, ok, it, 1e-6, 0.5, 0.1, 1e-2, 2.0, 20.0, 100, m->obs_site, 5);
    bad |= !finite_all(q, 8 * m->nq);
  }
  free(m), free(hv), free(hadr), free(hadj);
  printf("selftest %s\n", bad ? "FAILED" : "ok");
  return bad ? 1 : 0;
}
