// soarm_substep.h — the env-step kernels of the contact-free and the contact scenes (k_step,
// k_geom, k_substep) and the per-env forward they share; included by soarm_sim.hip (the launch
// code and the C ABI) and by diagnostic translation units that instantiate one kernel alone.
#pragma once
#include "soarm_collide.h"
#include "soarm_env.h"
#include "soarm_pgs.h"

namespace soarm {

#ifdef SOARM_PHASE_PROF
// diagnostic build: summed wave cycles per k_substep phase
//   [0] state load + checks, [1] kinematics..smooth forces, [2] constraint rows,
//   [3] PGS sweeps, [4] qacc/fcon + Euler + obs + geom poses, [5] waves,
//   [6] sum over envs of PGS sweeps, [7] env count, [8] max wave cycles,
//   [9] waves on the register fast path, [10] max wave PGS cycles,
//   [11] sum over waves of the wave's max sweep count, [12] waves with an active
//   joint limit, [13] waves with a contact outside the register block, [14] waves
//   with more than LDS_CON contacts, [15] max contacts of an env, [16] rows: up to
//   the built contact rows, [17] rows: warm start + cost, [18] rows: block setup
//   [19..22] waves per sweep variant (y-pure, y+arm slot, block-first general, other),
//   [23..26] max wave cycles per variant, [27] waves with a non-block contact on the free body
//   [28..42] wave cycles between consecutive fine stamps (g_stamp, see PSTAMP sites)
// (accumulated per wave in g_wphase, soarm_pgs.h; this is the layout)
//                                          [53..56] contact-row build split (g_rowprof),
                                            // [57] waves that retired the arm rows, [58] sum of their retire sweeps,
                                            // [59] / [60] max wave cycles of the waves that did not / did retire
                                            // y+arm slot waves by (F slot, E coupled to the cube) = 2 F + coupled:
                                            // [61..64] waves, [65..68] max wave cycles, [69..72] sum of PGS
                                            // cycles, [73..76] sum of the arm-retire sweep (0: not retired)
#define PHASE_T(v) const long long v = clock64()
#else
#define PHASE_T(v)
#endif

// one mj_forward (position + velocity + acceleration stages); the contacts
// (cbuf/ccount, may be null) were produced by k_collide from this substep's positions
template <int NA, int NF, bool CON, int SOL, bool RS = false>
DEVI int forward(Sim<NA, NF>& S, const float* cbuf, const int* ccount, const uint32_t* pmask, int n, int e,
                 const RowLds& L, const ContactRows<NA, NF>& cr, const float* applied = nullptr,
                 PairMask pm = PairMask{}) {
  S.kinematics();
  S.com_crb();
  S.factor();
  S.smooth_forces();
  pm.hold();
  if (applied) S.add_applied(applied, n, e);
  return solve_constraints<NA, NF, CON, SOL, RS>(S, cbuf, ccount, pmask, n, e, L, cr, pm);
}

// contact-free scenes (mjDSBL_CONTACT): all frame_skip substeps fused in one launch.
// AP: st.qfrc_applied is set (a separate instantiation keeps the common case's code as is)
template <int NA, int NF, bool AP, int SOL>
__global__ __launch_bounds__(64) void k_step(const DModel* __restrict__ dm, int n, int nsub,
                                             sim_state st, const float* __restrict__ action,
                                             float* __restrict__ obs, sim_params pp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const DModel& m = *dm;
  Sim<NA, NF> S(dm, pp.mass_scale ? pp.mass_scale[e] : 1.f, pp.friction ? pp.friction[e] : -1.f,
                pp.damping_scale ? pp.damping_scale[e] : 1.f);
  load_state(S, st, n, e);
  if (action) {
#pragma unroll
    for (int k = 0; k < NA; k++)
      if (k < m.nact) S.ctrl[k] = action[(size_t)e * m.nact + k];
  }
  __shared__ float s_lim[NA * LF][64];
  const RowLds L{nullptr, &s_lim[0][0], nullptr, nullptr, (int)threadIdx.x, (int)threadIdx.x, 64};
  const ContactRows<NA, NF> cr{nullptr, n};
  float* const applied = AP ? st.qfrc_applied : nullptr;
  for (int s = 0; s < nsub; s++) {
    S.relaunder();
    if (S.check_state() && AP) zero_applied(applied, Sim<NA, NF>::NV, n, e);
    forward<NA, NF, false, SOL>(S, nullptr, nullptr, nullptr, n, e, L, cr, applied);
    if (S.acc_bad()) {
      S.soft_reset(SIM_ST_BADQACC);
      if (AP) zero_applied(applied, Sim<NA, NF>::NV, n, e);
      forward<NA, NF, false, SOL>(S, nullptr, nullptr, nullptr, n, e, L, cr);
    }
    S.integrate();
  }
  store_state(S, st, n, e);
  if (obs) write_obs(S, obs, e);
}

// body world frames from the current qpos (collision input); GEOM_LPE lanes per env split the
// stores (the FK chain runs on each of them)
constexpr int GEOM_LPE = 4;
// XCD-aware block index: workgroups are dealt round-robin over the 8 XCDs, so renumber them to give
// each XCD a contiguous range of envs.  A 16-env workgroup touches half of each 128-B line of the
// [row][env] state; its neighbour, which reads the other half, is then in the same L2.
__device__ __forceinline__ int xcd_block() {
  const int g = (int)gridDim.x, b = (int)blockIdx.x;
  return (g & 7) ? b : (b & 7) * (g >> 3) + (b >> 3);
}

template <int NA, int NF>
__global__ __launch_bounds__(64) void k_geom(const DModel* __restrict__ dm, int n, sim_state st,
                                             float* __restrict__ gpose) {
  const int e = xcd_block() * (64 / GEOM_LPE) + (int)threadIdx.x / GEOM_LPE;
  if (e >= n) return;
  Sim<NA, NF> S(dm, 1.f, -1.f, 1.f);
  load_state(S, st, n, e);
  S.kinematics();
  write_body_frames(S, gpose, n, e, (int)threadIdx.x % GEOM_LPE, GEOM_LPE);
}
inline dim3 geom_grid(int n) { return dim3((n + 64 / GEOM_LPE - 1) / (64 / GEOM_LPE)); }

// a soft-reset env's contact input: the model's contacts at qpos0 (DModel c0_*) into its own slots of
// the collide output and its pair mask.  Every lane of the env writes the same records, so each lane
// reads back its own stores in the build that follows.  Cold: taken only by envs that soft-reset.
DEVI void qpos0_contacts(const DModel& m, float* cbuf, int n, int e, PairMask& pm) {
  const int nw = (m.npair + 31) >> 5;
#pragma unroll
  for (int k = 0; k < PairMask::MAXW; k++) pm.w[k] = k < nw ? m.c0_w[k] : 0u;
  pm.cw = m.c0_w[nw];
  for (int c = 0; c < m.c0_n; c++)
#pragma unroll
    for (int f = 0; f < 7; f++) soa(cbuf, m.c0_slot[c] * 7 + f, n, e) = m.c0_rec[c][f];
}

// one substep with contacts: gather -> forward -> Euler -> next substep's geom poses
// (AP: st.qfrc_applied is set, as in k_step)
// RS (PGS, free-body scene): the row-space kernel -- 16 lanes per env, 4 envs per wave.  The
// per-env code runs on each of the env's 4 quads (identical values; the contact rows and the next
// geom poses are split over the 16 lanes) and the constraint solve holds one row per lane
// (soarm_pgs.h, RS_MAXROW): at 4096 envs 1024 waves, one per SIMD.
template <int NA, int NF, bool AP, int SOL, bool RS = false>
__global__ __launch_bounds__(64) void k_substep(const DModel* __restrict__ dm, int n, sim_state st,
                                                const float* __restrict__ action,
                                                float* __restrict__ obs, sim_params pp,
                                                float* __restrict__ scratch,
                                                const float* __restrict__ cbuf,
                                                const int* __restrict__ ccount,
                                                uint32_t* __restrict__ pmask,
                                                float* __restrict__ gpose, const float* gpose_in) {
  // envs per workgroup: lpe<NF>() lanes per env (soarm_pgs.h) run the same per-env code; the RS
  // kernel has 16 per env (4 quads)
  constexpr int COLS = RS ? RS_EPW : 64 / lpe<NF>();
  constexpr int LPE = 64 / COLS;
  const int e = xcd_block() * COLS + (int)threadIdx.x / LPE;
  static_assert(!RS || (NF == 1 && SOL == SIM_SOL_PGS), "RS kernel: PGS, scene with a free body");
  if (e >= n) return;
  PHASE_T(t0);
  const DModel& m = *dm;
  Sim<NA, NF> S(dm, pp.mass_scale ? pp.mass_scale[e] : 1.f, pp.friction ? pp.friction[e] : -1.f,
                pp.damping_scale ? pp.damping_scale[e] : 1.f);
  load_state(S, st, n, e);
  if (action) {
#pragma unroll
    for (int k = 0; k < NA; k++)
      if (k < m.nact) S.ctrl[k] = action[(size_t)e * m.nact + k];
  }
  __shared__ float s_rows[(LDS_CON + 1) * CF][COLS];  // + one all-zero record
  __shared__ float s_lim[NA * LF][COLS];
  __shared__ float s_keep[keep_floats<NA, NF>()][COLS];
  // contact list (quad), y-sweep slots; Newton: its line-search rows (8 per LDS contact)
  __shared__ float s_ext[NF == 1 ? XS_EXT : (lpe<NF>() == 4 ? XS_LIST + (SOL == SIM_SOL_NEWTON ? 12 * LDS_CON : 0) : 1)][COLS];
  RowLds L{&s_rows[0][0], &s_lim[0][0], NF == 1 ? &s_keep[0][0] : nullptr, &s_ext[0][0], (int)threadIdx.x,
           (int)threadIdx.x / LPE, COLS};
  __shared__ __attribute__((aligned(16))) float s_rsw[RS ? COLS * RS_WENV : 1];  // row-space W rows
  if constexpr (RS) L.rsw = s_rsw;
  const ContactRows<NA, NF> cr{scratch + e, n};
  const float ncon_prev = st.ncon ? st.ncon[e] : 0.f;  // issued early: consumed at the end
  // (the status bits are sticky: a reset is this substep's when check_state sets a cleared bit)
  const int st0 = S.status;
  S.status = st0 & ~(SIM_ST_BADQPOS | SIM_ST_BADQVEL);
  S.check_state();
  const bool reset = S.status != (st0 & ~(SIM_ST_BADQPOS | SIM_ST_BADQVEL));
  S.status |= st0;
  // positions / velocities are re-read from HBM after the solve instead of being held in
  // registers through it: a soft reset must reach HBM first
  if (reset) {
    store_state(S, st, n, e);
    if (AP) zero_applied(st.qfrc_applied, Sim<NA, NF>::NV, n, e);
  }
  // a soft reset moved the env to qpos0: the collide output no longer applies, the contacts at
  // qpos0 do (mj_resetData then mj_forward, collision included)
  const bool use = ccount != nullptr;
  // Newton's frictionloss-zone history (two substeps, past the contact rows of the scratch slab):
  // a period-2 pattern predicts this substep's zones (soarm_newton.h)
  uint32_t zh1 = 0u, zh2 = 0u;
  if constexpr (SOL == SIM_SOL_NEWTON) {
    const uint32_t* zh = (const uint32_t*)(scratch + e) + (size_t)zhist_row<NA, NF>() * n;
    zh1 = zh[0], zh2 = zh[n];
    if ((zh1 >> 31) && (zh2 >> 31) && zh1 != zh2) S.zpred = zh2;
  }
  PairMask pm;
  if (use) pm.load(pmask, m, n, e);  // (stays zero otherwise: no contact list)
  if (use && reset) qpos0_contacts(m, const_cast<float*>(cbuf), n, e, pm);
#ifdef SOARM_PHASE_PROF
  PHASE_T(t1);
  PSTAMP(0);
  S.kinematics();
  PSTAMP(1);
  S.com_crb();
  PSTAMP(2);
  S.factor();
  PSTAMP(3);
  S.smooth_forces();
  PSTAMP(4);
  PHASE_T(t2);
  PSTAMP(5);
  pm.hold();
  if (AP) S.add_applied(st.qfrc_applied, n, e);
  int ncon = solve_constraints<NA, NF, true, SOL, RS>(S, use ? cbuf : nullptr, use ? ccount : nullptr, pmask, n, e, L, cr, pm);
#else
  int ncon = forward<NA, NF, true, SOL, RS>(S, use ? cbuf : nullptr, use ? ccount : nullptr, pmask, n, e, L, cr,
                                        AP ? st.qfrc_applied : nullptr, pm);
#endif
  if (S.acc_bad()) {
    S.soft_reset(SIM_ST_BADQACC);
    store_state(S, st, n, e);
    if (AP) zero_applied(st.qfrc_applied, Sim<NA, NF>::NV, n, e);
    PairMask p0;
    if (use) qpos0_contacts(m, const_cast<float*>(cbuf), n, e, p0);
    ncon = forward<NA, NF, true, SOL, RS>(S, use ? cbuf : nullptr, use ? ccount : nullptr, pmask, n, e, L, cr,
                                          nullptr, p0);
  }
  PSTAMP(10);
  if constexpr (SOL == SIM_SOL_NEWTON) {
    if ((threadIdx.x & (lpe<NF>() - 1)) == 0) {
      uint32_t* zh = (uint32_t*)(scratch + e) + (size_t)zhist_row<NA, NF>() * n;
      zh[0] = S.zfin, zh[n] = zh1;
    }
  }
  if constexpr (NF == 1) {  // reload (laundered pointers: not CSE'd with the first load)
    const float* qp = launder(st.qpos);
    const float* qv = launder(st.qvel);
#pragma unroll
    for (int i = 0; i < Sim<NA, NF>::NQ; i++) S.qpos[i] = soa(qp, i, n, e);
#pragma unroll
    for (int i = 0; i < Sim<NA, NF>::NV; i++) S.qvel[i] = soa(qv, i, n, e);
  }
  if (pmask)  // consumed: clear for the next collide
    for (int w = 0; w < pmask_words(m); w++) soa(pmask, w, n, e) = 0u;
  const float ee[3] = {S.ee[0], S.ee[1], S.ee[2]};
  PSTAMP(11);
  if constexpr (RS)
    S.integrate_qacc();  // (the damped step's factor was made before the solve)
  else
    S.integrate();
  PSTAMP(12);
  store_state(S, st, n, e);
  if (st.ncon) st.ncon[e] = ncon_prev + (float)ncon;
  if (obs) {
    S.ee[0] = ee[0], S.ee[1] = ee[1], S.ee[2] = ee[2];
    write_obs(S, obs, e);
  }
  PSTAMP(13);
  if (gpose) {
    S.kinematics();
    PSTAMP(14);
    if constexpr (RS)  // (the W rows' LDS is free after the solve: the body frames are staged there)
      write_body_frames_lds(S, gpose, n, e, (int)threadIdx.x % LPE, LPE, s_rsw + L.col * RS_WENV);
    else
      write_body_frames(S, gpose, n, e, (int)threadIdx.x % LPE, LPE);
  } else {
    PSTAMP(14);  // (the last substep writes no poses: both phases empty)
  }
#ifdef SOARM_PHASE_PROF
  PHASE_T(t5);
  PSTAMP(15);
  const long long p0 = g_pgs_prof[8 * e], p1 = g_pgs_prof[8 * e + 1];
  const int nsw = (int)g_pgs_prof[8 * e + 2];
  const bool anylim = __any(g_pgs_prof[8 * e + 4] > 0), anyslow = __any(g_pgs_prof[8 * e + 3] == 0),
             anyovf = __any(g_pgs_prof[8 * e + 5] > LDS_CON), anyfree = __any(g_pgs_prof[8 * e + 3] & 16);
  // (wave reductions first: one row per wave in g_wphase, no shared-address atomics)
  auto wsum = [](int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
  };
  int wmax = nsw, cmax = (int)g_pgs_prof[8 * e + 5];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o)), cmax = max(cmax, __shfl_xor(cmax, o));
  // per-lane census of lanes in waves on a non-y sweep: [43..46] npost 0..3+, [47..49] extras on
  // the free body 0/1/2+, [50] > 5 contacts, [51] active limit, [52] overflow rows
  const long long cv = g_pgs_prof[8 * e + 3];
  const bool ny = (cv & 15) >= 2;
  int census[10];
#pragma unroll
  for (int k = 0; k < 4; k++) census[k] = wsum(ny && ((cv >> 8) & 3) == k);
#pragma unroll
  for (int k = 0; k < 3; k++) census[4 + k] = wsum(ny && min((int)((cv >> 12) & 3), 2) == k);
  census[7] = wsum(ny && ((cv >> 16) & 1)), census[8] = wsum(ny && ((cv >> 17) & 1)),
  census[9] = wsum(ny && ((cv >> 18) & 1));
  const int nsw_sum = wsum(nsw), lanes = wsum(1);
  int why[7];
#pragma unroll
  for (int k = 0; k < 7; k++) why[k] = wsum((int)((cv >> (41 + k)) & 1));
  if ((threadIdx.x & 63) == 0 && WPH_ID() < WPH_MAXW) {
    WPH_MAX(15, cmax);
    WPH_ADD(6, nsw_sum);
    WPH_ADD(7, lanes);
#pragma unroll
    for (int k = 0; k < 10; k++) WPH_ADD(43 + k, census[k]);
    WPH_ADD(0, t1 - t0);
    WPH_ADD(1, t2 - t1);
    WPH_ADD(2, p0 - t2);
    WPH_ADD(3, p1 - p0);
    WPH_ADD(4, t5 - p1);
    WPH_MAX(8, t5 - t0);
    {
      int var = (int)g_pgs_prof[8 * e + 3] & 15;
      WPH_ADD(9, var == 0);
      WPH_ADD(19 + var, 1);
      WPH_MAX(23 + var, t5 - t0);
    }
    WPH_ADD(27, anyfree);
    for (int k = 0; k < 15; k++) WPH_ADD(28 + k, g_stamp[16 * e + k + 1] - g_stamp[16 * e + k]);
    for (int k = 0; k < 4; k++) WPH_ADD(53 + k, g_rowprof[4 * e + k]);
    WPH_ADD(16, g_pgs_prof[8 * e + 6] - t2);
    WPH_ADD(17, g_pgs_prof[8 * e + 7] - g_pgs_prof[8 * e + 6]);
    WPH_ADD(18, p0 - g_pgs_prof[8 * e + 7]);
    WPH_ADD(12, anylim);
    WPH_ADD(13, anyslow);
    WPH_ADD(14, anyovf);
    WPH_MAX(10, p1 - p0);
    WPH_ADD(11, wmax);
    WPH_ADD(5, 1);
    if ((cv >> 40) & 1) {
      WPH_ADD(82, 1), WPH_MAX(83, t5 - t0), WPH_ADD(84, t5 - t0);
#pragma unroll
      for (int k = 0; k < 7; k++) WPH_ADD(85 + k, why[k]);
    }
    const int ast = (int)((g_pgs_prof[8 * e + 3] >> 20) & 255);
    if (ast) WPH_ADD(57, 1), WPH_ADD(58, ast);
    WPH_MAX(ast ? 60 : 59, t5 - t0);
    const int xv = (int)((g_pgs_prof[8 * e + 3] >> 28) & 7);
    if (xv >= 4) {
      WPH_ADD(61 + xv - 4, 1);
      WPH_MAX(65 + xv - 4, t5 - t0);
      WPH_ADD(69 + xv - 4, p1 - p0);
      WPH_ADD(73 + xv - 4, ast);
    }
  }
#endif
}

}  // namespace soarm
