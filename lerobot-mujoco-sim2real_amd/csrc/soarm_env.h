// soarm_env.h — the per-env bodies of reset / observe / bias / IK / keyed draws and the state
// load / store: shared by the device kernels (soarm_sim.hip, one lane per env) and the CPU
// backend (soarm_cpu.hip, device = -1), so both run the same code.
#pragma once
#include "../../include/soarm_sim.h"
#include "soarm_step.h"

namespace soarm {

// ------------------------------------------------------------- Philox4x32-10
struct u4 {
  uint32_t x, y, z, w;
};
HDI u4 philox(u4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
HDI float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
// lo + (hi - lo) u with two roundings (no FMA contraction): the host mirror
// (sim.reset_qpos_draw / workloads.philox_uniform) reproduces it bit for bit
HDI float uniform_range(float lo, float width, float u) {
#pragma clang fp contract(off)
  const float t = width * u;
  return lo + t;
}

template <int NA, int NF>
HDI void load_state(Sim<NA, NF>& S, const sim_state& st, int n, int e) {
  constexpr int NQ = Sim<NA, NF>::NQ, NV = Sim<NA, NF>::NV;
#pragma unroll
  for (int i = 0; i < NQ; i++) S.qpos[i] = soa(launder(st.qpos), i, n, e);
#pragma unroll
  for (int i = 0; i < NV; i++) {
    S.qvel[i] = soa(launder(st.qvel), i, n, e);
    S.warm[i] = soa(launder(st.qacc_warmstart), i, n, e);
  }
#pragma unroll
  for (int i = 0; i < NA; i++) S.ctrl[i] = (i < S.mp->nu) ? soa(launder(st.ctrl), i, n, e) : 0.f;
  S.status = st.status[e];
}
template <int NA, int NF>
HDI void store_state(const Sim<NA, NF>& S, const sim_state& st, int n, int e) {
  constexpr int NQ = Sim<NA, NF>::NQ, NV = Sim<NA, NF>::NV;
#pragma unroll
  for (int i = 0; i < NQ; i++) soa(launder(st.qpos), i, n, e) = S.qpos[i];
#pragma unroll
  for (int i = 0; i < NV; i++) {
    soa(launder(st.qvel), i, n, e) = S.qvel[i];
    soa(launder(st.qacc_warmstart), i, n, e) = S.warm[i];
  }
#pragma unroll
  for (int i = 0; i < NA; i++)
    if (i < S.mp->nu) soa(launder(st.ctrl), i, n, e) = S.ctrl[i];
  st.status[e] = S.status;
}
template <int NA, int NF>
HDI void write_obs(const Sim<NA, NF>& S, float* obs, int e) {
  constexpr int NQ = Sim<NA, NF>::NQ;
  const int no = 3 + S.mp->obs_nq;
  float* o = obs + (size_t)e * no;
  o[0] = S.ee[0], o[1] = S.ee[1], o[2] = S.ee[2];
  for (int k = 0; k < S.mp->obs_nq; k++) {
    const int a = S.mp->obs_qadr[k];
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NQ; i++)
      if (i == a) v = S.qpos[i];
    o[3 + k] = v;
  }
}


// mj_resetData zeroes d.qfrc_applied: a reset / soft reset of env e clears its row
HDI void zero_applied(float* applied, int nv, int n, int e) {
  for (int i = 0; i < nv; i++) soa(applied, i, n, e) = 0.f;
}


template <int NA, int NF>
HDI void env_reset(const DModel* __restrict__ dm, int n, int e, const sim_state& st,
                                              const float* __restrict__ init_qpos,
                                              const float* __restrict__ init_qvel,
                                              const float* __restrict__ extra_qpos, uint32_t k0,
                                              uint32_t k1, long long env_offset,
                                              const uint8_t* __restrict__ mask,
                                              float* __restrict__ obs) {
  constexpr int NQ = Sim<NA, NF>::NQ, NV = Sim<NA, NF>::NV;
  if (mask && !mask[e]) return;
  const DModel& m = *dm;
  Sim<NA, NF> S(dm, 1.f, -1.f, 1.f);
#pragma unroll
  for (int i = 0; i < NQ; i++) S.qpos[i] = extra_qpos ? extra_qpos[(size_t)i * n + e] : m.qpos0[i];
#pragma unroll
  for (int i = 0; i < NV; i++) S.qvel[i] = S.warm[i] = 0.f;
#pragma unroll
  for (int i = 0; i < NA; i++) S.ctrl[i] = 0.f;
  S.status = 0;
  // SOARM101_Env.py:90-99: qpos[joint_ids] = U(-0.3, 0.3) (or options), qvel[joint_ids] = 0 (or options)
  const unsigned long long gid = (unsigned long long)(env_offset + e);
  u4 r0 = philox(u4{(uint32_t)gid, (uint32_t)(gid >> 32), 0u, 0u}, k0, k1);
  u4 r1 = philox(u4{(uint32_t)gid, (uint32_t)(gid >> 32), 1u, 0u}, k0, k1);
  const uint32_t rr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
  for (int k = 0; k < m.obs_nq; k++) {
    const int a = m.obs_qadr[k];  // arm joint: qpos address == dof address
    const float qv = init_qpos ? init_qpos[(size_t)k * n + e] : uniform_range(-0.3f, 0.6f, u01(rr[k & 7]));
    const float vv = init_qvel ? init_qvel[(size_t)k * n + e] : 0.f;
#pragma unroll
    for (int i = 0; i < NQ; i++)
      if (i == a) S.qpos[i] = qv;
#pragma unroll
    for (int i = 0; i < NV; i++)
      if (i == a) S.qvel[i] = vv;
  }
  S.kinematics();
  store_state(S, st, n, e);
  if (st.ncon) st.ncon[e] = 0.f;
  if (st.qfrc_applied) zero_applied(st.qfrc_applied, NV, n, e);
  if (obs) write_obs(S, obs, e);
}

// keyed uniform draws of sim_rand_uniform for env e (stream layout: k_rand, soarm_sim.hip)
HDI void env_rand(int e, uint32_t k0, uint32_t k1, long long env_offset, uint32_t counter, int k, float lo,
                  float width, float* __restrict__ out) {
  const unsigned long long gid = (unsigned long long)(env_offset + e);
  for (int b = 0; 4 * b < k; b++) {
    const u4 r = philox(u4{(uint32_t)gid, (uint32_t)(gid >> 32), counter, 1u + (uint32_t)b}, k0, k1);
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (4 * b + j < k) out[(size_t)e * k + 4 * b + j] = uniform_range(lo, width, u01(rr[j]));
  }
}

// qfrc_bias at the current state (mj_comVel + mj_rne with flg_acc = 0, as left by mj_forward)
template <int NA, int NF>
HDI void env_bias(const DModel* __restrict__ dm, int n, int e, const sim_state& st, float* __restrict__ bias,
                  const sim_params& pp) {
  Sim<NA, NF> S(dm, pp.mass_scale ? pp.mass_scale[e] : 1.f, pp.friction ? pp.friction[e] : -1.f,
                pp.damping_scale ? pp.damping_scale[e] : 1.f);
  load_state(S, st, n, e);
  S.kinematics();
  S.com_crb();
  S.template smooth_forces<true>();
#pragma unroll
  for (int i = 0; i < Sim<NA, NF>::NV; i++) soa(bias, i, n, e) = -S.fsmooth[i];
}

template <int NA, int NF>
HDI void env_observe(const DModel* __restrict__ dm, int n, int e, const sim_state& st, float* __restrict__ obs) {
  Sim<NA, NF> S(dm, 1.f, -1.f, 1.f);
  load_state(S, st, n, e);
  S.kinematics();
  write_obs(S, obs, e);
}

// ------------------------------------------------------------ DLS site IK
// dm_control qpos_from_site_pose (control/TrajectoryGenerator.py:96-107), joints = the first
// `ndof` arm hinges; tq (target quaternions [N][4], w x y z) null = position only
// (target_quat=None at Koopman_MPC.py:252):
//   err = [target - site_xpos ; quat2vel(target_quat * conj(site_xquat))]   (3 or 6 rows)
//   err_norm = |err_pos| + rot_weight |err_rot|;  stop (success) if err_norm < tol
//   J = site jacobian [jacp; jacr];  reg = strength if err_norm > threshold else 0
//   position only: dq = J' (J J' + reg I)^-1 err  (== (J'J + reg I)^-1 J' err; reg = 0 -> min-norm)
//   pose: dq = (J'J + reg I)^-1 J' err  (6 rows over 5 dofs: J'J is regular away from singular
//         poses; where its LDL' meets a non-positive pivot the solve stops as failed, where
//         dm_control's lstsq would drop the direction)
//   stop (fail) if err_norm / |dq| > progress_thresh;  clip |dq| <= max_update_norm
//   q += dq  (hinges: mj_integratePos is plain addition; joint ranges not enforced)
template <int NA>
HDI void env_ik(const DModel* __restrict__ dm, int n, int e, const float* __restrict__ target,
                const float* __restrict__ tq, float* __restrict__ q, int32_t* __restrict__ ok,
                int32_t* __restrict__ iters, const sim_ik_opts& o) {
  const DModel& m = *dm;
  Sim<NA, 0> S(dm, 1.f, -1.f, 1.f);
#pragma unroll
  for (int i = 0; i < NA; i++) S.qpos[i] = q[(size_t)i * n + e];
  const float tx = target[3 * (size_t)e], ty = target[3 * (size_t)e + 1], tz = target[3 * (size_t)e + 2];
  float tqt[4] = {1.f, 0.f, 0.f, 0.f};
  if (tq)
#pragma unroll
    for (int k = 0; k < 4; k++) tqt[k] = tq[4 * (size_t)e + k];
  const int sb = m.site_bodyid[m.obs_site];
  int success = 0, it = 0;
  for (; it < o.max_steps; it++) {
    S.kinematics();
    float err[6] = {tx - S.ee[0], ty - S.ee[1], tz - S.ee[2], 0.f, 0.f, 0.f};
    float en = sqrtf(dot3(err, err));
    if (tq) {
      // site quaternion = body quaternion * site quaternion; err quat = target * conj(site)
      float bq[4] = {1.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 1; b < Sim<NA, 0>::NB; b++)
        if (b == sb) bq[0] = S.xquat[b][0], bq[1] = S.xquat[b][1], bq[2] = S.xquat[b][2], bq[3] = S.xquat[b][3];
      const float sq_[4] = {m.site_quat[m.obs_site][0], m.site_quat[m.obs_site][1], m.site_quat[m.obs_site][2],
                            m.site_quat[m.obs_site][3]};
      float sq[4], eq[4];
      qmul(sq, bq, sq_);
      qnormalize(sq);
      const float cq[4] = {sq[0], -sq[1], -sq[2], -sq[3]};
      qmul(eq, tqt, cq);
      const float s = sqrtf(eq[1] * eq[1] + eq[2] * eq[2] + eq[3] * eq[3]);  // mju_quat2Vel, dt = 1
      if (s >= 1e-15f) {
        float speed = 2.f * atan2f(s, eq[0]);
        if (speed > 3.14159265358979f) speed -= 6.28318530717959f;
        err[3] = eq[1] / s * speed, err[4] = eq[2] / s * speed, err[5] = eq[3] / s * speed;
      }
      en += (float)o.rot_weight * sqrtf(err[3] * err[3] + err[4] * err[4] + err[5] * err[5]);
    }
    if (en < (float)o.tol) {
      success = 1;
      break;
    }
    // site jacobian: hinge i moves the site iff its body is an ancestor of the site body
    float J[6][NA];
#pragma unroll
    for (int i = 0; i < NA; i++) {
      float r[3] = {S.ee[0] - S.anchor[i][0], S.ee[1] - S.anchor[i][1], S.ee[2] - S.anchor[i][2]};
      float c[3];
      cross(c, S.axis[i], r);
      const bool use = (i < o.ndof) && (sb >= i + 2);
#pragma unroll
      for (int k = 0; k < 3; k++) J[k][i] = use ? c[k] : 0.f, J[3 + k][i] = use ? S.axis[i][k] : 0.f;
    }
    const float reg = en > (float)o.regularization_threshold ? (float)o.regularization_strength : 0.f;
    float dq[NA], dn2 = 0.f;
    if (!tq) {
      // A = J J' + reg I (3x3 SPD), solve A y = err, dq = J' y
      float A[6];
      A[0] = reg, A[1] = 0, A[2] = reg, A[3] = 0, A[4] = 0, A[5] = reg;  // packed lower: 00,10,11,20,21,22
#pragma unroll
      for (int i = 0; i < NA; i++) {
        A[0] += J[0][i] * J[0][i];
        A[1] += J[1][i] * J[0][i];
        A[2] += J[1][i] * J[1][i];
        A[3] += J[2][i] * J[0][i];
        A[4] += J[2][i] * J[1][i];
        A[5] += J[2][i] * J[2][i];
      }
      float Ad[3], y[3];
      ldl_factor<3>(A, Ad);
      ldl_solve<3>(A, Ad, y, err);
#pragma unroll
      for (int i = 0; i < NA; i++) dq[i] = J[0][i] * y[0] + J[1][i] * y[1] + J[2][i] * y[2];
    } else {
      // H = J'J + reg I over the joints (unused joints: identity rows, zero right-hand side)
      float H[NA * (NA + 1) / 2], g[NA], Hd[NA];
#pragma unroll
      for (int a = 0; a < NA; a++) {
        float ga = 0.f;
#pragma unroll
        for (int k = 0; k < 6; k++) ga += J[k][a] * err[k];
        g[a] = ga;
#pragma unroll
        for (int b = 0; b <= a; b++) {
          float h = 0.f;
#pragma unroll
          for (int k = 0; k < 6; k++) h += J[k][a] * J[k][b];
          const bool used = a < o.ndof && sb >= a + 2;
          H[a * (a + 1) / 2 + b] = a == b ? (used ? h + reg : 1.f) : h;
        }
      }
      ldl_factor<NA>(H, Hd);
      bool spd = true;  // a non-positive pivot: J'J singular to fp32 (singular pose) -> fail
#pragma unroll
      for (int a = 0; a < NA; a++) spd &= Hd[a] > 0.f && Hd[a] < 3.0e38f;
      if (!spd) break;
      ldl_solve<NA>(H, Hd, dq, g);
    }
#pragma unroll
    for (int i = 0; i < NA; i++) dn2 += dq[i] * dq[i];
    const float dn = sqrtf(dn2);
    if (en / dn > (float)o.progress_thresh) break;
    if (dn > (float)o.max_update_norm) {
      const float s = (float)o.max_update_norm / dn;
#pragma unroll
      for (int i = 0; i < NA; i++) dq[i] *= s;
    }
#pragma unroll
    for (int i = 0; i < NA; i++) S.qpos[i] += dq[i];
  }
#pragma unroll
  for (int i = 0; i < NA; i++) q[(size_t)i * n + e] = S.qpos[i];
  if (ok) ok[e] = success;
  if (iters) iters[e] = it;
}

}  // namespace soarm
