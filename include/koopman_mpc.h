/*
 * koopman_mpc.h — C ABI of the batched Koopman-MPC controller.
 *
 * The reference runs one Koopman-MPC controller on one env, serially, with casadi/IPOPT
 * (control/MPC_Controler.py) inside the Koopman_MPC.py tracking loop:
 *
 *   MPCController.Psi_o(s)        z = [x, MLP(x)] lifted state       control/MPC_Controler.py:154-167
 *                                 (Koopmanlinear.x_encoder, models/KoopmanBase.py:45-47)
 *   MPCController.setup_delta_mpc unconstrained QP over H = 10 moves   control/MPC_Controler.py:100-141
 *   MPCController.setup_mpc       (the same over absolute inputs)      control/MPC_Controler.py:65-98
 *   MPCController.get_control(p)  u0 = u_opt[0] + u_prev, a = clip    control/MPC_Controler.py:143-152
 *   Test.runMPC                   lifted refs, z0, solve, env.step     Koopman_MPC.py:197-222
 *
 * The QP has no constraints (nlpsol is called without bounds, MPC_Controler.py:145) and a
 * constant Hessian for the linear Koopman model (DKUC, the default), so IPOPT's optimum is the
 * closed form  u0 = Gr·r + Gz·z0 + Gu·u_prev  (r = the H lifted reference points stacked).
 * The host computes (Gr, Gz, Gu) once per controller; these entry points run the per-env work
 * on the GPU for a whole batch of envs:
 *
 *   sim_koopman_encode       Psi_o for M states (f64 MFMA encoder)
 *   sim_koopman_feedforward  Gr·r for every frame of a reference trajectory (f64 MFMA)
 *   sim_koopman_mpc_step     z0 = Psi_o(x); u0; a = clip(u0); u_prev = u0 (one launch)
 *
 * Arithmetic is float64 throughout, as in the reference (model.double(), Koopman_MPC.py:263).
 * Device buffers are caller-owned; calls are asynchronous on the given stream (void* =
 * hipStream_t, NULL = default).  Errors: negative SIM_E_* codes (soarm_sim.h) and
 * sim_last_error().
 */
#ifndef KOOPMAN_MPC_H
#define KOOPMAN_MPC_H

#include <stdint.h>

#include "soarm_sim.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SIM_KMAXLAYER 6 /* encoder linear layers */
#define SIM_KMAXW 64    /* hidden / output width of every encoder layer */
#define SIM_KMAXX 8     /* x_dim */
#define SIM_KMAXU 8     /* u_dim */
#define SIM_KMAXH 32    /* horizon */

typedef struct sim_koopman_desc {
  int32_t x_dim;                    /* 8: [ee_xyz(3), q(5)] (args.x_dim)  */
  int32_t u_dim;                    /* 5 (args.u_dim) */
  int32_t nlayer;                   /* linear layers of x_encode_net (5 for args.layers) */
  int32_t width[SIM_KMAXLAYER + 1]; /* [x_dim, 64, 64, 64, 64, 24] (args.py:103) */
  int32_t horizon;                  /* H = 10 (MPC_Controler.py:27) */
  int32_t _pad;
  double u_clip;                    /* 0.5: a = clip(u0, -0.5, 0.5) (MPC_Controler.py:149) */
} sim_koopman_desc;

typedef struct sim_koopman sim_koopman;

/* weights: per layer l, W_l [width[l+1]][width[l]] row-major (nn.Linear.weight) then b_l
   [width[l+1]]; ReLU between layers, none after the last (models/KoopmanBase.py:20-25).
   gain: [u_dim][H*nz + nz + u_dim] row-major = [Gr | Gz | Gu], nz = x_dim + width[nlayer]. */
int sim_koopman_create(const sim_koopman_desc* desc, const double* weights, const double* gain,
                       int device, sim_koopman** out);
void sim_koopman_free(sim_koopman* k);

/* Psi_o: z [nz][m] (SoA) = [x, MLP(x)] for x [m][x_dim] float32 rows (the reference lifts
   DoubleTensor(obs), obs being float32, Koopman_MPC.py:220-221). */
int sim_koopman_encode(sim_koopman* k, int m, const float* x, double* z, void* stream);

/* Feedforward of a lifted reference trajectory: for frame f < nframe,
   ff[f][u][e] = sum_t Gr_t · zref[f + 1 + t][:][e], terms with f + 1 + t >= nref being zero
   (the reference pads the window past the trajectory end with zero rows, Koopman_MPC.py:199-205).
   zref [nref][nz][n], ff [nframe][u_dim][n]. */
int sim_koopman_feedforward(sim_koopman* k, int nframe, int nref, int n, const double* zref, double* ff,
                            void* stream);

/* One control step for n envs: z0 = Psi_o(x) (or the given z0 [nz][n]), then
   u0 = ff + Gz z0 + Gu u_prev; u_prev <- u0; action = clip(u0) as float32.
   x [n][x_dim] float32 (ignored when z0 != NULL), ff [u_dim][n] (NULL = 0),
   u_prev [u_dim][n] in/out, action [n][u_dim]. */
int sim_koopman_mpc_step(sim_koopman* k, int n, const float* x, const double* z0, const double* ff,
                         double* u_prev, float* action, void* stream);

/* The bilinear DBKN model (models/KoopmanBase.py:62-110): its input matrix is linearised at each
   env's lifted state, B_total = B + sum_j z0_j Hhat_j (linearize_B, MPC_Controler.py:46-63), so
   the condensed QP of MPC_Controler.py:65-141 (state_full: Q = q I, R = r I) is solved per env and
   frame.  set_bilinear: A [nz][nz], B [nz][u_dim], Hhat [nz (j)][nz][u_dim] (get_Hi_numpy), delta
   (1 = 'delta_mpc', 0 = 'mpc'), q = 50, r = 0.5.  bilinear_step: z0 [nz][n], window [H][nz][n]
   (lifted reference rows k+1 .. k+H, zero past the end), u_prev [u_dim][n] in/out (u_prev <- u0),
   action [n][u_dim] = clip(u0) float32.  Replaces the casadi solve of get_control for DBKN. */
int sim_koopman_set_bilinear(sim_koopman* k, const double* A, const double* B, const double* Hhat, int delta,
                             double q, double r);
int sim_koopman_bilinear_step(sim_koopman* k, int n, const double* z0, const double* window, double* u_prev,
                              float* action, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KOOPMAN_MPC_H */
