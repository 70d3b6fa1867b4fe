/*
 * soarm_sim.h — C ABI of the MI355X-native batched SO-ARM101 simulator.
 *
 * This is the drop-in boundary for the reference's hot path
 * (SURVEY.md §8b).  In the reference, the Python layer calls MuJoCo's C engine
 * through its Python bindings:
 *
 *   mujoco.MjModel.from_xml_path(xml)        SOARM101/SOARM101_Env.py:34
 *   mujoco.MjData(model)                     SOARM101/SOARM101_Env.py:43
 *   mujoco.mj_resetData(model, data)         SOARM101/SOARM101_Env.py:87
 *   mujoco.mj_forward(model, data)           SOARM101/SOARM101_Env.py:102
 *   mujoco.mj_step(model, data)  (x frame_skip) SOARM101/SOARM101_Env.py:131-132
 *   data.site_xpos / data.qpos  (obs)        SOARM101/SOARM101_Env.py:71-75
 *   dm_control qpos_from_site_pose (IK)      control/TrajectoryGenerator.py:96-107
 *
 * Each of those is replaced by one batched entry point below that runs on a
 * whole batch of environments (envs) on one GPU.  Plain C types only: device
 * pointers are passed as raw pointers, sizes as ints, streams as void*
 * (a hipStream_t; NULL = the default stream).  Every function returns 0 on
 * success or a negative SIM_E* code; sim_last_error() returns a thread-local
 * message for the last failure.
 *
 * Memory: the library owns the model constants (one device copy per
 * sim_batch) and its scratch.  Env state is caller-owned device memory laid out
 * structure-of-arrays, [field][env] (so lane i of a wave reads env i: coalesced).
 * Nothing inside sim_step/sim_reset allocates, synchronises or copies between
 * host and device, so a caller may capture them in a hipGraph.
 */
#ifndef SOARM_SIM_H
#define SOARM_SIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ABI version: the leading (struct_size, abi_version) of every by-pointer struct below is
   checked by the entry point that reads it, so a caller built against another layout gets
   SIM_E_ARG instead of a misread.  Bumped with any layout change. ---- */
#define SIM_ABI_VERSION 2

/* ---- capacity of the compiled model (MuJoCo mjModel subset) ---- */
#define SIM_MAXBODY 12
#define SIM_MAXJNT 12
#define SIM_MAXDOF 16
#define SIM_MAXQ 20
#define SIM_MAXGEOM 40
#define SIM_MAXPAIR 160
#define SIM_MAXSITE 4
#define SIM_MAXU 8
#define SIM_MAXOBSQ 8
#define SIM_MAXCON 16 /* contacts kept per env per substep */

/* MuJoCo enum values (mjtJoint, mjtGeom) */
enum { SIM_JNT_FREE = 0, SIM_JNT_BALL = 1, SIM_JNT_SLIDE = 2, SIM_JNT_HINGE = 3 };
enum { SIM_GEOM_PLANE = 0, SIM_GEOM_SPHERE = 2, SIM_GEOM_BOX = 6, SIM_GEOM_MESH = 7 };
/* mjtSolver values */
enum { SIM_SOL_PGS = 0, SIM_SOL_CG = 1, SIM_SOL_NEWTON = 2 };
/* convex-convex narrowphase: libccd MPR (MuJoCo's classic path) or MuJoCo's native GJK/EPA
   ("nativeccd", the default of current releases) */
enum { SIM_CCD_MPR = 0, SIM_CCD_NATIVE = 1 };

/* error codes */
enum {
  SIM_OK = 0,
  SIM_E_ARG = -1,      /* bad argument / shape */
  SIM_E_MODEL = -2,    /* model outside what the kernels support */
  SIM_E_HIP = -3,      /* HIP runtime error */
  SIM_E_NODEVICE = -4, /* no GPU visible */
};

/* per-env status bits (sim_state.status) */
enum {
  SIM_ST_BADQPOS = 1,   /* mj_checkPos: non-finite or |qpos| > 1e10 -> env auto-reset */
  SIM_ST_BADQVEL = 2,   /* mj_checkVel */
  SIM_ST_BADQACC = 4,   /* mj_checkAcc */
  SIM_ST_CONOVERFLOW = 8 /* more than SIM_MAXCON contacts in a substep (extra dropped) */
};

/*
 * Compiled model.  Field names and meanings follow MuJoCo's mjModel
 * (mjmodel.h) so the MJCF compiler (lerobot-mujoco-sim2real_amd/mjcf.py) and
 * the oracle read the same numbers.  Quaternions are (w, x, y, z).
 */
typedef struct sim_model_desc {
  int32_t struct_size;   /* sizeof(sim_model_desc) as the caller compiled it */
  int32_t abi_version;   /* SIM_ABI_VERSION */
  int32_t nbody, njnt, nq, nv, nu, ngeom, nsite, npair;
  int32_t nhullvert, nhulladj; /* lengths of the hull arrays passed beside */

  /* mjOption */
  double timestep;
  double gravity[3];
  double impratio;
  double tolerance;      /* solver: stop when the scaled cost improvement is below this */
  double meaninertia;    /* mjStatistic.meaninertia = trace(M(qpos0)) / nv (mj_setConst): the
                            solvers' stopping tests scale by 1 / (meaninertia * max(1, nv)) */
  int32_t iterations;    /* solver: max PGS sweeps / Newton iterations */
  int32_t disable_contact; /* mjDSBL_CONTACT */
  int32_t disable_eulerdamp;
  int32_t solver;        /* mjtSolver: SIM_SOL_PGS (soarm_pgs.h) or SIM_SOL_NEWTON (MuJoCo's
                            default, soarm_newton.h); SIM_SOL_CG is rejected (SIM_E_MODEL) */
  int32_t ccd;           /* SIM_CCD_*: mesh-mesh / box-mesh narrowphase (mjDSBL_NATIVECCD off = native) */
  int32_t _pad0;

  /* bodies (0 = world) */
  int32_t body_parentid[SIM_MAXBODY];
  int32_t body_rootid[SIM_MAXBODY];
  int32_t body_weldid[SIM_MAXBODY];
  int32_t body_jntnum[SIM_MAXBODY];
  int32_t body_jntadr[SIM_MAXBODY];
  int32_t body_dofnum[SIM_MAXBODY];
  int32_t body_dofadr[SIM_MAXBODY];
  double body_pos[SIM_MAXBODY][3];
  double body_quat[SIM_MAXBODY][4];
  double body_ipos[SIM_MAXBODY][3];
  double body_iquat[SIM_MAXBODY][4];
  double body_mass[SIM_MAXBODY];
  double body_inertia[SIM_MAXBODY][3]; /* principal moments */
  double body_invweight0[SIM_MAXBODY][2];

  /* joints */
  int32_t jnt_type[SIM_MAXJNT];
  int32_t jnt_bodyid[SIM_MAXJNT];
  int32_t jnt_qposadr[SIM_MAXJNT];
  int32_t jnt_dofadr[SIM_MAXJNT];
  int32_t jnt_limited[SIM_MAXJNT];
  int32_t _pad1;
  double jnt_pos[SIM_MAXJNT][3];
  double jnt_axis[SIM_MAXJNT][3];
  double jnt_range[SIM_MAXJNT][2];
  double jnt_solref[SIM_MAXJNT][2];
  double jnt_solimp[SIM_MAXJNT][5];
  double jnt_margin[SIM_MAXJNT];
  double qpos0[SIM_MAXQ];

  /* dofs */
  int32_t dof_bodyid[SIM_MAXDOF];
  int32_t dof_jntid[SIM_MAXDOF];
  int32_t dof_parentid[SIM_MAXDOF];
  double dof_armature[SIM_MAXDOF];
  double dof_damping[SIM_MAXDOF];
  double dof_frictionloss[SIM_MAXDOF];
  double dof_invweight0[SIM_MAXDOF];
  double dof_solref[SIM_MAXDOF][2];
  double dof_solimp[SIM_MAXDOF][5];

  /* geoms (only collidable geoms are compiled in; visual ones are dropped) */
  int32_t geom_type[SIM_MAXGEOM];
  int32_t geom_bodyid[SIM_MAXGEOM];
  int32_t geom_condim[SIM_MAXGEOM];
  int32_t geom_hulladr[SIM_MAXGEOM]; /* first vertex in hull_vert (mesh only, else -1) */
  int32_t geom_hullnum[SIM_MAXGEOM];
  int32_t _pad2;
  double geom_pos[SIM_MAXGEOM][3];
  double geom_quat[SIM_MAXGEOM][4];
  double geom_size[SIM_MAXGEOM][3];
  double geom_friction[SIM_MAXGEOM][3];
  double geom_solref[SIM_MAXGEOM][2];
  double geom_solimp[SIM_MAXGEOM][5];
  double geom_margin[SIM_MAXGEOM];
  double geom_rbound[SIM_MAXGEOM];     /* bounding-sphere radius about geom_aabb centre */
  double geom_aabb[SIM_MAXGEOM][6];    /* local-frame box: centre(3), half-size(3) */

  /* candidate collision pairs, in MuJoCo's deterministic contact order */
  int32_t pair_geom1[SIM_MAXPAIR];
  int32_t pair_geom2[SIM_MAXPAIR];

  /* sites */
  int32_t site_bodyid[SIM_MAXSITE];
  double site_pos[SIM_MAXSITE][3];
  double site_quat[SIM_MAXSITE][4];

  /* actuators: joint transmission, fixed gain, affine bias (mjGAIN_FIXED/mjBIAS_AFFINE) */
  int32_t actuator_trnid[SIM_MAXU]; /* joint id */
  int32_t actuator_ctrllimited[SIM_MAXU];
  int32_t actuator_forcelimited[SIM_MAXU];
  double actuator_gear[SIM_MAXU];
  double actuator_gainprm[SIM_MAXU];    /* gainprm[0] */
  double actuator_biasprm[SIM_MAXU][3];
  double actuator_ctrlrange[SIM_MAXU][2];
  double actuator_forcerange[SIM_MAXU][2];

  /* observation recipe (SOARM101Env._get_state, SOARM101_Env.py:69-75):
     obs = [site_xpos[obs_site] (3), qpos[obs_qadr[0..obs_nq-1]]] */
  int32_t obs_site;
  int32_t obs_nq;
  int32_t obs_qadr[SIM_MAXOBSQ];
  int32_t nact; /* how many leading ctrl entries an action writes (udim = 5) */
  int32_t _pad3;
} sim_model_desc;

/* DLS-IK options (dm_control qpos_from_site_pose semantics) */
typedef struct sim_ik_opts {
  int32_t struct_size;        /* sizeof(sim_ik_opts) */
  int32_t abi_version;        /* SIM_ABI_VERSION */
  double tol;                 /* 1e-6 */
  double regularization_threshold; /* 0.1 */
  double regularization_strength;  /* 1e-2 */
  double max_update_norm;     /* 2.0 */
  double progress_thresh;     /* 20.0 */
  int32_t max_steps;          /* 100 */
  int32_t site;               /* site id */
  int32_t ndof;               /* number of leading dofs moved (5) */
  int32_t _pad;
  double rot_weight;          /* 0.5: weight of |err_rot| in the error norm (pose targets) */
} sim_ik_opts;

/* Env state: caller-owned DEVICE buffers, SoA [field][n_envs]. */
typedef struct sim_state {
  float* qpos;            /* [nq][N]  */
  float* qvel;            /* [nv][N]  */
  float* qacc_warmstart;  /* [nv][N]  */
  float* ctrl;            /* [nu][N]  */
  int32_t* status;        /* [N]      SIM_ST_* bits, OR-ed since last reset */
  float* ncon;            /* [N]      running contact-count sum (for contacts/env/substep) */
  float* qfrc_applied;    /* [nv][N]  MjData.qfrc_applied, or NULL (= 0): added to the smooth
                             forces of every substep; zeroed with the env on a reset / soft
                             reset, as mj_resetData does.  Koopman_MPC.py:119 writes it
                             (gravity compensation qfrc_applied = qfrc_bias) */
} sim_state;

/* Optional per-env domain-randomisation parameters (DEVICE, [N] each; NULL = nominal). */
typedef struct sim_params {
  const float* mass_scale;     /* body mass (and inertia) x scale, all bodies */
  const float* friction;       /* sliding friction of every collidable geom */
  const float* damping_scale;  /* dof damping x scale */
} sim_params;

typedef struct sim_model sim_model;
typedef struct sim_batch sim_batch;

const char* sim_last_error(void);
const char* sim_version(void);

/* replaces MjModel.from_xml_path (compilation itself happens in mjcf.py);
   hull_vert [nhullvert][3], hull_adr [nhullvert+1] CSR, hull_adj [nhulladj] local ids */
int sim_model_create(const sim_model_desc* desc, const float* hull_vert, const int32_t* hull_adr,
                     const int32_t* hull_adj, sim_model** out);
/* frees the model and its device copies; every batch of the model must be freed first */
void sim_model_free(sim_model* m);

/* Compiled-model files, the MjModel.from_xml_path (SOARM101_Env.py:34) of a C / C++ caller with no
   Python at run time: mjcf.py compiles the MJCF once (CompiledModel.save) and writes the desc and
   hull arrays; sim_model_load reads them back and calls sim_model_create.  Format (little endian):
   "SOARMMDL" | u32 version (2) | u32 sizeof(sim_model_desc) | desc | f32 hull_vert[nhullvert][3] |
   i32 hull_adr[nhullvert+1] (absent when nhullvert = 0) | i32 hull_adj[nhulladj].  A file of
   another version or desc size, or a short file, is rejected (SIM_E_ARG). */
int sim_model_save(const sim_model_desc* desc, const float* hull_vert, const int32_t* hull_adr,
                   const int32_t* hull_adj, const char* path);
int sim_model_load(const char* path, sim_model** out);

/* replaces MjData(model) for n_envs envs on `device` (HIP ordinal).  The model's
   read-only device data (constants, hull records, support LUT) is uploaded by the
   first batch on a device and shared by the model's later batches there.
   device = -1: the CPU backend -- the same per-env physics compiled
   for the host, envs split over SOARM_CPU_THREADS (else OMP_NUM_THREADS, else all
   cores) threads.  Every call then takes HOST pointers in the same layouts, ignores
   `stream` and returns when done; sim_profile_* / sim_collide_profile need a GPU batch.
   The constraint solve is a dense scalar restatement of mj_solPGS / mj_solNewton in
   MuJoCo's row order (the kernels' lane-cooperative sweeps do not exist on the host). */
int sim_batch_create(const sim_model* m, int n_envs, int device, sim_batch** out);
void sim_batch_free(sim_batch* b);
int sim_batch_set_params(sim_batch* b, const sim_params* p);

/* replaces mj_resetData + qpos/qvel overwrite + mj_forward (SOARM101_Env.py:87-102)
   for envs with mask[i] != 0 (mask NULL = all).  init_qpos/init_qvel are
   [obs_nq][N] SoA device arrays written into qpos[obs_qadr]/qvel (NULL ->
   qpos drawn U(-0.3, 0.3) from Philox4x32-10 keyed by (seed, env_offset + i),
   qvel 0).  extra_qpos [nq][N] (or NULL) overrides the whole qpos0 first
   (used for the build-defined cube pose).  obs [N][3+obs_nq] row-major. */
int sim_reset(sim_batch* b, const sim_state* s, const float* init_qpos, const float* init_qvel,
              const float* extra_qpos, uint64_t seed, int64_t env_offset, const uint8_t* mask,
              float* obs, void* stream);

/* replaces ctrl[:nact] = action; frame_skip x mj_step; _get_state
   (SOARM101_Env.py:128-135).  action [N][nact] row-major, obs [N][3+obs_nq]. */
int sim_step(sim_batch* b, const sim_state* s, const float* action, int frame_skip, float* obs,
             void* stream);

/* keyed uniform draws of the rollout loop's input streams (replaces the reference's serial
   np.random.rand draws, SOARM101_DataCollection.py:115,132): out [N][k] row-major, out[i][j] =
   lo + (hi - lo) u, u from Philox4x32-10 keyed by (seed, env_offset + i, counter, j): the same
   env gets the same draws for any batch split or GPU count.  k <= 64. */
int sim_rand_uniform(sim_batch* b, uint64_t seed, int64_t env_offset, uint32_t counter, int k, float lo,
                     float hi, float* out, void* stream);

/* one plain mj_step-equivalent on the current ctrl, no obs (frame_skip substeps) */
int sim_substeps(sim_batch* b, const sim_state* s, int nsub, void* stream);

/* replaces reading d.qfrc_bias after mj_forward (Koopman_MPC.py:119,126): RNE with the
   current qvel, gravity + Coriolis/centrifugal, out [nv][N] */
int sim_bias(sim_batch* b, const sim_state* s, float* qfrc_bias, void* stream);

/* observation only (mj_kinematics + _get_state) */
int sim_observe(sim_batch* b, const sim_state* s, float* obs, void* stream);

/* replaces reading d.contact[:d.ncon] after mj_kinematics + mj_collision:
   out [N][SIM_MAXCON][8] = (dist, pos[3], normal[3] geom1->geom2, pair id as
   int32 bits), ncon [N].  Contact order = candidate-pair order (MuJoCo's). */
int sim_contacts(sim_batch* b, const sim_state* s, float* out, int32_t* ncon, void* stream);

/* diagnostic: geom poses + one collide pass with per-pair timing; cycles [2][npair]
   (host) = per pair, the sum over its waves of each wave's shader-clock cycles, then the
   largest single wave's.  Synchronous. */
int sim_collide_profile(sim_batch* b, const sim_state* s, double* cycles, void* stream);

/* diagnostic: summed wave cycles per phase of the contact substep kernel in a
   build compiled with -DSOARM_PHASE_PROF (out[101]; the first 19: load, smooth dynamics, rows,
   PGS, integrate+output, waves, sum of PGS sweeps over envs, envs, max wave
   cycles, waves on the register fast path, max wave PGS cycles, sum of per-wave
   max sweeps, waves with an active limit / a non-block contact / contact
   overflow past LDS, max contacts per env; then the rows phase split: contact rows,
   warm start + cost, register-block setup; the rest to 77: see g_phase in soarm_substep.h; 77..100:
   the Newton solver's counters, g_newton in soarm_newton.h, with the RS kernel's solve split in
   85..88, 93 and its fallback waves in 94..96; 101..107: the fallback lanes by cause -- out holds
   108 doubles);
   returns SIM_E_ARG in a regular build. */
int sim_phase_profile(double* out, int reset);

/* kernel timing: between begin and end, sim_step brackets every kernel launch
   with HIP events on its stream; end synchronises and returns the summed
   milliseconds and launch counts per kernel kind
   [0] fused step, [1] collide, [2] contact substep, [3] geom poses. */
#define SIM_PROF_KINDS 4
int sim_profile_begin(sim_batch* b);
int sim_profile_end(sim_batch* b, double* ms, int32_t* launches);

/* replaces dm_control qpos_from_site_pose, position-only (control/TrajectoryGenerator.py:96-107):
   target [N][3], q [nq][N] SoA in/out (warm start), ok [N] (1 = converged), iters [N] or NULL */
int sim_ik_dls(sim_batch* b, const float* target, float* q, int32_t* ok, int32_t* iters,
               const sim_ik_opts* opts, void* stream);
/* replaces dm_control qpos_from_site_pose with target_quat (control/TrajectoryGenerator.py:96-107,
   rot_weight 0.5): target_quat [N][4] (w, x, y, z) or NULL (= sim_ik_dls) */
int sim_ik_dls_pose(sim_batch* b, const float* target, const float* target_quat, float* q, int32_t* ok,
                    int32_t* iters, const sim_ik_opts* opts, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SOARM_SIM_H */
