// soarm_sim.hip — C ABI (include/soarm_sim.h) + kernels of the MI355X batched
// SO-ARM101 simulator.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC.
//
//   k_step   : ctrl[:nact] = action; frame_skip x mj_step; obs     (SOARM101_Env.py:108-142)
//   k_reset  : mj_resetData + init qpos/qvel + mj_forward + obs     (SOARM101_Env.py:77-106)
//   k_observe: mj_kinematics + _get_state                           (SOARM101_Env.py:69-75)
//   k_ik     : batched damped-least-squares site IK                 (control/TrajectoryGenerator.py:96-107)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <mutex>
#include <thread>
#include <vector>
#include <dlfcn.h>
#include <sched.h>
#include <vector>

#include "../../include/soarm_sim.h"
#ifdef SOARM_DIAG_SKIPP
// (diagnostic build: SOARM_DIAG_SKIP names pairs k_collide returns from at once; SOARM_DIAG_STAGE:
// 1 midphase only, 2 no mask atomics, 3 native GJK without EPA, else everything)
__device__ uint32_t g_diag_skip[4];
__device__ int g_diag_stage;
#define SOARM_DIAG_NO_EPA (g_diag_stage == 3)
#endif
#ifdef SOARM_DIAG_SUPPORT
__device__ unsigned long long g_diag_sup[16][4];  // (soarm_collide.h diag_support)
__device__ uint32_t g_diag_prev[2][128 * 8192];
#endif
#include "soarm_collide.h"
#include "soarm_env.h"
#include "sim_internal.h"
#include "soarm_pgs.h"

using namespace soarm;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
// the same error slot for the library's other translation units (koopman_mpc.hip)
int soarm_set_error(int code, const std::string& msg) { return fail(code, msg); }
#define HIPCHECK(x)                                                                   \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) return fail(SIM_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ tracing
// roctx ranges (SURVEY.md §5 tracing): with SOARM_ROCTX=1 every ABI call, and each stage of the
// contact env-step (geom poses, collide, substep, per substep), is bracketed by a roctx range
// that `rocprofv3 --marker-trace` records beside the kernel trace.  The roctx library is opened
// at run time, so the product has no link dependency on the profiler; the env-step is then
// launched stage by stage (no hipGraph replay) so that the ranges bracket real launches.
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* on = getenv("SOARM_ROCTX");
    if (!on || on[0] != '1') return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    pop = (int (*)())dlsym(h, "roctxRangePop");
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};
static const Roctx& roctx() {
  static const Roctx r;
  return r;
}
struct TraceRange {
  const bool on;
  explicit TraceRange(const char* name) : on(roctx().push != nullptr) {
    if (on) roctx().push(name);
  }
  ~TraceRange() {
    if (on) roctx().pop();
  }
};

// read-only model data on one device (constants, hull records, support LUT):
// uploaded by the first batch created on that device, shared by every later
// batch of the same model there, freed with the model
struct DevModel {
  int device = -1;
  DModel* d_model = nullptr;
  float4* d_hv = nullptr;
  int32_t *d_hadr = nullptr, *d_hadj = nullptr;
  uint16_t* d_hlut = nullptr;
  uint4 *d_hrec = nullptr, *d_hlutrec = nullptr;
  uint16_t* d_hovf = nullptr;
  float* d_hsb = nullptr;
  void release() {
    (void)hipSetDevice(device);
    (void)hipFree(d_model);
    (void)hipFree(d_hv);
    (void)hipFree(d_hadr);
    (void)hipFree(d_hadj);
    (void)hipFree(d_hlut);
    (void)hipFree(d_hrec);
    (void)hipFree(d_hlutrec);
    (void)hipFree(d_hovf);
    (void)hipFree(d_hsb);
  }
};

sim_model::~sim_model() {
  for (DevModel* d : dev) {
    d->release();
    delete d;
  }
}

struct sim_batch {
  const sim_model* model = nullptr;
  int n = 0, device = 0;
  CpuBatch* cpu = nullptr;     // device = -1: the CPU backend (soarm_cpu.hip) runs every call
  DModel* d_model = nullptr;   // shared per (model, device): DevModel
  float* d_scratch = nullptr;  // contact rows, [slot][env]
  size_t scratch_floats = 0;
  float* d_gpose = nullptr;    // body world frames [body*BREC+k][env] (soarm_collide.h load_pose)
  float* d_cbuf = nullptr;     // collide output [slot*7+f][env]
  int* d_ccount = nullptr;     // contacts per pair [pair][env]
  uint32_t* d_pmask = nullptr; // pairs with contacts, bit p%32 of word p/32: [word][env]
  float* d_sepax = nullptr;    // separating-axis cache [pair*3+k][env] (soarm_collide.h SepCache)
  // profiling (sim_profile_begin/end)
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<std::pair<int, size_t>> ev_marks;  // (kind, index of start event)
  sim_params params{nullptr, nullptr, nullptr};
  // hipGraph cache of the contact env-step's 1 + 2 x frame_skip launches, keyed by the
  // buffers the kernels are bound to (SOARM_NO_GRAPH=1 disables)
  struct GraphKey {
    sim_state s;
    const float* action;
    float* obs;
    int frame_skip;
    bool rs;  // the RS substep chosen (SOARM_RS, read per call): part of what the graph captured
    bool operator==(const GraphKey& o) const {
      return !memcmp(&s, &o.s, sizeof(s)) && action == o.action && obs == o.obs && frame_skip == o.frame_skip &&
             rs == o.rs;
    }
  };
  bool use_graphs = true;
  int rs_cap = 0;  // envs the RS substep runs in one round (4 per wave, one wave per SIMD)
  hipStream_t cap_stream = nullptr;
  std::vector<std::pair<GraphKey, hipGraphExec_t>> graphs;
  void drop_graphs() {
    for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
    graphs.clear();
  }
};

#include "soarm_substep.h"


// mj_collision, one lane per (env, candidate pair); blockIdx.y = pair
#ifndef SOARM_COLLIDE_BLOCK
#define SOARM_COLLIDE_BLOCK 256  // envs (lanes) per collide workgroup
#endif
#ifndef SOARM_EPA_SLOTS
#define SOARM_EPA_SLOTS 8  // EPA polytopes per native-collide workgroup in LDS (2.1 KB each)
#endif
#ifndef SOARM_COLLIDE_WAVES
#define SOARM_COLLIDE_WAVES 3  // min waves per SIMD (VGPR cap 512 / 3 = 168)
#endif
// CCD: one instantiation per narrowphase, so the MPR kernel carries none of EPA's private-memory
// polytope (2.2 KB of scratch per lane)
__device__ __forceinline__ int m_pair_order(const DModel* dm, int y) { return dm->pair_order[y]; }
template <int CCD>
__global__ __launch_bounds__(SOARM_COLLIDE_BLOCK, SOARM_COLLIDE_WAVES) void k_collide(const DModel* __restrict__ dm, int n,
                                                 const float* __restrict__ gpose,
                                                 float* __restrict__ cbuf, int* __restrict__ ccount,
                                                 uint32_t* __restrict__ pmask,
                                                 float* __restrict__ sepax,
                                                 unsigned long long* __restrict__ pcyc) {
  // (env chunks numbered per XCD as in k_geom / k_substep: the geom records this reads and the
  // contact buffer it writes stay in the L2 of the XCD whose substep waves own those envs)
  // native: LDS slots for the EPA polytopes of this workgroup's penetrating lanes (EpaPool)
  constexpr int NSLOT = CCD == SIM_CCD_NATIVE ? SOARM_EPA_SLOTS : 0;
  __shared__ EpaPoly s_epa[NSLOT > 0 ? NSLOT : 1];
  __shared__ int s_epa_used;
  if constexpr (NSLOT > 0) {
    if (threadIdx.x == 0) s_epa_used = 0;
    __syncthreads();
  }
  const EpaPool pool{s_epa, &s_epa_used, NSLOT};
  const int e = xcd_block() * blockDim.x + threadIdx.x;
  const int p = m_pair_order(dm, blockIdx.y);  // (DModel::pair_order: the heavy pairs dispatch first)
  if (e >= n) return;
#ifdef SOARM_DIAG_SKIPP
  if ((g_diag_skip[p >> 5] >> (p & 31)) & 1u) return;  // (diagnostic: the pairs SOARM_DIAG_SKIP names cost nothing)
#endif
  const long long t0 = pcyc ? clock64() : 0;
  const DModel& m = *dm;
  PairOut o{cbuf, n, e, m.pair_slot[p], m.pair_cap[p], 0};
#ifdef SOARM_DIAG_SKIPP
  if (g_diag_stage == 1) {
    GeomPose P1, P2;
    if (midphase(m, p, gpose, n, e, P1, P2)) soa(cbuf, 0, n, e) = P1.p[0] + P2.p[0];
    return;
  }
#endif
  collide_pair<CCD>(m, p, gpose, n, e, o, SepCache{sepax, n, e}, NSLOT > 0 ? &pool : nullptr);
#ifdef SOARM_DIAG_SKIPP
  if (g_diag_stage == 2) return;
#endif
  // (no per-pair count is stored: the pair mask bit and, for multi-contact pairs, its 2-bit
  // count word carry it -- an empty pair costs no store)
  (void)ccount;
  if (o.n > 0) {
    atomicOr(&pmask[(size_t)(p >> 5) * n + e], 1u << (p & 31));
    const int cq = m.pair_cq[p];
    if (cq >= 0) atomicOr(&pmask[(size_t)((m.npair + 31) >> 5) * n + e], (uint32_t)(o.n - 1) << (2 * cq));
  }
#ifdef SOARM_COLLIDE_STATS
  // diagnostic build: per pair, how many envs each test decided (13-bit counters: codes 0-3 in
  // the first word, 4-7 in the second; see PairOut::xc)
  if (pcyc) atomicAdd(&pcyc[(o.xc >> 2) * gridDim.y + p], 1ull << (13 * (o.xc & 3)));
#else
  if (pcyc && (threadIdx.x & 63) == 0) {
    const unsigned long long dt = (unsigned long long)(clock64() - t0);
    atomicAdd(&pcyc[p], dt);
    atomicMax(&pcyc[gridDim.y + p], dt);
  }
#endif
}

// the collide launch: (env, pair) lanes, SOARM_COLLIDE_BLOCK-env blocks x npair
static void launch_collide(const sim_batch* b, hipStream_t q, unsigned long long* pcyc) {
  auto kern = b->model->desc.ccd == SIM_CCD_NATIVE ? k_collide<SIM_CCD_NATIVE> : k_collide<SIM_CCD_MPR>;
  int rows = b->model->desc.npair;
#ifdef SOARM_DIAG_SKIPP
  // (diagnostic: SOARM_DIAG_ROWS=k launches only the first k rows of the dispatch order -- timings only)
  if (const char* v = getenv("SOARM_DIAG_ROWS")) rows = std::min(rows, std::max(1, atoi(v)));
#endif
  hipLaunchKernelGGL(kern, dim3((b->n + SOARM_COLLIDE_BLOCK - 1) / SOARM_COLLIDE_BLOCK, rows),
                     dim3(SOARM_COLLIDE_BLOCK), 0, q, b->d_model, b->n,
                     b->d_gpose, b->d_cbuf, b->d_ccount, b->d_pmask, b->d_sepax, pcyc);
}

// walk the pairs in order and append their contacts (deterministic indexing)
DEVI int gather_contacts(const DModel& m, int n, int e, const float* __restrict__ cbuf, const PairMask& pm,
                         const ConLds& C, int& status) {
  int ncon = 0;
  for (int p = 0; p < m.npair; p++) {
    const int c = (pm.w[p >> 5] >> (p & 31)) & 1u ? pm.count(m, p) : 0;
    const int s0 = m.pair_slot[p];
    for (int k = 0; k < c; k++) {
      if (ncon >= SIM_MAXCON) {
        status |= SIM_ST_CONOVERFLOW;
        break;
      }
      C.dist(ncon) = cbuf[((size_t)(s0 + k) * 7) * n + e];
#pragma unroll
      for (int f = 0; f < 3; f++) {
        C.pos(ncon, f) = cbuf[((size_t)(s0 + k) * 7 + 1 + f) * n + e];
        C.n(ncon, f) = cbuf[((size_t)(s0 + k) * 7 + 4 + f) * n + e];
      }
      C.set_pair(ncon, p);
      ncon++;
    }
  }
  return ncon;
}

// diagnostic: compacted contact list [N][SIM_MAXCON][8] (dist, pos, normal, pair) + count
__global__ __launch_bounds__(64) void k_gather(const DModel* __restrict__ dm, int n,
                                               const float* __restrict__ cbuf,
                                               const int* __restrict__ ccount, uint32_t* __restrict__ pmask,
                                               float* __restrict__ out, int* __restrict__ nout) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  PairMask pm;
  pm.load(pmask, *dm, n, e);  // the pairs with contacts (and multi-contact counts)
  for (int w = 0; w < pmask_words(*dm); w++) soa(pmask, w, n, e) = 0u;
  __shared__ float s_con[SIM_MAXCON * 8][64];
  const ConLds C{s_con, (int)threadIdx.x};
  int status = 0;
  const int nc = gather_contacts(*dm, n, e, cbuf, pm, C, status);
  for (int c = 0; c < nc; c++)
    for (int f = 0; f < 8; f++) out[((size_t)e * SIM_MAXCON + c) * 8 + f] = s_con[c * 8 + f][threadIdx.x];
  nout[e] = nc;
}

template <int NA, int NF>
__global__ __launch_bounds__(64) void k_reset(const DModel* __restrict__ dm, int n, sim_state st,
                                              const float* __restrict__ init_qpos,
                                              const float* __restrict__ init_qvel,
                                              const float* __restrict__ extra_qpos, uint32_t k0,
                                              uint32_t k1, long long env_offset,
                                              const uint8_t* __restrict__ mask,
                                              float* __restrict__ obs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) env_reset<NA, NF>(dm, n, e, st, init_qpos, init_qvel, extra_qpos, k0, k1, env_offset, mask, obs);
}

// Keyed uniform draws for the rollout's action / phase streams: out[e][j] = lo + width u, u from
// Philox4x32-10 keyed by `seed`, counter (gid, gid >> 32, counter, 1 + j / 4) — sim_reset's draws
// use the 4th word 0, so the streams never overlap.  Keyed by global env id, so a dataset is the
// same for any env chunking / GPU count.  Host mirror: workloads.keyed_uniform.
__global__ __launch_bounds__(64) void k_rand(int n, uint32_t k0, uint32_t k1, long long env_offset,
                                             uint32_t counter, int k, float lo, float width,
                                             float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) env_rand(e, k0, k1, env_offset, counter, k, lo, width, out);
}

// qfrc_bias at the current state (mj_comVel + mj_rne with flg_acc = 0, as left by mj_forward)
template <int NA, int NF>
__global__ __launch_bounds__(64) void k_bias(const DModel* __restrict__ dm, int n, sim_state st,
                                             float* __restrict__ bias, sim_params pp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) env_bias<NA, NF>(dm, n, e, st, bias, pp);
}

template <int NA, int NF>
__global__ __launch_bounds__(64) void k_observe(const DModel* __restrict__ dm, int n, sim_state st,
                                                float* __restrict__ obs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) env_observe<NA, NF>(dm, n, e, st, obs);
}

// DLS site IK (soarm_env.h env_ik)
template <int NA>
__global__ __launch_bounds__(64) void k_ik(const DModel* __restrict__ dm, int n,
                                           const float* __restrict__ target, const float* __restrict__ tq,
                                           float* __restrict__ q, int32_t* __restrict__ ok,
                                           int32_t* __restrict__ iters, sim_ik_opts o) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) env_ik<NA>(dm, n, e, target, tq, q, ok, iters, o);
}


// ------------------------------------------------------------- dispatch
// Supported topologies: arm chain of NA=6 hinges, NF in {0, 1} free bodies.
template <class F>
static void dispatch_nf(int nf, F&& f) {
  if (nf == 0)
    f(std::integral_constant<int, 0>{});
  else
    f(std::integral_constant<int, 1>{});
}

// solver of the compiled model: PGS (the north star's) or MuJoCo's default Newton
template <class F>
static void dispatch_sol(int sol, F&& f) {
  if (sol == SIM_SOL_NEWTON)
    f(std::integral_constant<int, SIM_SOL_NEWTON>{});
  else
    f(std::integral_constant<int, SIM_SOL_PGS>{});
}

static inline dim3 grid_for(int n) { return dim3((n + 63) / 64); }

// profiling: kind >= 0 records a start event for that kernel kind, -1 the matching stop
static void prof_mark(sim_batch* b, int kind, hipStream_t st) {
  if (!b->prof) return;
  if (b->ev_used == b->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    b->ev_pool.push_back(e);
  }
  if (kind >= 0) b->ev_marks.emplace_back(kind, b->ev_used);
  (void)hipEventRecord(b->ev_pool[b->ev_used++], st);
}

// ------------------------------------------------------------------ model
static int host_threads() {
  int n = 1;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    n = CPU_COUNT(&set);
  else
    n = (int)std::thread::hardware_concurrency();
  return std::min(16, std::max(1, n));
}

static float host_impedance(const double* si, double pos, double margin) {
  double dmin = std::fmin(std::fmax(si[0], 1e-4), 0.9999), dmax = std::fmin(std::fmax(si[1], 1e-4), 0.9999);
  if (dmin == dmax || si[2] <= 1e-15) return 0.5 * (dmin + dmax);
  double x = std::fabs((pos - margin) / si[2]);
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y = si[4] == 1 ? x
             : x <= si[3] ? std::pow(x, si[4]) / std::pow(si[3], si[4] - 1)
                          : 1 - std::pow(1 - x, si[4]) / std::pow(1 - si[3], si[4] - 1);
  return dmin + y * (dmax - dmin);
}
static void host_KB(const double* solref, const double* solimp, double timestep, float KB[2]) {
  double dmax = std::fmin(std::fmax(solimp[1], 1e-4), 0.9999);
  if (solref[0] > 0) {
    double tc = std::fmax(solref[0], 2 * timestep), dr = solref[1];
    KB[0] = (float)(1.0 / (dmax * dmax * tc * tc * dr * dr));
    KB[1] = (float)(2.0 / (dmax * tc));
  } else {
    KB[0] = (float)(-solref[0] / (dmax * dmax));
    KB[1] = (float)(-solref[1] / dmax);
  }
}
static void quat2mat_h(float R[9], const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  double n = std::sqrt(w * w + x * x + y * y + z * z);
  w /= n, x /= n, y /= n, z /= n;
  R[0] = 1 - 2 * (y * y + z * z), R[1] = 2 * (x * y - w * z), R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z), R[4] = 1 - 2 * (x * x + z * z), R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y), R[7] = 2 * (y * z + w * x), R[8] = 1 - 2 * (x * x + y * y);
}

static int validate_and_build(const sim_model_desc& d, sim_model* M) {
  // topology: world, welded base, serial hinge chain, then free bodies under the world
  if (d.nbody < 3 || d.nbody > SIM_MAXBODY) return fail(SIM_E_MODEL, "nbody out of range");
  if (d.body_parentid[1] != 0 || d.body_jntnum[1] != 0)
    return fail(SIM_E_MODEL, "body 1 must be a welded base under the world");
  int na = 0;
  int b = 2;
  for (; b < d.nbody; b++) {
    if (d.body_parentid[b] != b - 1) break;
    if (d.body_jntnum[b] != 1 || d.jnt_type[d.body_jntadr[b]] != SIM_JNT_HINGE)
      return fail(SIM_E_MODEL, "chain bodies must carry exactly one hinge");
    int j = d.body_jntadr[b];
    if (j != na || d.jnt_dofadr[j] != na || d.jnt_qposadr[j] != na)
      return fail(SIM_E_MODEL, "chain hinge addresses must equal their chain index");
    na++;
  }
  int nf = 0;
  for (; b < d.nbody; b++) {
    if (d.body_parentid[b] != 0 || d.body_jntnum[b] != 1 ||
        d.jnt_type[d.body_jntadr[b]] != SIM_JNT_FREE)
      return fail(SIM_E_MODEL, "bodies after the chain must be free bodies under the world");
    int j = d.body_jntadr[b];
    if (d.jnt_dofadr[j] != na + 6 * nf || d.jnt_qposadr[j] != na + 7 * nf)
      return fail(SIM_E_MODEL, "free joint addresses out of order");
    nf++;
  }
  if (na != 6 || nf > 1) return fail(SIM_E_MODEL, "kernels are compiled for a 6-hinge arm + <=1 free body");
  if (d.solver != SIM_SOL_PGS && d.solver != SIM_SOL_NEWTON)
    return fail(SIM_E_MODEL, "solver must be PGS or Newton");
  if (d.ccd != SIM_CCD_MPR && d.ccd != SIM_CCD_NATIVE) return fail(SIM_E_MODEL, "ccd must be MPR or native");
  if (d.nv != na + 6 * nf || d.nq != na + 7 * nf) return fail(SIM_E_MODEL, "nq/nv mismatch");
  if (d.nu > na) return fail(SIM_E_MODEL, "more actuators than arm hinges");
  for (int a = 0; a < d.nu; a++)
    if (d.actuator_trnid[a] != a) return fail(SIM_E_MODEL, "actuator a must drive joint a");
  for (int i = na; i < d.nv; i++)
    if (d.dof_frictionloss[i] > 0) return fail(SIM_E_MODEL, "frictionloss on free dofs unsupported");
  // one limit row per joint at a time (the kernels' LDS holds NA): both sides active at once needs
  // range width < 2 margin
  for (int j = 0; j < na; j++)
    if (d.jnt_limited[j] && d.jnt_range[j][1] - d.jnt_range[j][0] < 2.0 * d.jnt_margin[j])
      return fail(SIM_E_MODEL, "joint margin wider than half its range (both limit rows active) unsupported");
  if (d.nact > na || d.obs_nq > na) return fail(SIM_E_MODEL, "obs/act larger than the arm");
  for (int k = 0; k < d.obs_nq; k++)
    if (d.obs_qadr[k] >= na) return fail(SIM_E_MODEL, "observed joints must be arm hinges");
  for (int g = 0; g < d.ngeom; g++) {
    int t = d.geom_type[g];
    if (t != SIM_GEOM_PLANE && t != SIM_GEOM_BOX && t != SIM_GEOM_MESH)
      return fail(SIM_E_MODEL, "geom type unsupported by the kernels");
    if (d.geom_condim[g] != 3) return fail(SIM_E_MODEL, "only condim 3 contacts supported");
  }
  if (!d.disable_contact && d.ngeom > CON_MAXG) return fail(SIM_E_MODEL, "too many collidable geoms");
  M->na = na;
  M->nf = nf;

  DModel& m = M->dm;
  std::memset(&m, 0, sizeof(m));
  m.nq = d.nq, m.nv = d.nv, m.nu = d.nu, m.ngeom = d.ngeom, m.npair = d.npair, m.nact = d.nact;
  m.obs_site = d.obs_site, m.obs_nq = d.obs_nq;
  for (int k = 0; k < SIM_MAXOBSQ; k++) m.obs_qadr[k] = d.obs_qadr[k];
  m.iterations = d.iterations, m.disable_contact = d.disable_contact;
  m.ccd = d.ccd;
  bool anyd = false;
  for (int i = 0; i < d.nv; i++) anyd |= d.dof_damping[i] > 0;
  m.eulerdamp = (!d.disable_eulerdamp && anyd) ? 1 : 0;
  m.nhullvert = d.nhullvert;
  m.timestep = (float)d.timestep, m.impratio = (float)d.impratio;
  m.tolerance = (float)d.tolerance;
  m.pgs_scale = (float)(1.0 / ((d.meaninertia > 1e-15 ? d.meaninertia : 1.0) * std::max(1, d.nv)));
  for (int k = 0; k < 3; k++) m.gravity[k] = (float)d.gravity[k];
  for (int b2 = 0; b2 < d.nbody; b2++) {
    for (int k = 0; k < 3; k++) {
      m.body_pos[b2][k] = (float)d.body_pos[b2][k];
      m.body_ipos[b2][k] = (float)d.body_ipos[b2][k];
      m.body_inertia[b2][k] = (float)d.body_inertia[b2][k];
    }
    double qn = 0;
    for (int k = 0; k < 4; k++) qn += d.body_quat[b2][k] * d.body_quat[b2][k];
    for (int k = 0; k < 4; k++) m.body_quat[b2][k] = (float)(d.body_quat[b2][k] / std::sqrt(qn));
    quat2mat_h(m.body_imat[b2], d.body_iquat[b2]);
    m.body_mass[b2] = (float)d.body_mass[b2];
    m.body_invweight0[b2][0] = (float)d.body_invweight0[b2][0];
    m.body_invweight0[b2][1] = (float)d.body_invweight0[b2][1];
  }
  for (int j = 0; j < d.njnt; j++) {
    for (int k = 0; k < 3; k++) {
      m.jnt_pos[j][k] = (float)d.jnt_pos[j][k];
      m.jnt_axis[j][k] = (float)d.jnt_axis[j][k];
    }
    m.jnt_range[j][0] = (float)d.jnt_range[j][0], m.jnt_range[j][1] = (float)d.jnt_range[j][1];
    for (int k = 0; k < 5; k++) m.jnt_solimp[j][k] = (float)d.jnt_solimp[j][k];
    host_KB(d.jnt_solref[j], d.jnt_solimp[j], d.timestep, m.jnt_KB[j]);
    m.jnt_margin[j] = (float)d.jnt_margin[j];
    m.jnt_limited[j] = d.jnt_limited[j] && d.jnt_type[j] == SIM_JNT_HINGE;
  }
  for (int i = 0; i < d.nq; i++) m.qpos0[i] = (float)d.qpos0[i];
  for (int i = 0; i < d.nv; i++) {
    m.dof_armature[i] = (float)d.dof_armature[i];
    m.dof_damping[i] = (float)d.dof_damping[i];
    m.dof_frictionloss[i] = (float)d.dof_frictionloss[i];
    m.dof_invweight0[i] = (float)d.dof_invweight0[i];
    double imp = host_impedance(d.dof_solimp[i], 0.0, 0.0);
    m.dof_fricR[i] = (float)std::fmax(1e-15, (1 - imp) * d.dof_invweight0[i] / imp);
    float KB[2];
    host_KB(d.dof_solref[i], d.dof_solimp[i], d.timestep, KB);
    m.dof_fricB[i] = KB[1];
  }
  for (int g = 0; g < d.ngeom; g++) {
    m.geom_type[g] = d.geom_type[g], m.geom_bodyid[g] = d.geom_bodyid[g];
    m.geom_hulladr[g] = d.geom_hulladr[g], m.geom_hullnum[g] = d.geom_hullnum[g];
    for (int k = 0; k < 3; k++) {
      m.geom_pos[g][k] = (float)d.geom_pos[g][k];
      m.geom_size[g][k] = (float)d.geom_size[g][k];
      m.geom_center[g][k] = (float)d.geom_aabb[g][k];
      m.geom_half[g][k] = (float)d.geom_aabb[g][3 + k];
    }
    quat2mat_h(m.geom_mat[g], d.geom_quat[g]);
    for (int k = 0; k < 3; k++) {
      double c = d.geom_pos[g][k];
      for (int j = 0; j < 3; j++) c += (double)m.geom_mat[g][3 * k + j] * d.geom_aabb[g][j];
      m.geom_cbody[g][k] = (float)c;
    }
    m.geom_rbound[g] = (float)d.geom_rbound[g];
    m.geom_friction[g] = (float)d.geom_friction[g][0];
  }
  for (int p = 0; p < d.npair; p++) {
    int g1 = d.pair_geom1[p], g2 = d.pair_geom2[p];
    m.pair_geom1[p] = g1, m.pair_geom2[p] = g2;
    double sr[2], si[5];
    for (int k = 0; k < 2; k++) sr[k] = 0.5 * (d.geom_solref[g1][k] + d.geom_solref[g2][k]);
    for (int k = 0; k < 5; k++) {
      si[k] = 0.5 * (d.geom_solimp[g1][k] + d.geom_solimp[g2][k]);
      m.pair_solimp[p][k] = (float)si[k];
    }
    host_KB(sr, si, d.timestep, m.pair_KB[p]);
    m.pair_margin[p] = (float)std::fmax(d.geom_margin[g1], d.geom_margin[g2]);
    m.pair_tran[p] = (float)(d.body_invweight0[d.geom_bodyid[g1]][0] + d.body_invweight0[d.geom_bodyid[g2]][0]);
    m.pair_friction[p] = (float)std::fmax(d.geom_friction[g1][0], d.geom_friction[g2][0]);
    // slot capacity: box-box and plane-box can return up to 4 contacts, the rest 1
    const int t1 = d.geom_type[g1], t2 = d.geom_type[g2];
    const int cap = (t2 == SIM_GEOM_BOX && (t1 == SIM_GEOM_BOX || t1 == SIM_GEOM_PLANE)) ? 4 : 1;
    m.pair_slot[p] = m.nslot;
    m.pair_cap[p] = cap;
    m.pair_cq[p] = cap > 1 ? m.ncq++ : -1;
    m.pair_body1[p] = d.geom_bodyid[g1], m.pair_body2[p] = d.geom_bodyid[g2];
    m.nslot += cap;
  }
  if (m.ncq > 16) return fail(SIM_E_MODEL, "more than 16 box-box / plane-box pairs");
  for (int w = 0; w < (MAXP + 31) / 32; w++)
    m.pair_mw_multi[w] = m.pair_mw_arm[w] = m.pair_mw_free[w] = 0u, m.pair_cqbase[w] = 0;
  for (int p = 0, q = 0; p < d.npair; p++) {
    const int w = p >> 5;
    const uint32_t bit = 1u << (p & 31);
    if ((p & 31) == 0) m.pair_cqbase[w] = q;
    if (m.pair_cq[p] >= 0) m.pair_mw_multi[w] |= bit, q++;
    const int b1 = m.pair_body1[p], b2 = m.pair_body2[p];
    if ((b1 >= 2 && b1 < 2 + na) || (b2 >= 2 && b2 < 2 + na)) m.pair_mw_arm[w] |= bit;
    if (b1 >= 2 + na || b2 >= 2 + na) m.pair_mw_free[w] |= bit;
  }
  {  // collide dispatch order: by class (convex-convex and box-box with the free body or the world's
     // boxes, then the arm's own mesh pairs, then plane pairs), later pairs first within a class
     // (round 4's order): a class-0 pair dispatched among the last workgroups started after the
     // grid had filled and set the launch's tail
    auto cls = [&](int p) {
      const int t1 = d.geom_type[d.pair_geom1[p]], t2 = d.geom_type[d.pair_geom2[p]];
      if (t1 == SIM_GEOM_PLANE || t2 == SIM_GEOM_PLANE) return 2;
      const int b1 = d.geom_bodyid[d.pair_geom1[p]], b2 = d.geom_bodyid[d.pair_geom2[p]];
      return (b1 == 0 || b2 == 0 || b1 >= 2 + na || b2 >= 2 + na) ? 0 : 1;
    };
    int k = 0;
    for (int c = 0; c < 3; c++)
      for (int p = d.npair - 1; p >= 0; p--)
        if (cls(p) == c) m.pair_order[k++] = p;
  }
  // free bodies: the kernels use a diagonal 6x6 mass block, which needs the inertia frame at
  // the body frame (ipos = 0, iquat = identity) — true for the build-defined cube
  m.free_diag = 1;
  for (int b2 = 2 + na; b2 < d.nbody; b2++) {
    const double* ip = d.body_ipos[b2];
    const double* iq = d.body_iquat[b2];
    if (ip[0] != 0 || ip[1] != 0 || ip[2] != 0 || iq[0] != 1 || iq[1] != 0 || iq[2] != 0 || iq[3] != 0)
      return fail(SIM_E_MODEL, "free bodies need ipos = 0 and an inertia frame equal to the body frame");
  }
  for (int s = 0; s < d.nsite; s++) {
    m.site_bodyid[s] = d.site_bodyid[s];
    for (int k = 0; k < 3; k++) m.site_pos[s][k] = (float)d.site_pos[s][k];
    double qn = 0;
    for (int k = 0; k < 4; k++) qn += d.site_quat[s][k] * d.site_quat[s][k];
    for (int k = 0; k < 4; k++) m.site_quat[s][k] = (float)(qn > 0 ? d.site_quat[s][k] / std::sqrt(qn) : k == 0);
  }
  for (int a = 0; a < d.nu; a++) {
    m.act_ctrllimited[a] = d.actuator_ctrllimited[a];
    m.act_forcelimited[a] = d.actuator_forcelimited[a];
    m.act_gear[a] = (float)d.actuator_gear[a];
    m.act_gain[a] = (float)d.actuator_gainprm[a];
    for (int k = 0; k < 3; k++) m.act_bias[a][k] = (float)d.actuator_biasprm[a][k];
    for (int k = 0; k < 2; k++) {
      m.act_ctrlrange[a][k] = (float)d.actuator_ctrlrange[a][k];
      m.act_forcerange[a][k] = (float)d.actuator_forcerange[a][k];
    }
  }
  return SIM_OK;
}

static int upload_into(const sim_model* m, DevModel* D) {
  DModel dm = m->dm;
  auto up = [&](auto*& dst, const auto& src) -> int {
    using T = typename std::remove_reference<decltype(src)>::type::value_type;
    const size_t bytes = std::max<size_t>(src.size(), 1) * sizeof(T);
    HIPCHECK(hipMalloc(&dst, bytes));
    if (!src.empty()) HIPCHECK(hipMemcpy(dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return SIM_OK;
  };
  if (!m->hull_vert.empty()) {
    if (int rc = up(D->d_hv, m->hull_vert)) return rc;
    if (int rc = up(D->d_hadr, m->hull_adr)) return rc;
    if (int rc = up(D->d_hadj, m->hull_adj)) return rc;
  }
  if (int rc = up(D->d_hlut, m->hull_lut)) return rc;
  if (int rc = up(D->d_hrec, m->hull_rec)) return rc;
  if (int rc = up(D->d_hlutrec, m->hull_lutrec)) return rc;
  if (int rc = up(D->d_hovf, m->hull_ovf)) return rc;
  if (int rc = up(D->d_hsb, m->hull_sb)) return rc;
  dm.hull_vert = D->d_hv;
  dm.hull_adr = D->d_hadr;
  dm.hull_adj = D->d_hadj;
  dm.hull_lut = D->d_hlut;
  dm.hull_rec = D->d_hrec;
  dm.hull_lutrec = D->d_hlutrec;
  dm.hull_ovf = D->d_hovf;
  dm.hull_sb = D->d_hsb;
  for (int g = 0; g < MAXG; g++) {
    dm.geom_lutadr[g] = g < m->desc.ngeom ? m->lutadr[g] : -1;
    dm.geom_sbadr[g] = g < m->desc.ngeom ? m->sbadr[g] : -1;
  }
  HIPCHECK(hipMalloc(&D->d_model, sizeof(DModel)));
  HIPCHECK(hipMemcpy(D->d_model, &dm, sizeof(DModel), hipMemcpyHostToDevice));
  return SIM_OK;
}

// the model's device copy on `device`: made by the first batch there, reused after
static int upload_model(const sim_model* m, int device, DModel** out) {
  std::lock_guard<std::mutex> lk(m->mu);
  for (DevModel* d : m->dev)
    if (d->device == device) {
      *out = d->d_model;
      return SIM_OK;
    }
  DevModel* D = new DevModel();
  D->device = device;
  const int rc = upload_into(m, D);
  if (rc) {  // nothing half-uploaded stays cached
    D->release();
    delete D;
    return rc;
  }
  m->dev.push_back(D);
  *out = D->d_model;
  return SIM_OK;
}
// the (struct_size, abi_version) header every by-pointer struct carries (soarm_sim.h)
template <class T>
static int check_struct(const T* p, const char* what) {
  if (p->struct_size != (int32_t)sizeof(T) || p->abi_version != SIM_ABI_VERSION)
    return fail(SIM_E_ARG, std::string(what) + ": struct_size / abi_version do not match this library (built for abi " +
                               std::to_string(SIM_ABI_VERSION) + ", sizeof " + std::to_string(sizeof(T)) + ")");
  return SIM_OK;
}

// ============================================================== C ABI
extern "C" {

const char* sim_last_error(void) { return g_err.c_str(); }
const char* sim_version(void) { return "soarm_sim 0.2.0 gfx950 (abi 2)"; }


int sim_model_create(const sim_model_desc* desc, const float* hull_vert, const int32_t* hull_adr,
                     const int32_t* hull_adj, sim_model** out) {
  if (!desc || !out) return fail(SIM_E_ARG, "null argument");
  if (int rc = check_struct(desc, "sim_model_desc")) return rc;
  sim_model* M = new sim_model();
  M->desc = *desc;
  int rc = validate_and_build(*desc, M);
  if (rc) {
    delete M;
    return rc;
  }
  M->hull_vert.resize(desc->nhullvert);
  for (int i = 0; i < desc->nhullvert; i++)
    M->hull_vert[i] = make_float4(hull_vert[3 * i], hull_vert[3 * i + 1], hull_vert[3 * i + 2], 0.f);
  if (desc->nhullvert) {
    if (!hull_adr || !hull_adj) {
      delete M;
      return fail(SIM_E_ARG, "hull graph missing");
    }
    M->hull_adr.assign(hull_adr, hull_adr + desc->nhullvert + 1);
    M->hull_adj.assign(hull_adj, hull_adj + desc->nhulladj);
  }
  // vertex records carry their adjacency range (start << 8 | degree) in w
  for (int i = 0; i < desc->nhullvert; i++) {
    const int32_t a0 = M->hull_adr[i], deg = M->hull_adr[i + 1] - a0;
    if (a0 < 0 || a0 >= (1 << 24) || deg < 0 || deg > 255) {
      delete M;
      return fail(SIM_E_MODEL, "hull graph too large for packed vertex records");
    }
    const uint32_t bits = ((uint32_t)a0 << 8) | (uint32_t)deg;
    float wf;
    memcpy(&wf, &bits, sizeof(wf));
    M->hull_vert[i].w = wf;
  }
  // support start table: per mesh geom, the argmax vertex of each cube-map cell's centre direction
  int nmesh = 0;
  for (int g = 0; g < desc->ngeom; g++) nmesh += desc->geom_type[g] == SIM_GEOM_MESH;
  M->hull_lut.assign((size_t)std::max(nmesh, 1) * HULL_LUT_CELLS, 0);
  for (int g = 0, k = 0; g < desc->ngeom; g++) {
    M->lutadr[g] = -1;
    if (desc->geom_type[g] != SIM_GEOM_MESH) continue;
    if (desc->geom_hullnum[g] > 65535) {
      delete M;
      return fail(SIM_E_MODEL, "hull with more than 65535 vertices");
    }
    M->lutadr[g] = k * HULL_LUT_CELLS;
    const float* hv = hull_vert + 3 * (size_t)desc->geom_hulladr[g];
    const int nv = desc->geom_hullnum[g];
    uint16_t* out = &M->hull_lut[(size_t)k * HULL_LUT_CELLS];
    // exact argmax per cell (brute force), cells split over host threads
    auto cells = [hv, nv, out](int c0, int c1) {
      for (int c = c0; c < c1; c++) {
        double d[3];
        lut_dir(c, d);
        int best = 0;
        double bd = -1e300;
        for (int i = 0; i < nv; i++) {
          const double s = d[0] * hv[3 * i] + d[1] * hv[3 * i + 1] + d[2] * hv[3 * i + 2];
          if (s > bd) bd = s, best = i;
        }
        out[c] = (uint16_t)best;
      }
    };
    // pool sized to the CPUs this process may run on (the GPU box gives each job a share of
    // the machine), at most 16; if a thread cannot be started its cells run on this one
    const int nt = host_threads();
    std::vector<std::thread> pool;
    int started = 0;
    for (int t = 0; t < nt; t++) {
      const int c0 = (int)((long)HULL_LUT_CELLS * t / nt), c1 = (int)((long)HULL_LUT_CELLS * (t + 1) / nt);
      if (t + 1 < nt && started == t) {
        try {
          pool.emplace_back(cells, c0, c1);
          started++;
          continue;
        } catch (...) {
        }
      }
      cells(c0, c1);
    }
    for (auto& th : pool) th.join();
    k++;
  }
  // climbing records (HULL_LUTREC uint4 per vertex): coordinates and degree, the first 8 neighbour
  // ids, then those neighbours' coordinates and ids
  M->hull_rec.assign((size_t)HULL_LUTREC * std::max(desc->nhullvert, 1), make_uint4(0, 0, 0, 0));
  M->hull_ovf.assign(1, 0);
  for (int g = 0; g < desc->ngeom; g++) {
    if (desc->geom_type[g] != SIM_GEOM_MESH) continue;
    const int base = desc->geom_hulladr[g];
    for (int li = 0; li < desc->geom_hullnum[g]; li++) {
      const int i = base + li;
      const int32_t a0 = M->hull_adr[i], deg = M->hull_adr[i + 1] - a0;
      const size_t ovf = M->hull_ovf.size();
      for (int a = 8; a < deg; a++) M->hull_ovf.push_back((uint16_t)M->hull_adj[a0 + a]);
      if (ovf >= (1u << 24)) {
        delete M;
        return fail(SIM_E_MODEL, "hull adjacency overflow table too large");
      }
      uint32_t xb, yb, zb;
      memcpy(&xb, &hull_vert[3 * i], 4), memcpy(&yb, &hull_vert[3 * i + 1], 4), memcpy(&zb, &hull_vert[3 * i + 2], 4);
      M->hull_rec[HULL_LUTREC * i] = make_uint4(xb, yb, zb, (uint32_t)deg | (deg > 8 ? (uint32_t)ovf << 8 : 0u));
      uint32_t id[8];
      for (int a = 0; a < 8; a++) id[a] = a < deg ? (uint32_t)M->hull_adj[a0 + a] : (uint32_t)li;
      M->hull_rec[HULL_LUTREC * i + 1] =
          make_uint4(id[0] | id[1] << 16, id[2] | id[3] << 16, id[4] | id[5] << 16, id[6] | id[7] << 16);
    }
    for (int li = 0; li < desc->geom_hullnum[g]; li++)  // neighbour k in record order (padding = the vertex itself)
      for (int k = 0; k < 8; k++) {
        const uint4 ids = M->hull_rec[HULL_LUTREC * (base + li) + 1];
        const uint32_t w[4] = {ids.x, ids.y, ids.z, ids.w};
        const uint32_t u = (w[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        const uint4 r = M->hull_rec[HULL_LUTREC * (base + u)];
        M->hull_rec[HULL_LUTREC * (base + li) + 2 + k] = make_uint4(r.x, r.y, r.z, u);
      }
  }
  // support-bound table: exact support at every grid point, rounded up to the next float
  M->hull_sb.assign((size_t)std::max(nmesh, 1) * 6 * HULL_SB_FACE, 0.f);
  for (int g = 0, k = 0; g < desc->ngeom; g++) {
    M->sbadr[g] = -1;
    if (desc->geom_type[g] != SIM_GEOM_MESH) continue;
    M->sbadr[g] = k * 6 * HULL_SB_FACE;
    const float* hv = hull_vert + 3 * (size_t)desc->geom_hulladr[g];
    const int nv = desc->geom_hullnum[g];
    for (int f = 0; f < 6; f++)
      for (int i = 0; i <= HULL_SB_K; i++)
        for (int j = 0; j <= HULL_SB_K; j++) {
          const double u = -1.0 + 2.0 * i / HULL_SB_K, v = -1.0 + 2.0 * j / HULL_SB_K, sg = (f & 1) ? -1.0 : 1.0;
          double d[3];
          switch (f >> 1) {
            case 0: d[0] = sg, d[1] = u, d[2] = v; break;
            case 1: d[0] = u, d[1] = sg, d[2] = v; break;
            default: d[0] = u, d[1] = v, d[2] = sg; break;
          }
          double bd = -1e300;
          for (int a = 0; a < nv; a++)
            bd = std::fmax(bd, d[0] * hv[3 * a] + d[1] * hv[3 * a + 1] + d[2] * hv[3 * a + 2]);
          M->hull_sb[(size_t)M->sbadr[g] + f * HULL_SB_FACE + i * (HULL_SB_K + 1) + j] =
              std::nextafter((float)bd, 3.0e38f);
        }
    k++;
  }
  M->hull_lutrec.assign((size_t)HULL_LUTREC * M->hull_lut.size(), make_uint4(0, 0, 0, 0));
  for (int g = 0; g < desc->ngeom; g++) {
    if (M->lutadr[g] < 0) continue;
    const size_t base = (size_t)desc->geom_hulladr[g];
    for (int c = 0; c < HULL_LUT_CELLS; c++) {
      const size_t cell = (size_t)M->lutadr[g] + c;
      const size_t v = base + M->hull_lut[cell];
      for (int k = 0; k < HULL_LUTREC; k++)  // (a copy of its start vertex's record)
        M->hull_lutrec[HULL_LUTREC * cell + k] = M->hull_rec[HULL_LUTREC * v + k];
    }
  }
  cpu_qpos0_contacts(M);  // (the hull tables above are its input)
  *out = M;
  return SIM_OK;
}

// compiled-model files (soarm_sim.h): the desc and hull arrays as sim_model_create takes them
static const char kModelMagic[8] = {'S', 'O', 'A', 'R', 'M', 'M', 'D', 'L'};
static const uint32_t kModelVersion = 2;  // 2: desc carries (struct_size, abi_version)

int sim_model_save(const sim_model_desc* desc, const float* hull_vert, const int32_t* hull_adr,
                   const int32_t* hull_adj, const char* path) {
  if (!desc || !path) return fail(SIM_E_ARG, "null argument");
  if (int rc = check_struct(desc, "sim_model_desc")) return rc;
  if (desc->nhullvert < 0 || desc->nhulladj < 0) return fail(SIM_E_ARG, "bad hull sizes");
  if (desc->nhullvert > 0 && (!hull_vert || !hull_adr || !hull_adj)) return fail(SIM_E_ARG, "hull arrays missing");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(SIM_E_ARG, "cannot open model file for writing");
  const uint32_t hdr[2] = {kModelVersion, (uint32_t)sizeof(sim_model_desc)};
  bool ok = fwrite(kModelMagic, 1, 8, f) == 8 && fwrite(hdr, sizeof(uint32_t), 2, f) == 2 &&
            fwrite(desc, sizeof(sim_model_desc), 1, f) == 1;
  if (ok && desc->nhullvert > 0)
    ok = fwrite(hull_vert, sizeof(float), 3 * (size_t)desc->nhullvert, f) == 3 * (size_t)desc->nhullvert &&
         fwrite(hull_adr, sizeof(int32_t), (size_t)desc->nhullvert + 1, f) == (size_t)desc->nhullvert + 1 &&
         fwrite(hull_adj, sizeof(int32_t), (size_t)desc->nhulladj, f) == (size_t)desc->nhulladj;
  ok = (fclose(f) == 0) && ok;
  return ok ? SIM_OK : fail(SIM_E_ARG, "model file write failed");
}

int sim_model_load(const char* path, sim_model** out) {
  if (!path || !out) return fail(SIM_E_ARG, "null argument");
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return fail(SIM_E_ARG, "cannot open model file");
  char magic[8];
  uint32_t hdr[2];
  sim_model_desc d;
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, kModelMagic, 8) != 0 || fread(hdr, sizeof(uint32_t), 2, f) != 2) {
    fclose(f);
    return fail(SIM_E_ARG, "not a compiled SO-ARM101 model file");
  }
  if (hdr[0] != kModelVersion || hdr[1] != sizeof(sim_model_desc)) {
    fclose(f);
    return fail(SIM_E_ARG, "model file version / layout does not match this library");
  }
  if (fread(&d, sizeof(d), 1, f) != 1 || d.nhullvert < 0 || d.nhulladj < 0 || d.nhullvert > (1 << 24) ||
      d.nhulladj > (1 << 26)) {
    fclose(f);
    return fail(SIM_E_ARG, "model file truncated or corrupt");
  }
  std::vector<float> hv(3 * (size_t)d.nhullvert);
  std::vector<int32_t> ha(d.nhullvert > 0 ? (size_t)d.nhullvert + 1 : 0), hj((size_t)d.nhulladj);
  bool ok = true;
  if (d.nhullvert > 0)
    ok = fread(hv.data(), sizeof(float), hv.size(), f) == hv.size() &&
         fread(ha.data(), sizeof(int32_t), ha.size(), f) == ha.size() &&
         fread(hj.data(), sizeof(int32_t), hj.size(), f) == hj.size();
  char extra;
  ok = ok && fread(&extra, 1, 1, f) == 0;  // nothing after the arrays
  fclose(f);
  if (!ok) return fail(SIM_E_ARG, "model file truncated or corrupt");
  return sim_model_create(&d, d.nhullvert ? hv.data() : nullptr, d.nhullvert ? ha.data() : nullptr,
                          d.nhullvert ? hj.data() : nullptr, out);
}

void sim_model_free(sim_model* m) { delete m; }

int sim_batch_create(const sim_model* m, int n_envs, int device, sim_batch** out) {
  if (!m || !out || n_envs <= 0) return fail(SIM_E_ARG, "bad argument");
  if (device == -1) {  // the CPU backend: host buffers, synchronous calls
    sim_batch* B = new sim_batch();
    B->model = m;
    B->n = n_envs;
    B->device = -1;
    if (int rc = cpu_batch_create(m, n_envs, &B->cpu)) {
      delete B;
      return rc;
    }
    *out = B;
    return SIM_OK;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SIM_E_NODEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(SIM_E_ARG, "bad device ordinal");
  HIPCHECK(hipSetDevice(device));
  sim_batch* B = new sim_batch();
  B->model = m;
  B->n = n_envs;
  if (const char* ng = getenv("SOARM_NO_GRAPH")) B->use_graphs = ng[0] != '1';
  B->device = device;
  {  // the RS kernel holds one wave per SIMD (256 VGPRs + AGPRs): past 4 envs per SIMD its waves
     // run in a second round, where the quad kernel's 16-env waves still fit in one (r05: 8192
     // envs 5.2 M env-steps/s RS against 7.9 M quad)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess)
      B->rs_cap = cus * 4 * RS_EPW;
#ifdef SOARM_DIAG_SKIPP
  {  // SOARM_DIAG_SKIP: "p,p,..." pairs to skip; a leading '~' skips every pair but those
    static uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (const char* v = getenv("SOARM_DIAG_SKIP")) {
      const bool inv = *v == '~';
      for (const char* c = v + inv; *c;) {
        const int p = atoi(c);
        if (p >= 0 && p < 128) w[p >> 5] |= 1u << (p & 31);
        while (*c && *c != ',') c++;
        if (*c) c++;
      }
      if (inv)
        for (auto& x : w) x = ~x;
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag_skip), w, sizeof(w), 0, hipMemcpyHostToDevice);
    const int stage = getenv("SOARM_DIAG_STAGE") ? atoi(getenv("SOARM_DIAG_STAGE")) : 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag_stage), &stage, sizeof(stage), 0, hipMemcpyHostToDevice);
  }
#endif
  }
  if (int rc = upload_model(m, device, &B->d_model)) {
    delete B;
    return rc;
  }
  if (!m->desc.disable_contact) {
    const int nv = m->desc.nv;
    // contact rows, then two rows of Newton's zone history (zero: none)
    B->scratch_floats = ((size_t)4 * SIM_MAXCON * (2 * nv + 4) + 2) * n_envs;
    HIPCHECK(hipMalloc(&B->d_scratch, B->scratch_floats * sizeof(float)));
    HIPCHECK(hipMemset(B->d_scratch, 0, B->scratch_floats * sizeof(float)));
    HIPCHECK(hipMalloc(&B->d_gpose, (size_t)m->desc.nbody * BREC * n_envs * sizeof(float)));
    HIPCHECK(hipMalloc(&B->d_cbuf, (size_t)(m->dm.nslot > 0 ? m->dm.nslot : 1) * 7 * n_envs * sizeof(float)));
    HIPCHECK(hipMalloc(&B->d_ccount, (size_t)(m->desc.npair > 0 ? m->desc.npair : 1) * n_envs * sizeof(int)));
    const size_t nw = (size_t)std::max(pmask_words(m->dm), 1);
    HIPCHECK(hipMalloc(&B->d_pmask, nw * n_envs * sizeof(uint32_t)));
    HIPCHECK(hipMemset(B->d_pmask, 0, nw * n_envs * sizeof(uint32_t)));
    const size_t ns = (size_t)std::max(m->desc.npair, 1) * 3 * n_envs;
    HIPCHECK(hipMalloc(&B->d_sepax, ns * sizeof(float)));
    HIPCHECK(hipMemset(B->d_sepax, 0, ns * sizeof(float)));
  }
  *out = B;
  return SIM_OK;
}

void sim_batch_free(sim_batch* b) {
  if (!b) return;
  if (b->cpu) {
    cpu_batch_free(b->cpu);
    delete b;
    return;
  }
  (void)hipSetDevice(b->device);
#ifdef SOARM_DIAG_SUPPORT
  {  // (diagnostic build: the support-query counters of every collide so far)
    unsigned long long c[CON_MAXG][4];
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_diag_sup), sizeof(c), 0, hipMemcpyDeviceToHost);
    for (int g = 0; g < CON_MAXG; g++)
      if (c[g][0])
        fprintf(stderr, "support geom %d: queries %llu, same cell %llu, same answer %llu, climb trips %llu\n", g,
                c[g][0], c[g][1], c[g][2], c[g][3]);
  }
#endif
  (void)hipFree(b->d_scratch);
  (void)hipFree(b->d_gpose);
  (void)hipFree(b->d_cbuf);
  (void)hipFree(b->d_ccount);
  (void)hipFree(b->d_pmask);
  (void)hipFree(b->d_sepax);
  for (auto e : b->ev_pool) (void)hipEventDestroy(e);
  b->drop_graphs();
  if (b->cap_stream) (void)hipStreamDestroy(b->cap_stream);
  delete b;
}

int sim_batch_set_params(sim_batch* b, const sim_params* p) {
  if (!b) return fail(SIM_E_ARG, "null batch");
  b->params = p ? *p : sim_params{nullptr, nullptr, nullptr};
  b->drop_graphs();  // the parameters are bound into captured launches
  return SIM_OK;
}

static int check_state(const sim_batch* b, const sim_state* s) {
  if (!b || !s) return fail(SIM_E_ARG, "null argument");
  if (!s->qpos || !s->qvel || !s->qacc_warmstart || !s->ctrl || !s->status)
    return fail(SIM_E_ARG, "state buffers must all be set");
  return SIM_OK;
}

int sim_reset(sim_batch* b, const sim_state* s, const float* init_qpos, const float* init_qvel,
              const float* extra_qpos, uint64_t seed, int64_t env_offset, const uint8_t* mask,
              float* obs, void* stream) {
  const TraceRange tr_("sim_reset");
  if (int rc = check_state(b, s)) return rc;
  if (b->cpu) return cpu_reset(b->cpu, s, init_qpos, init_qvel, extra_qpos, seed, env_offset, mask, obs);
  hipStream_t st = (hipStream_t)stream;
  dispatch_nf(b->model->nf, [&](auto nfc) {
    constexpr int NA = 6, NF = decltype(nfc)::value;
    hipLaunchKernelGGL((k_reset<NA, NF>), grid_for(b->n), dim3(64), 0, st,
                                             b->d_model, b->n, *s, init_qpos, init_qvel, extra_qpos,
                                             (uint32_t)seed, (uint32_t)(seed >> 32), (long long)env_offset,
                                             mask, obs);
  });
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

// the row-space PGS substep (k_substep<..., RS>) for the scene with a free body, up to rs_cap envs
// (one round of waves); SOARM_RS=0 selects the quad kernel (16 envs per wave), read per env-step call
// (and part of the graph cache's key)
static bool rs_on() {
  const char* v = getenv("SOARM_RS");
  return !(v && v[0] == '0');
}

int sim_step(sim_batch* b, const sim_state* s, const float* action, int frame_skip, float* obs,
             void* stream) {
  const TraceRange tr_("sim_step");
  if (int rc = check_state(b, s)) return rc;
  if (frame_skip < 1) return fail(SIM_E_ARG, "frame_skip must be >= 1");
  if (b->cpu) return cpu_step(b->cpu, s, b->params, action, frame_skip, obs);
  hipStream_t st = (hipStream_t)stream;
  const bool con = !b->model->desc.disable_contact;
  const int sol = b->model->desc.solver;
  if (!con) {
    dispatch_nf(b->model->nf, [&](auto nfc) {
      dispatch_sol(sol, [&](auto solc) {
        constexpr int NA = 6, NF = decltype(nfc)::value, SOL = decltype(solc)::value;
        prof_mark(b, 0, st);
        if (s->qfrc_applied)
          hipLaunchKernelGGL((k_step<NA, NF, true, SOL>), grid_for(b->n), dim3(64), 0, st, b->d_model, b->n,
                             frame_skip, *s, action, obs, b->params);
        else
          hipLaunchKernelGGL((k_step<NA, NF, false, SOL>), grid_for(b->n), dim3(64), 0, st, b->d_model, b->n,
                             frame_skip, *s, action, obs, b->params);
        prof_mark(b, -1, st);
      });
    });
    HIPCHECK(hipGetLastError());
    return SIM_OK;
  }
  // contacts: geom poses, then per substep (env, pair)-parallel collide + per-env dynamics
  const int np = b->model->desc.npair;
  const bool rs = rs_on() && b->n <= b->rs_cap;
  auto enqueue = [&](hipStream_t q) {
    dispatch_nf(b->model->nf, [&](auto nfc) {
     dispatch_sol(sol, [&](auto solc) {
      constexpr int NA = 6, NF = decltype(nfc)::value, SOL = decltype(solc)::value;
      prof_mark(b, 3, q);
      {
        const TraceRange tr_("geom_poses");
        hipLaunchKernelGGL((k_geom<NA, NF>), geom_grid(b->n), dim3(64), 0, q, b->d_model, b->n, *s,
                           b->d_gpose);
      }
      prof_mark(b, -1, q);
      for (int sub = 0; sub < frame_skip; sub++) {
        if (np > 0) {
          prof_mark(b, 1, q);
          const TraceRange tr_("collide");
          launch_collide(b, q, nullptr);
          prof_mark(b, -1, q);
        }
        const bool last = sub == frame_skip - 1;
        const TraceRange tr_("substep");
        prof_mark(b, 2, q);
        auto kern = s->qfrc_applied ? k_substep<NA, NF, true, SOL> : k_substep<NA, NF, false, SOL>;
        int epb = 64 / lpe<NF>();  // envs per 64-thread workgroup
        if constexpr (NF == 1 && SOL == SIM_SOL_PGS) {
          if (rs) {
            kern = s->qfrc_applied ? k_substep<NA, NF, true, SOL, true> : k_substep<NA, NF, false, SOL, true>;
            epb = RS_EPW;
          }
        }
        size_t lds_pad = 0;
#ifdef SOARM_PHASE_PROF
        // (diagnostic build: SOARM_LDS_PAD bytes of unused dynamic LDS cap the workgroups per CU)
        if (const char* v = getenv("SOARM_LDS_PAD")) lds_pad = (size_t)atol(v);
        // (SOARM_DIAG_NOGPOSE: the substep writes no geom records -- timing only, wrong contacts)
        const bool nogpose = getenv("SOARM_DIAG_NOGPOSE") != nullptr;
        {  // (static: a captured graph's memcpy node reads this address at every replay)
          static int f11;
          f11 = getenv("SOARM_RS_FORCE11") != nullptr;
          (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_rs_force11), &f11, sizeof(f11), 0, hipMemcpyHostToDevice, q);
        }
#else
        constexpr bool nogpose = false;
#endif
        hipLaunchKernelGGL(kern, dim3((b->n + epb - 1) / epb), dim3(64), lds_pad, q,
                           b->d_model, b->n, *s,
                           sub == 0 ? action : nullptr, last ? obs : nullptr, b->params, b->d_scratch,
                           b->d_cbuf, np > 0 ? b->d_ccount : nullptr, np > 0 ? b->d_pmask : nullptr,
                           last || nogpose ? nullptr : b->d_gpose, b->d_gpose);
        prof_mark(b, -1, q);
      }
     });
    });
  };
  if (b->prof || !b->use_graphs || roctx().push) {  // profiling / tracing brackets every launch: no graph
    enqueue(st);
    HIPCHECK(hipGetLastError());
    return SIM_OK;
  }
  // replay a captured graph of the whole env-step (one launch instead of 1 + 2 x frame_skip)
  const sim_batch::GraphKey key{*s, action, obs, frame_skip, rs};
  hipGraphExec_t exec = nullptr;
  for (auto& g : b->graphs)
    if (g.first == key) exec = g.second;
  if (!exec) {
    if (!b->cap_stream) HIPCHECK(hipStreamCreateWithFlags(&b->cap_stream, hipStreamNonBlocking));
    HIPCHECK(hipStreamBeginCapture(b->cap_stream, hipStreamCaptureModeThreadLocal));
    enqueue(b->cap_stream);
    hipGraph_t graph = nullptr;
    HIPCHECK(hipStreamEndCapture(b->cap_stream, &graph));
    HIPCHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    (void)hipGraphDestroy(graph);
    if (b->graphs.size() >= 8) {  // small LRU-less cache: start over
      b->drop_graphs();
    }
    b->graphs.emplace_back(key, exec);
  }
  HIPCHECK(hipGraphLaunch(exec, st));
  return SIM_OK;
}

int sim_profile_begin(sim_batch* b) {
  if (!b) return fail(SIM_E_ARG, "null batch");
  if (b->cpu) return fail(SIM_E_ARG, "launch profiling needs a GPU batch");
  b->prof = true;
  b->ev_used = 0;
  b->ev_marks.clear();
  return SIM_OK;
}

int sim_profile_end(sim_batch* b, double* ms, int32_t* launches) {
  if (!b || !ms || !launches) return fail(SIM_E_ARG, "null argument");
  b->prof = false;
  for (int k = 0; k < SIM_PROF_KINDS; k++) ms[k] = 0, launches[k] = 0;
  for (auto& mk : b->ev_marks) {
    HIPCHECK(hipEventSynchronize(b->ev_pool[mk.second + 1]));
    float t = 0.f;
    HIPCHECK(hipEventElapsedTime(&t, b->ev_pool[mk.second], b->ev_pool[mk.second + 1]));
    ms[mk.first] += t;
    launches[mk.first] += 1;
  }
  b->ev_marks.clear();
  b->ev_used = 0;
  return SIM_OK;
}

int sim_contacts(sim_batch* b, const sim_state* s, float* out, int32_t* ncon, void* stream) {
  const TraceRange tr_("sim_contacts");
  if (int rc = check_state(b, s)) return rc;
  if (!out || !ncon) return fail(SIM_E_ARG, "null output");
  if (b->cpu) return cpu_contacts(b->cpu, s, out, ncon);
  if (b->model->desc.disable_contact) return fail(SIM_E_ARG, "model compiled with contacts disabled");
  hipStream_t st = (hipStream_t)stream;
  const int np = b->model->desc.npair;
  dispatch_nf(b->model->nf, [&](auto nfc) {
    constexpr int NA = 6, NF = decltype(nfc)::value;
    hipLaunchKernelGGL((k_geom<NA, NF>), geom_grid(b->n), dim3(64), 0, st, b->d_model, b->n, *s,
                       b->d_gpose);
  });
  if (np > 0)
    launch_collide(b, st, nullptr);
  hipLaunchKernelGGL(k_gather, grid_for(b->n), dim3(64), 0, st, b->d_model, b->n, b->d_cbuf, b->d_ccount, b->d_pmask,
                     out, ncon);
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_collide_profile(sim_batch* b, const sim_state* s, double* cycles, void* stream) {
  if (int rc = check_state(b, s)) return rc;
  if (!cycles) return fail(SIM_E_ARG, "null output");
  if (b->cpu) return fail(SIM_E_ARG, "collide profiling needs a GPU batch");
  if (b->model->desc.disable_contact) return fail(SIM_E_ARG, "model compiled with contacts disabled");
  hipStream_t st = (hipStream_t)stream;
  const int np = b->model->desc.npair;
  if (np <= 0) return SIM_OK;
  unsigned long long* d_cyc = nullptr;
  HIPCHECK(hipMalloc(&d_cyc, 2 * np * sizeof(unsigned long long)));
  HIPCHECK(hipMemsetAsync(d_cyc, 0, 2 * np * sizeof(unsigned long long), st));
  dispatch_nf(b->model->nf, [&](auto nfc) {
    constexpr int NA = 6, NF = decltype(nfc)::value;
    hipLaunchKernelGGL((k_geom<NA, NF>), geom_grid(b->n), dim3(64), 0, st, b->d_model, b->n, *s,
                       b->d_gpose);
  });
  launch_collide(b, st, d_cyc);
  HIPCHECK(hipMemsetAsync(b->d_pmask, 0, (size_t)pmask_words(b->model->dm) * b->n * sizeof(uint32_t), st));
  std::vector<unsigned long long> h(2 * np);
  HIPCHECK(hipMemcpyAsync(h.data(), d_cyc, 2 * np * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  HIPCHECK(hipFree(d_cyc));
  for (int p = 0; p < 2 * np; p++) cycles[p] = (double)h[p];
  return SIM_OK;
}

int sim_phase_profile(double* out, int reset) {
  if (!out) return fail(SIM_E_ARG, "null output");
#ifdef SOARM_PHASE_PROF
  unsigned long long nw[24];
  std::vector<unsigned long long> w((size_t)WPH_MAXW * WPH);
  HIPCHECK(hipDeviceSynchronize());
  HIPCHECK(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_wphase), w.size() * sizeof(w[0])));
  HIPCHECK(hipMemcpyFromSymbol(nw, HIP_SYMBOL(g_newton), sizeof(nw)));
  // per-wave rows (soarm_pgs.h g_wphase): maxima where g_phase's layout keeps a max, sums elsewhere
  const auto is_max = [](int k) {
    return k == 8 || k == 10 || k == 15 || (k >= 23 && k <= 26) || k == 59 || k == 60 || (k >= 65 && k <= 68) ||
           k == 83;
  };
  unsigned long long h[WPH] = {};
  for (int r = 0; r < WPH_MAXW; r++)
    for (int k = 0; k < WPH; k++) {
      const unsigned long long v = w[(size_t)r * WPH + k];
      h[k] = is_max(k) ? std::max(h[k], v) : h[k] + v;
    }
  for (int k = 0; k < 77; k++) out[k] = (double)h[k];
  for (int k = 0; k < 24; k++) out[77 + k] = (double)nw[k];
  // the RS solve's split, in the slots the Newton profiler leaves free in PGS builds
  out[77 + 8] = (double)h[77], out[77 + 9] = (double)h[78], out[77 + 10] = (double)h[79];
  out[77 + 11] = (double)h[80], out[77 + 16] = (double)h[81];
  out[77 + 17] = (double)h[82], out[77 + 18] = (double)h[83], out[77 + 19] = (double)h[84];  // RS fallback waves
  for (int k = 0; k < 7; k++) out[101 + k] = (double)h[85 + k];  // (callers pass >= 108 doubles)
  if (reset) {
    void* a = nullptr;
    HIPCHECK(hipGetSymbolAddress(&a, HIP_SYMBOL(g_wphase)));
    HIPCHECK(hipMemset(a, 0, w.size() * sizeof(w[0])));
    const unsigned long long z[24] = {};
    HIPCHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_newton), z, sizeof(nw)));
  }
  return SIM_OK;
#else
  (void)reset;
  for (int k = 0; k < 19; k++) out[k] = 0.0;
  return SIM_E_ARG;  // not a profiling build
#endif
}

int sim_rand_uniform(sim_batch* b, uint64_t seed, int64_t env_offset, uint32_t counter, int k, float lo,
                     float hi, float* out, void* stream) {
  const TraceRange tr_("sim_rand_uniform");
  if (!b || !out) return fail(SIM_E_ARG, "null argument");
  if (k < 1 || k > 64) return fail(SIM_E_ARG, "k must be in [1, 64]");
  if (b->cpu) return cpu_rand_uniform(b->cpu, seed, env_offset, counter, k, lo, hi, out);
  hipLaunchKernelGGL(k_rand, grid_for(b->n), dim3(64), 0, (hipStream_t)stream, b->n, (uint32_t)seed,
                     (uint32_t)(seed >> 32), (long long)env_offset, counter, k, lo, hi - lo, out);
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_substeps(sim_batch* b, const sim_state* s, int nsub, void* stream) {
  return sim_step(b, s, nullptr, nsub, nullptr, stream);
}

int sim_bias(sim_batch* b, const sim_state* s, float* qfrc_bias, void* stream) {
  const TraceRange tr_("sim_bias");
  if (int rc = check_state(b, s)) return rc;
  if (!qfrc_bias) return fail(SIM_E_ARG, "qfrc_bias is null");
  if (b->cpu) return cpu_bias(b->cpu, s, b->params, qfrc_bias);
  hipStream_t st = (hipStream_t)stream;
  dispatch_nf(b->model->nf, [&](auto nfc) {
    constexpr int NA = 6, NF = decltype(nfc)::value;
    hipLaunchKernelGGL((k_bias<NA, NF>), grid_for(b->n), dim3(64), 0, st, b->d_model, b->n, *s, qfrc_bias,
                       b->params);
  });
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_observe(sim_batch* b, const sim_state* s, float* obs, void* stream) {
  const TraceRange tr_("sim_observe");
  if (int rc = check_state(b, s)) return rc;
  if (!obs) return fail(SIM_E_ARG, "obs is null");
  if (b->cpu) return cpu_observe(b->cpu, s, obs);
  hipStream_t st = (hipStream_t)stream;
  dispatch_nf(b->model->nf, [&](auto nfc) {
    constexpr int NA = 6, NF = decltype(nfc)::value;
    hipLaunchKernelGGL((k_observe<NA, NF>), grid_for(b->n), dim3(64), 0, st,
                                             b->d_model, b->n, *s, obs);
  });
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_ik_dls_pose(sim_batch* b, const float* target, const float* target_quat, float* q, int32_t* ok,
                    int32_t* iters, const sim_ik_opts* opts, void* stream) {
  const TraceRange tr_("sim_ik_dls");
  if (opts)
    if (int rc = check_struct(opts, "sim_ik_opts")) return rc;
  if (!b || !target || !q || !opts) return fail(SIM_E_ARG, "null argument");
  if (opts->ndof < 1 || opts->ndof > 6 || opts->max_steps < 0) return fail(SIM_E_ARG, "bad ik options");
  if (b->cpu) return cpu_ik(b->cpu, target, target_quat, q, ok, iters, *opts);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL((k_ik<6>), grid_for(b->n), dim3(64), 0, st, b->d_model, b->n, target, target_quat, q, ok,
                     iters, *opts);
  HIPCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_ik_dls(sim_batch* b, const float* target, float* q, int32_t* ok, int32_t* iters,
               const sim_ik_opts* opts, void* stream) {
  return sim_ik_dls_pose(b, target, nullptr, q, ok, iters, opts, stream);
}

}  // extern "C"
