// sim_internal.h — what the library's two translation units share: the model object behind
// the opaque `sim_model` handle, the error channel of sim_last_error(), and the CPU backend's
// entry points (soarm_cpu.hip, `device = -1` in sim_batch_create; SURVEY.md §8(b) "Threading").
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/soarm_sim.h"
#include "dmodel.h"

struct DevModel;  // one device's copy of the model (soarm_sim.hip)

struct sim_model {
  sim_model_desc desc;
  soarm::DModel dm;  // host copy; hull pointers filled per device upload (CPU backend: host vectors below)
  std::vector<float4> hull_vert;
  std::vector<int32_t> hull_adr, hull_adj;
  std::vector<uint16_t> hull_lut;
  std::vector<uint4> hull_rec, hull_lutrec;  // climbing records (dmodel.h)
  std::vector<uint16_t> hull_ovf;
  std::vector<float> hull_sb;  // support-bound table (dmodel.h HULL_SB_K)
  int lutadr[SIM_MAXGEOM], sbadr[SIM_MAXGEOM];
  int na = 0, nf = 0;
  mutable std::mutex mu;  // guards dev (batches may be created from several threads)
  mutable std::vector<DevModel*> dev;
  ~sim_model();
};

// sets the calling thread's sim_last_error() text; returns code
int soarm_set_error(int code, const std::string& msg);

// ---- CPU backend: the same per-env code as the kernels (soarm_step.h, soarm_collide.h,
// soarm_env.h) compiled for the host, envs split over threads; the constraint solve is a
// dense fp32 restatement of mj_solPGS / mj_solNewton over MuJoCo's row order.  All pointers
// are host memory; calls are synchronous.
struct CpuBatch;
int cpu_batch_create(const sim_model* m, int n, CpuBatch** out);
// the model's contacts at qpos0 (DModel c0_*: what a soft reset's mj_forward collides), at model creation
int cpu_qpos0_contacts(sim_model* m);
// test hook (not part of the C ABI): the kernels' hull support query (soarm_collide.h hull_support,
// compiled for the host) of mesh geom g along nd local directions dirs [nd][3] -> out [nd][3]
extern "C" int soarm_test_hull_support(const sim_model* m, int g, const float* dirs, int nd, float* out);
void cpu_batch_free(CpuBatch* c);
int cpu_reset(CpuBatch* c, const sim_state* s, const float* init_qpos, const float* init_qvel,
              const float* extra_qpos, uint64_t seed, int64_t env_offset, const uint8_t* mask, float* obs);
int cpu_step(CpuBatch* c, const sim_state* s, const sim_params& p, const float* action, int frame_skip,
             float* obs);
int cpu_bias(CpuBatch* c, const sim_state* s, const sim_params& p, float* qfrc_bias);
int cpu_observe(CpuBatch* c, const sim_state* s, float* obs);
int cpu_contacts(CpuBatch* c, const sim_state* s, float* out, int32_t* ncon);
int cpu_rand_uniform(CpuBatch* c, uint64_t seed, int64_t env_offset, uint32_t counter, int k, float lo, float hi,
                     float* out);
int cpu_ik(CpuBatch* c, const float* target, const float* target_quat, float* q, int32_t* ok, int32_t* iters,
           const sim_ik_opts& o);
