// Diagnostic translation unit: the RS contact substep kernel alone (register / ISA inspection in
// seconds instead of the whole library's minutes):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -S --offload-device-only \
//         tools/rs_only.hip -o /tmp/rs.s -Rpass-analysis=kernel-resource-usage
#include "../lerobot-mujoco-sim2real_amd/csrc/soarm_substep.h"
namespace soarm {
template __global__ void k_substep<6, 1, false, SIM_SOL_PGS, true>(const DModel* __restrict__, int, sim_state,
                                                                    const float* __restrict__, float* __restrict__,
                                                                    sim_params, float* __restrict__,
                                                                    const float* __restrict__, const int* __restrict__,
                                                                    uint32_t* __restrict__, float* __restrict__,
                                                                    const float*);
}
