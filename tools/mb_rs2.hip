// Diagnostic microbenchmark: cycles per sweep of the RS kernel's row-space PGS (soarm_pgs.h rs_sweep),
// the sweep alone and inside the solve's stopping-test loop; one wave per SIMD (1024 waves).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/_mb/mb_rs2 tools/mb_rs2.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../lerobot-mujoco-sim2real_amd/csrc/soarm_pgs.h"
using namespace soarm;
#define R 100
template <int K, int NRB, bool DEC>
__global__ __launch_bounds__(64) void k(float* out, long long* cyc, float a, float tol) {
  const float l = (threadIdx.x & 15) * 1e-3f;
  f2 CA[NRB], CB[NRB];
  float NF[NRB], NH[6];
#pragma unroll
  for (int q = 0; q < NRB; q++) CA[q] = f2{-l * q * 0.01f, -l * 0.01f}, CB[q] = f2{-l * q * 0.02f, l * 0.01f}, NF[q] = -a * q;
#pragma unroll
  for (int q = 0; q < 6; q++) NH[q] = a * q;
  f2 sA = {l, 0}, sB = {-l, 0};
  bool done = false;
  const long long t0 = clock64();
  for (int it = 0; it < R; it++) {
    if constexpr (K == 0) {
      rs_sweep<6, NRB, DEC>(sA, sB, CA, CB, NF, NH);
    } else {
      if (!done) {
        const float s0A = sA.x, s0B = sB.x;
        sA.y = 0.f, sB.y = 0.f;
        rs_sweep<6, NRB, DEC>(sA, sB, CA, CB, NF, NH);
        float P = 0.5f * (sA.y - (sA.x - s0A)) * (s0A + sA.x);
        P = fmaf(0.7f * (sB.y - (sB.x - s0B)), s0B + sB.x, P);
        done = rowsum16(P) * 1e-3f < tol;
      }
      if (__all(done)) break;
    }
  }
  const long long t1 = clock64();
  float acc = sA.x + sA.y + sB.x + sB.y;
#pragma unroll
  for (int q = 0; q < NRB; q++) acc += NF[q];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int K, int NRB, bool DEC>
void run(const char* name, int nblk) {
  float* o;
  long long* c;
  (void)hipMalloc(&o, nblk * 64 * 4);
  (void)hipMalloc(&c, nblk * 8);
  for (int w = 0; w < 2; w++) hipLaunchKernelGGL((k<K, NRB, DEC>), dim3(nblk), dim3(64), 0, 0, o, c, 0.5f, -1.f);
  (void)hipDeviceSynchronize();
  long long* h = new long long[nblk];
  (void)hipMemcpy(h, c, nblk * 8, hipMemcpyDeviceToHost);
  double s = 0, mx = 0;
  for (int i = 0; i < nblk; i++) s += h[i], mx = h[i] > mx ? h[i] : mx;
  printf("%-36s waves %5d  cycles/sweep mean %7.1f max %7.1f\n", name, nblk, s / nblk / R, mx / R);
  (void)hipFree(o), (void)hipFree(c);
  delete[] h;
}
int main() {
  run<0, 22, true>("DEC 22 sweep only", 1024);
  run<1, 22, true>("DEC 22 sweep + stop loop", 1024);
  run<0, 22, false>("generic 22 sweep only", 1024);
  run<1, 22, false>("generic 22 sweep + stop loop", 1024);
  run<0, 26, false>("generic 26 sweep only", 1024);
  run<1, 26, false>("generic 26 sweep + stop loop", 1024);
  return 0;
}
