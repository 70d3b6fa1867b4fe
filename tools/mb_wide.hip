// Diagnostic microbenchmark: cycles per row step of the wide PGS sweep (soarm_pgs.h
// wide_step) for one wave per SIMD (1024 waves of 64), against variants: quad_perm instead of
// row_newbcast, no broadcast, and the bare dependent chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/_mb/mb_wide tools/mb_wide.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <utility>

#define R 400
template <int Q, int K>
__device__ __forceinline__ float bc(float x) {
  if constexpr (K == 0 || K == 3) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x150 + Q, 0xF, 0xF, true));
  if constexpr (K == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), (Q & 3) * 0x55, 0xF, 0xF, true));
  return x;
}
template <int Q, int K>
__device__ __forceinline__ void step(const float (&C)[16], const float (&oh)[16], float& s, float& f) {
  float cand;
  asm("v_max_f32_e64 %0, %1, -%2" : "=v"(cand) : "v"(s), "v"(f));
  s = fmaf(C[Q], bc<Q, K>(cand), s);
  if constexpr (K != 3) f = fmaf(oh[Q], cand, f);
}
template <int K, int... Qs>
__device__ __forceinline__ void sweep(const float (&C)[16], const float (&oh)[16], float& s, float& f, std::integer_sequence<int, Qs...>) {
  (step<Qs, K>(C, oh, s, f), ...);
}
template <int K>
__global__ __launch_bounds__(64) void k(float* out, long long* cyc, const float* Cg) {
  const int r = threadIdx.x & 15;
  float C[16], oh[16];
#pragma unroll
  for (int q = 0; q < 16; q++) C[q] = Cg[r * 16 + q], oh[q] = q == r ? 1.f : 0.f;
  float s = 0.01f * r, f = 0.02f;
  const long long t0 = clock64();
  for (int i = 0; i < R; i++) sweep<K>(C, oh, s, f, std::make_integer_sequence<int, 16>{});
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = s + f;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const int nb = 1024;
  float *out, *C;
  long long* cyc;
  hipMalloc(&out, nb * 64 * 4);
  hipMalloc(&cyc, nb * 8);
  hipMalloc(&C, 256 * 4);
  float h[256];
  for (int i = 0; i < 256; i++) h[i] = (i % 17 == 0) ? -1.f : 1e-3f * ((i * 37) % 11 - 5);
  hipMemcpy(C, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[4] = {"wide step (row_newbcast)", "quad_perm bcast", "no bcast", "chain only (no f update)"};
  for (int K = 0; K < 4; K++) {
    for (int rep = 0; rep < 2; rep++) {
      if (K == 0) hipLaunchKernelGGL(k<0>, dim3(nb), dim3(64), 0, 0, out, cyc, C);
      if (K == 1) hipLaunchKernelGGL(k<1>, dim3(nb), dim3(64), 0, 0, out, cyc, C);
      if (K == 2) hipLaunchKernelGGL(k<2>, dim3(nb), dim3(64), 0, 0, out, cyc, C);
      if (K == 3) hipLaunchKernelGGL(k<3>, dim3(nb), dim3(64), 0, 0, out, cyc, C);
      hipDeviceSynchronize();
    }
    long long hc[1024];
    hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nb; i++) avg += hc[i];
    avg /= nb;
    printf("%-28s %.1f cycles per step (%.0f per 16-step sweep)\n", names[K], avg / (R * 16.0), avg / R);
  }
  return 0;
}
