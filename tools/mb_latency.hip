// Microbenchmark (tools/mb_latency.hip): scalar-cache (K$) and LDS load-to-use latency on one wave,
// dependent chains; build: hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -o tools/_mb/klat tools/mb_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef const __attribute__((address_space(4))) int cint;
__global__ void k_smem(const int* p, int iters, long long* out, int* sink) {
  cint* q = (cint*)p;
  int x = 0;
  for (int i = 0; i < 64; i++) x = q[x];  // warm
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = q[x];
  long long t1 = clock64();
  if (threadIdx.x == 0) out[0] = t1 - t0, sink[0] = x;
}
__global__ void k_lds(const int* p, int iters, long long* out, int* sink) {
  __shared__ int s[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) s[i] = p[i];
  __syncthreads();
  int x = 0;
  for (int i = 0; i < 64; i++) x = s[x];
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = s[x];
  long long t1 = clock64();
  if (threadIdx.x == 0) out[0] = t1 - t0, sink[0] = x;
}
__global__ void k_valu(int iters, long long* out, float* sink) {
  float x = threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = fmaf(x, 1.0001f, 0.5f);
  long long t1 = clock64();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = x;
}
int main() {
  const int N = 1024;  // 4 KB ring, stride 16 ints (64 B lines)
  std::vector<int> h(N);
  for (int i = 0; i < N; i++) h[i] = (i + 16) % N;
  int *d, *sink; long long* out; float* fs;
  hipMalloc(&d, N * 4); hipMalloc(&sink, 4); hipMalloc(&out, 8); hipMalloc(&fs, 256 * 4);
  hipMemcpy(d, h.data(), N * 4, hipMemcpyHostToDevice);
  long long c;
  const int it = 4096;
  hipLaunchKernelGGL(k_smem, 1, 64, 0, 0, d, it, out, sink); hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
  printf("smem dependent load: %.1f clk/iter\n", (double)c / it);
  hipLaunchKernelGGL(k_lds, 1, 64, 0, 0, d, it, out, sink); hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
  printf("lds dependent load: %.1f clk/iter\n", (double)c / it);
  hipLaunchKernelGGL(k_valu, 1, 64, 0, 0, it, out, fs); hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
  printf("valu dependent fma: %.1f clk/iter\n", (double)c / it);
  return 0;
}
