// Diagnostic microbenchmark: cycles per row step of row-space PGS sweep patterns (soarm_pgs.h
// rs_sweep), one wave per SIMD (1024 waves of 64 lanes, as the RS kernel at 4096 envs).
//   hipcc --offload-arch=gfx950 -O3 -o tools/_mb/mb_rs tools/mb_rs.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <utility>
typedef float f2 __attribute__((ext_vector_type(2)));
#define R 200
template <int Q>
__device__ __forceinline__ float maxb(float s, float nf) {
  float r;
  asm volatile("v_max_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(s), "v"(nf), "i"(Q));
  return r;
}
template <int Q>
__device__ __forceinline__ float movb(float s) {
  float r;
  asm volatile("v_mov_b32_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(s), "i"(Q));
  return r;
}
__device__ __forceinline__ f2 pkfma(f2 a, float d, f2 c) {
  f2 r;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(f2{d, 0.f}), "v"(c));
  return r;
}
__device__ __forceinline__ float fmac(float a, float d, float c) {
  asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(c) : "v"(a), "v"(d));
  return c;
}
__device__ __forceinline__ float vsub(float a, float b) {
  float r;
  asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <class F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) { (f(std::integral_constant<int, Is>{}), ...); }
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

template <int K>
__global__ __launch_bounds__(64) void k(float* out, long long* cyc, float a) {
  const float l = threadIdx.x * 1e-3f;
  f2 C[16], CB[16];
  float NF[16], NF2[16];
#pragma unroll
  for (int q = 0; q < 16; q++) C[q] = f2{l * q, -l}, CB[q] = f2{-l * q, l}, NF[q] = -a * q, NF2[q] = a * q;
  f2 sA = {l, 0}, sB = {-l, 0}, tA = {l * 2, 0}, tB = {l, 0};
  float xA = l, xB = -l;
  const long long t0 = clock64();
  for (int r = 0; r < R; r++) {
    sfor<16>([&](auto qc) {
      constexpr int Q = decltype(qc)::value;
      if constexpr (K == 0) {  // current: max_dpp, pk A, sub, pk B
        const float d = maxb<Q>(sA.x, NF[Q]);
        sA = pkfma(C[Q], d, sA);
        NF[Q] = vsub(NF[Q], d);
        sB = pkfma(CB[Q], d, sB);
      } else if constexpr (K == 1) {  // one slot: max_dpp, pk A, sub
        const float d = maxb<Q>(sA.x, NF[Q]);
        sA = pkfma(C[Q], d, sA);
        NF[Q] = vsub(NF[Q], d);
      } else if constexpr (K == 2) {  // unpacked: max_dpp, fmac, sub
        const float d = maxb<Q>(xA, NF[Q]);
        xA = fmac(C[Q].x, d, xA);
        NF[Q] = vsub(NF[Q], d);
      } else if constexpr (K == 3) {  // mov_dpp, max, fmac, sub
        const float d = vmax(movb<Q>(xA), NF[Q]);
        xA = fmac(C[Q].x, d, xA);
        NF[Q] = vsub(NF[Q], d);
      } else if constexpr (K == 4) {  // two independent envs interleaved (unpacked)
        const float d = maxb<Q>(xA, NF[Q]);
        const float e = maxb<Q>(xB, NF2[Q]);
        xA = fmac(C[Q].x, d, xA);
        xB = fmac(CB[Q].x, e, xB);
        NF[Q] = vsub(NF[Q], d);
        NF2[Q] = vsub(NF2[Q], e);
      } else if constexpr (K == 5) {  // chain only: max_dpp -> fmac
        const float d = maxb<Q>(xA, NF[Q]);
        xA = fmac(C[Q].x, d, xA);
      } else if constexpr (K == 6) {  // two envs, packed, 2 slots each
        const float d = maxb<Q>(sA.x, NF[Q]);
        const float e = maxb<Q>(tA.x, NF2[Q]);
        sA = pkfma(C[Q], d, sA);
        tA = pkfma(CB[Q], e, tA);
        NF[Q] = vsub(NF[Q], d);
        NF2[Q] = vsub(NF2[Q], e);
        sB = pkfma(CB[Q], d, sB);
        tB = pkfma(C[Q], e, tB);
      }
    });
  }
  const long long t1 = clock64();
  float acc = sA.x + sA.y + sB.x + sB.y + xA + xB + tA.x + tB.y;
#pragma unroll
  for (int q = 0; q < 16; q++) acc += NF[q] + NF2[q];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, int nblk) {
  float* o;
  long long* c;
  hipMalloc(&o, nblk * 64 * 4);
  hipMalloc(&c, nblk * 8);
  hipLaunchKernelGGL(k<K>, dim3(nblk), dim3(64), 0, 0, o, c, 0.5f);
  hipLaunchKernelGGL(k<K>, dim3(nblk), dim3(64), 0, 0, o, c, 0.5f);
  hipDeviceSynchronize();
  long long* h = new long long[nblk];
  hipMemcpy(h, c, nblk * 8, hipMemcpyDeviceToHost);
  double s = 0, mx = 0;
  for (int i = 0; i < nblk; i++) s += h[i], mx = h[i] > mx ? h[i] : mx;
  printf("%-40s waves %5d  cycles/step mean %6.2f max %6.2f\n", name, nblk, s / nblk / (R * 16.0), mx / (R * 16.0));
  hipFree(o), hipFree(c);
  delete[] h;
}
int main() {
  for (int nb : {1, 1024, 2048}) {
    run<0>("max_dpp, pk A, sub, pk B", nb);
    run<1>("max_dpp, pk A, sub", nb);
    run<2>("max_dpp, fmac, sub", nb);
    run<3>("mov_dpp, max, fmac, sub", nb);
    run<4>("2 envs: max_dpp x2, fmac x2, sub x2", nb);
    run<5>("chain: max_dpp, fmac", nb);
    run<6>("2 envs packed 2 slots", nb);
  }
  return 0;
}
