// Diagnostic microbenchmark: issue cost of VALU instruction patterns for one wave per
// SIMD (the k_substep regime).  Each kernel runs a fixed inline-asm sequence R times and
// reports cycles per instruction (clock64 around the loop, lane 0 of each wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/_mb/mb_chain tools/mb_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R 2000
#define FMA(x, a, b) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x) : "v"(a), "v"(b))
#define MULNEG(y, x, a) asm volatile("v_mul_f32_e64 %0, %1, -%2" : "=v"(y) : "v"(x), "v"(a))
#define MAX(y, x, a) asm volatile("v_max_f32 %0, %1, %2" : "=v"(y) : "v"(x), "v"(a))
#define DPP0(y, x) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf" : "=v"(y) : "v"(x))

template <int K>
__global__ __launch_bounds__(64) void k(float* out, long long* cyc, float a, float b) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 0, z = 0;
  float x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {x0, x1}, p1 = {x1, x2}, p2 = {x2, x3}, p3 = {x3, x0}, pa = {a, b}, pb = {b, a};
  f2 p4 = {x4, x1}, p5 = {x5, x2}, p6 = {x6, x3}, p7 = {x7, x0};
  int si = 0;
  const long long t0 = clock64();
  for (int r = 0; r < R; r++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if constexpr (K == 0) {  // 1 dependent chain: 16 fmac
        FMA(x0, a, b);
      } else if constexpr (K == 1) {  // 2 chains interleaved: 32 fmac
        FMA(x0, a, b);
        FMA(x1, a, b);
      } else if constexpr (K == 2) {  // 4 chains: 64 fmac
        FMA(x0, a, b);
        FMA(x1, a, b);
        FMA(x2, a, b);
        FMA(x3, a, b);
      } else if constexpr (K == 3) {  // dependent mul(neg) -> max -> fmac : 48 instrs
        MULNEG(y, x0, a);
        MAX(z, y, b);
        FMA(x0, z, a);
      } else if constexpr (K == 4) {  // dpp -> fmac dependent: 32 instrs
        DPP0(y, x0);
        FMA(y, a, b);
        x0 = y;
      } else if constexpr (K == 5) {  // 1 chain + 3 independent fills per link: 64 instrs
        FMA(x0, a, b);
        FMA(x1, a, b);
        FMA(x2, b, a);
        FMA(x3, a, a);
      } else if constexpr (K == 7) {  // 4 chains of v_pk_fma_f32 (2 fmas each)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p0) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p1) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p2) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p3) : "v"(pa), "v"(pb));
      } else if constexpr (K == 8) {  // 4 fmac chains + 4 salu
        FMA(x0, a, b);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(si));
        FMA(x1, a, b);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(si));
        FMA(x2, a, b);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(si));
        FMA(x3, a, b);
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(si));
      } else if constexpr (K == 9) {  // 8 independent chains
        FMA(x0, a, b);
        FMA(x1, a, b);
        FMA(x2, a, b);
        FMA(x3, a, b);
        FMA(x4, a, b);
        FMA(x5, a, b);
        FMA(x6, a, b);
        FMA(x7, a, b);
      } else if constexpr (K == 10) {  // dependent pk_fma chain
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p0) : "v"(pa), "v"(pb));
      } else if constexpr (K == 11) {  // 4 chains of v_pk_mul_f32
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p0) : "v"(pa));
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p1) : "v"(pa));
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p2) : "v"(pa));
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p3) : "v"(pa));
      } else if constexpr (K == 12) {  // 8 pk_fma chains
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p0) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p1) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p2) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p3) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p4) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p5) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p6) : "v"(pa), "v"(pb));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p7) : "v"(pa), "v"(pb));
      } else if constexpr (K == 13) {  // 8 independent accvgpr reads
        float t0, t1, t2, t3;
        asm volatile("v_accvgpr_read_b32 %0, a0" : "=v"(t0));
        asm volatile("v_accvgpr_read_b32 %0, a1" : "=v"(t1));
        asm volatile("v_accvgpr_read_b32 %0, a2" : "=v"(t2));
        asm volatile("v_accvgpr_read_b32 %0, a3" : "=v"(t3));
        asm volatile("v_accvgpr_read_b32 %0, a4" : "=v"(t0));
        asm volatile("v_accvgpr_read_b32 %0, a5" : "=v"(t1));
        asm volatile("v_accvgpr_read_b32 %0, a6" : "=v"(t2));
        asm volatile("v_accvgpr_read_b32 %0, a7" : "=v"(t3));
        x0 += t0 * 0.f;
      } else if constexpr (K == 14) {  // 8 independent dpp movs
        float t0, t1, t2, t3;
        DPP0(t0, x0); DPP0(t1, x1); DPP0(t2, x2); DPP0(t3, x3);
        DPP0(t0, x4); DPP0(t1, x5); DPP0(t2, x6); DPP0(t3, x7);
        asm volatile("" :: "v"(t0), "v"(t1), "v"(t2), "v"(t3));
      } else if constexpr (K == 15) {  // pk_fma -> scalar mul on .x -> max -> pk_fma(splat): 3 instrs
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p0) : "v"(pa), "v"(pb));
        float t = p0.x;
        MULNEG(y, t, a);
        MAX(z, y, b);
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(p0) : "v"(pa), "v"(f2{z, z}));
      } else if constexpr (K == 16) {  // same chain scalar: fma -> mul -> max -> fma
        FMA(x0, a, b);
        MULNEG(y, x0, a);
        MAX(z, y, b);
        FMA(x0, z, a);
      } else if constexpr (K == 6) {  // chain through an e64 fma with 3 vgpr sources
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x0) : "v"(a), "v"(b));
      }
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = x0 + x1 + x2 + x3 + y + z + x4 + x5 + x6 + x7 + p0.x + p1.y + p2.x + p3.y + p4.x + p5.x + p6.x + p7.x + si;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, int ninst, float* d, long long* c, int blocks) {
  hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, c, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks; i++) s += h[i];
  printf("%-28s blocks %4d  cycles/instr %.3f\n", name, blocks, s / blocks / ((double)R * 16 * ninst));
}

int main() {
  float* d;
  long long* c;
  hipMalloc(&d, 1024 * 64 * 4);
  hipMalloc(&c, 1024 * 8);
  for (int blocks : {256}) {
    run<0>("dep fmac chain", 1, d, c, blocks);
    run<1>("2 chains", 2, d, c, blocks);
    run<2>("4 chains", 4, d, c, blocks);
    run<3>("mul(neg)->max->fmac", 3, d, c, blocks);
    run<4>("dpp->fmac", 2, d, c, blocks);
    run<5>("chain + 3 fills", 4, d, c, blocks);
    run<6>("dep e64 fma", 1, d, c, blocks);
    run<7>("4 pk_fma chains", 4, d, c, blocks);
    run<8>("4 fmac chains + 4 salu", 8, d, c, blocks);
    run<9>("8 fmac chains", 8, d, c, blocks);
    run<10>("dep pk_fma chain", 1, d, c, blocks);
    run<11>("4 pk_mul chains", 4, d, c, blocks);
    run<12>("8 pk_fma chains", 8, d, c, blocks);
    run<13>("8 accvgpr reads (+1 valu)", 9, d, c, blocks);
    run<14>("8 dpp movs", 8, d, c, blocks);
    run<15>("pk->mul->max->pk chain", 4, d, c, blocks);
    run<16>("fma->mul->max->fma chain", 4, d, c, blocks);
  }
  return 0;
}
