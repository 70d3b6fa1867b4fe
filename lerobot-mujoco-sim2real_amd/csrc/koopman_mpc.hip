// koopman_mpc.hip — batched Koopman-MPC (include/koopman_mpc.h) on float64 MFMA.
//
// Reference: control/MPC_Controler.py (MPCController: Psi_o :154-167, setup_mpc :65-98,
// setup_delta_mpc :100-141, get_control :143-152) and the tracking loop Koopman_MPC.py:197-222,
// one env, casadi/IPOPT, float64.  Here one wave serves 16 envs:
//
//   encoder  z = [x, MLP(x)]  (models/KoopmanBase.py:45-47): every Linear layer is a chain of
//            v_mfma_f64_16x16x4_f64 with the 16 envs on the MFMA's N side and the layer's output
//            rows in 16-row tiles.  The f64 MFMA's C/D layout (lane l, register r holds row
//            (l >> 4) + 4r, column l & 15) is exactly its B-operand layout for the k-step that
//            covers those 4 rows (B: lane l holds row k = l >> 4 of the step, column l & 15), so a
//            layer's output tile T register r IS the next layer's B operand for k-step 4T + r:
//            activations never leave registers, no LDS round trip, no shuffles.
//   control  u0 = ff + [Gz | Gu] [z0; u_prev] is one more 16-row MFMA tile over the same B
//            operands (z0's tiles, then u_prev), with ff as the accumulator's initial value.
//
// The weights of every layer are stored by the host in MFMA fragment order (tile, k-step, lane),
// so a workgroup stages them into LDS with linear 16-B copies and every A-operand read is a
// conflict-free, lane-contiguous ds_read_b64.  4096 envs = 256 waves = 64 workgroups of 4 waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/koopman_mpc.h"

int soarm_set_error(int code, const std::string& msg);  // soarm_sim.hip (sim_last_error)

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int KT = SIM_KMAXW / 16;  // 16-row tiles of a layer's output (4)

// device-side layout of one controller (kernel argument; offsets in doubles into the fragment blob)
struct KDev {
  int xd, ud, nl, nz, H, outw;
  int ntile[SIM_KMAXLAYER];  // 16-row output tiles of layer l
  int ks[SIM_KMAXLAYER];     // 4-deep k-steps of layer l (2 for layer 0: x padded to 8)
  int frag[SIM_KMAXLAYER];   // A fragments of layer l: [ntile][ks][64]
  int bias;                  // [nl][64]
  int gain;                  // [Gz | Gu] fragments: [ks_gain][64], rows = u (one tile)
  int ks_gain;               // 2 (x) + 4 * ntile[nl-1] (features) + 2 (u_prev)
  int total;                 // doubles staged in LDS by k_mpc_step / k_encode
  int gr_ks;                 // Gr fragments (feedforward): [gr_ks][64], K = H * nz
  double uclip;
};

#define DEVI __device__ __forceinline__

DEVI d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// stage `count` doubles global -> LDS (16-B copies; count is a multiple of 2, offsets 16-B aligned)
DEVI void stage(double* lds, const double* __restrict__ g, int count) {
  const double2* src = reinterpret_cast<const double2*>(g);
  double2* dst = reinterpret_cast<double2*>(lds);
  for (int i = threadIdx.x; i < count / 2; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// the encoder for this wave's 16 envs: xb = x as the B operand of k-steps 0..1 (lane: row
// 4s + (lane >> 4), env lane & 15); returns the last layer's output tiles in `act`.
// Shapes are static so every MFMA, LDS offset and register index is a compile-time constant:
// layer 0 is 4 tiles x 2 k-steps (x padded to 8 rows), hidden layers 4 tiles x 16 k-steps
// (widths zero-padded to 64), the last layer NTL tiles x 16 k-steps.
template <int NTL>
DEVI void encode(const KDev& K, const double* lds, int lane, const double xb[2], d4 (&act)[KT]) {
  const int kq = lane >> 4;
  d4 acc[KT];
  {  // layer 0 (ReLU: nl >= 2)
    const double* A = lds + K.frag[0] + lane;
    const double* bias = lds + K.bias;
#pragma unroll
    for (int T = 0; T < KT; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) acc[T][r] = bias[16 * T + kq + 4 * r];
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int T = 0; T < KT; T++) acc[T] = mfma(A[(T * 2 + s) * 64], xb[s], acc[T]);
#pragma unroll
    for (int T = 0; T < KT; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) act[T][r] = fmax(acc[T][r], 0.0);
  }
  for (int l = 1; l < K.nl - 1; l++) {  // hidden layers: one static body, runtime count
    const double* A = lds + K.frag[l] + lane;
    const double* bias = lds + K.bias + l * SIM_KMAXW;
#pragma unroll
    for (int T = 0; T < KT; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) acc[T][r] = bias[16 * T + kq + 4 * r];
    // k-steps outer, tiles inner: KT independent accumulator chains
#pragma unroll
    for (int s = 0; s < 4 * KT; s++)
#pragma unroll
      for (int T = 0; T < KT; T++) acc[T] = mfma(A[(T * 16 + s) * 64], act[s >> 2][s & 3], acc[T]);
#pragma unroll
    for (int T = 0; T < KT; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) act[T][r] = fmax(acc[T][r], 0.0);
  }
  {  // last layer: no ReLU (models/KoopmanBase.py:20-25)
    const double* A = lds + K.frag[K.nl - 1] + lane;
    const double* bias = lds + K.bias + (K.nl - 1) * SIM_KMAXW;
#pragma unroll
    for (int T = 0; T < NTL; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) acc[T][r] = bias[16 * T + kq + 4 * r];
#pragma unroll
    for (int s = 0; s < 4 * KT; s++)
#pragma unroll
      for (int T = 0; T < NTL; T++) acc[T] = mfma(A[(T * 16 + s) * 64], act[s >> 2][s & 3], acc[T]);
#pragma unroll
    for (int T = 0; T < KT; T++) act[T] = T < NTL ? acc[T] : d4{0, 0, 0, 0};
  }
}

// x rows of the wave's envs as B operands (f32 obs -> f64, as torch.DoubleTensor(obs))
DEVI void load_x(const KDev& K, const float* __restrict__ x, int e, bool live, int kq, double xb[2]) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const int row = 4 * s + kq;
    xb[s] = (live && row < K.xd) ? (double)x[(size_t)e * K.xd + row] : 0.0;
  }
}

// Psi_o for m states: z [nz][m]
template <int NTL>
__global__ __launch_bounds__(256) void k_encode(KDev K, const double* __restrict__ frag, int m,
                                                const float* __restrict__ x, double* __restrict__ z) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  stage(lds, frag, K.total);
  const int lane = threadIdx.x & 63, kq = lane >> 4;
  const int e = blockIdx.x * 64 + (threadIdx.x >> 6) * 16 + (lane & 15);
  const bool live = e < m;  // every lane runs the MFMAs (they need the full wave)
  double xb[2];
  load_x(K, x, e, live, kq, xb);
  d4 act[KT];
  encode<NTL>(K, lds, lane, xb, act);
  if (!live) return;
#pragma unroll
  for (int s = 0; s < 2; s++)
    if (4 * s + kq < K.xd) z[(size_t)(4 * s + kq) * m + e] = xb[s];
#pragma unroll
  for (int T = 0; T < NTL; T++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = 16 * T + kq + 4 * r;
      if (row < K.outw) z[(size_t)(K.xd + row) * m + e] = act[T][r];
    }
}

// u0 = ff + Gz z0 + Gu u_prev (z0 = Psi_o(x) unless given); u_prev <- u0; action = clip(u0)
template <int NTL>
__global__ __launch_bounds__(256) void k_mpc_step(KDev K, const double* __restrict__ frag, int n,
                                                  const float* __restrict__ x, const double* __restrict__ z0,
                                                  const double* __restrict__ ff, double* __restrict__ uprev,
                                                  float* __restrict__ action) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  stage(lds, frag, K.total);
  const int lane = threadIdx.x & 63, kq = lane >> 4;
  const int e = blockIdx.x * 64 + (threadIdx.x >> 6) * 16 + (lane & 15);
  const bool live = e < n;
  // issued before the encoder: consumed after it
  double up[2], f0[4];
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const int row = 4 * s + kq;
    up[s] = (live && row < K.ud) ? uprev[(size_t)row * n + e] : 0.0;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = kq + 4 * r;
    f0[r] = (live && ff && row < K.ud) ? ff[(size_t)row * n + e] : 0.0;
  }
  double xb[2];
  d4 act[KT];
  if (z0) {  // lifted state given (get_control(p), MPC_Controler.py:143)
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int row = 4 * s + kq;
      xb[s] = (live && row < K.xd) ? z0[(size_t)row * n + e] : 0.0;
    }
#pragma unroll
    for (int T = 0; T < KT; T++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * T + kq + 4 * r;
        act[T][r] = (live && T < NTL && row < K.outw) ? z0[(size_t)(K.xd + row) * n + e] : 0.0;
      }
  } else {
    load_x(K, x, e, live, kq, xb);
    encode<NTL>(K, lds, lane, xb, act);
  }
  // one output tile: rows = u index (kq + 4r), columns = envs; ff is the initial accumulator
  d4 u = {f0[0], f0[1], f0[2], f0[3]};
  const double* G = lds + K.gain + lane;
  u = mfma(G[0], xb[0], u);
  u = mfma(G[64], xb[1], u);
#pragma unroll
  for (int s = 0; s < 4 * NTL; s++) u = mfma(G[(2 + s) * 64], act[s >> 2][s & 3], u);
#pragma unroll
  for (int s = 0; s < 2; s++) u = mfma(G[(2 + 4 * NTL + s) * 64], up[s], u);
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = kq + 4 * r;
    if (row < K.ud) {
      uprev[(size_t)row * n + e] = u[r];
      action[(size_t)e * K.ud + row] = (float)fmin(fmax(u[r], -K.uclip), K.uclip);
    }
  }
}

// ff[f][u][e] = sum_{t<H} Gr_t zref[f+1+t][:][e]  (zero past nref); FR frames per workgroup.
// gr_ks is a multiple of 4 (zero fragments past K = H nz): 4 static accumulator chains.
constexpr int FR = 16;
__global__ __launch_bounds__(256) void k_feedforward(KDev K, const double* __restrict__ grfrag, int nframe,
                                                     int nref, int n, const double* __restrict__ zref,
                                                     double* __restrict__ ff) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  stage(lds, grfrag, K.gr_ks * 64);
  const int lane = threadIdx.x & 63, kq = lane >> 4;
  const int e = blockIdx.x * 64 + (threadIdx.x >> 6) * 16 + (lane & 15);
  const bool live = e < n;
  const int kk = K.H * K.nz;
  const int f1 = min(nframe, (int)(blockIdx.y + 1) * FR);
  for (int f = blockIdx.y * FR; f < f1; f++) {
    d4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    // this lane's reference element of k-step s: g = 4s + kq -> (t, j) = divmod(g, nz)
    int t = 0, j = kq;
    while (j >= K.nz) j -= K.nz, t++;
    for (int s0 = 0; s0 < K.gr_ks; s0 += 4) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int g = 4 * (s0 + q) + kq;
        const int fr = f + 1 + t;
        const double b = (live && g < kk && fr < nref) ? zref[((size_t)fr * K.nz + j) * n + e] : 0.0;
        acc[q] = mfma(lds[(s0 + q) * 64 + lane], b, acc[q]);
        j += 4;
        while (j >= K.nz) j -= K.nz, t++;
      }
    }
    if (live) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = kq + 4 * r;
        if (row < K.ud) ff[((size_t)f * K.ud + row) * n + e] = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
      }
    }
  }
}

// ---------------------------------------------------------------- DBKN (bilinear) first move
// The bilinear model's input matrix depends on the lifted state: B_total = B + sum_j z0_j Hhat_j
// (linearize_B, MPC_Controler.py:46-63), so the condensed QP (MPC_Controler.py:100-141, state_full:
// Q = q I, R = r I) differs per env and frame.  One wave per env, float64, everything in LDS:
//   M_0 = B_total, M_k = A M_{k-1}; X_k = M_k ('mpc') or C_k = sum_{i<=k} M_i ('delta_mpc')
//     (A staged in LDS once per workgroup);
//   rhs[s] = q sum_{t >= s} X_{t-s}' e_t, e_t = ref_t - A^{t+1} z0 - [delta] C_t u_prev;
//   G = Xs' Xs, the Gram of the stacked X_k (N = H nu columns, nz rows) on the f64 MFMA, in
//     registers until every X_k is read, then stored packed lower over X's storage;
//   Hess[s1][s2] = q sum_{t >= max(s1,s2)} X_{t-s1}' X_{t-s2} + r I -- along each block diagonal
//     a prefix sum of G's blocks: with the block order reversed, flip(s nu + c) = (H-1-s) nu + c,
//     Hess[flip a][flip b] = q sum_{b' <= b} G[b' + a - b][b'] (blocks a >= b), so the prefix sums
//     overwrite G in place (one lane per block diagonal and (c1, c2)) and leave
//     P = Pi Hess Pi' packed lower, Pi the block reversal;
//   P v' = Pi rhs by a Cholesky with the rows in registers, a forward solve and the first nu steps
//   of the back substitution (pivots by readlane): v_0 = v'_{(H-1) nu + c} comes first there;
//   u0 = v_0 + u_prev, action = clip(u0).
// Shapes: nz <= 64, nu <= 8, N = H nu <= 64.  Per env LDS: the X region (X [H][xs], later G
// and P) and the M region (M [nz*nu] and Zs [H+1][nz], later Y [N][H], then the Cholesky's column
// buffer; >= 256 doubles): 17.3 KB at nz 32, nu 5, H 10; up to 8 envs (waves) per workgroup, or as
// many as the LDS holds with A [nz][nz].
struct BDev {
  int nz, nu, H, N, delta, per_env;  // per_env: doubles of LDS per env
  int epw;                           // envs (waves) per workgroup
  int xreg;                          // doubles of the X / Gram / packed-Hessian region
  int xs;                            // X_k's stride (>= nz nu, = nu mod 32: the rhs phase's lanes
                                     // (X_{t-s} column c) then fall in distinct LDS banks)
  int mreg;                          // doubles of the M region (M, Zs; Y; the Cholesky's column buffer)
  double q, r, uclip;
};
// a double of lane l (l wave-uniform) in every lane: two v_readlane
DEVI double rdlane(double x, int l) {
  const long long b = __double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// LDS written by other lanes of this wave is read after this (the wave's LDS operations complete
// in order once issued; the fence keeps the compiler from moving them across)
DEVI void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// sum_j x[j * sx] y[j], j < len: four independent FMA chains (the loads of a step do not wait for
// the previous step's FMA)
DEVI double dotn(const double* x, int sx, const double* y, int len) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int j = 0;
#pragma unroll 2
  for (; j + 4 <= len; j += 4) {
    s0 = fma(x[j * sx], y[j], s0);
    s1 = fma(x[(j + 1) * sx], y[j + 1], s1);
    s2 = fma(x[(j + 2) * sx], y[j + 2], s2);
    s3 = fma(x[(j + 3) * sx], y[j + 3], s3);
  }
  for (; j < len; j++) s0 = fma(x[j * sx], y[j], s0);
  return (s0 + s1) + (s2 + s3);
}
#ifdef SOARM_BL_PROF
// diagnostic build: per phase of k_bilinear, summed wave cycles ([0..7]) and waves ([8])
__device__ unsigned long long g_bl[9];
#define BL_STAMP(k)                                                                  \
  {                                                                                  \
    const long long t_ = clock64();                                                  \
    if ((k) > 0 && lane == 0) atomicAdd(&g_bl[(k) - 1], (unsigned long long)(t_ - bl_t)); \
    if ((k) == 8 && lane == 0) atomicAdd(&g_bl[8], 1ull);                            \
    bl_t = t_;                                                                       \
  }
#else
#define BL_STAMP(k)
#endif
// HS / NUS / NZS: a static horizon, input count and lifted dimension (0: read from K) -- the
// reference's configuration (horizon 10, u_dim 5, nz = 8 + 24 = 32: N = 50) gets an instantiation in
// which every loop bound and guard on N, nu, H and nz is a constant (the Cholesky's and the solves'
// unrolled loops lose their per-column branches)
template <int EPW, int HS = 0, int NUS = 0, int NZS = 0>
__global__ __launch_bounds__(64 * EPW) void k_bilinear(BDev K, const double* __restrict__ A,
                                                          const double* __restrict__ Bm,
                                                          const double* __restrict__ Hh, int n,
                                                          const double* __restrict__ z0g,
                                                          const double* __restrict__ win,
                                                          double* __restrict__ uprev, float* __restrict__ action) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // XCD-aware chunking: workgroups are dealt round-robin over the 8 XCDs, so chunk the envs per
  // XCD (workgroup b runs chunk (b % 8) G/8 + b / 8): neighbouring envs -- which share the cache
  // lines of z0 and of the [H][nz][n] window -- land in the same L2
  const int nwg = gridDim.x;
  const int b = (nwg & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (nwg >> 3) + ((int)blockIdx.x >> 3);
  const int e = b * EPW + w;
#ifdef SOARM_BL_PROF
  long long bl_t = 0;
#endif
  const int nz = NZS ? NZS : K.nz, nu = NUS ? NUS : K.nu, H = HS ? HS : K.H, N = (HS && NUS) ? HS * NUS : K.N;
  const int zu = nz * nu, xs = K.xs;
  // A, shared by the workgroup's envs, rows padded to an odd stride (nz + 1 doubles): lanes reading
  // one element of different rows hit different banks (a 256-B stride puts them all on one)
  const int as = nz + 1;
  double* As = lds + (size_t)EPW * K.per_env;
  for (int i = threadIdx.x; i < nz * nz; i += blockDim.x) As[(i / nz) * as + (i % nz)] = A[i];
  __syncthreads();
  if (e >= n) return;  // (whole waves: no workgroup barrier below)
  BL_STAMP(0);
  double* X = lds + (size_t)w * K.per_env;  // [H][xs]; later G and P, packed lower (N (N + 1) / 2)
  double* M = X + K.xreg;                   // [zu]; later Y, then the Cholesky's column buffer
  double* Zs = M + zu;                      // [H + 1][nz]: A^t z0 (t = 0..H), later e_t over row t + 1
  for (int i = lane; i < nz; i += 64) Zs[i] = z0g[(size_t)i * n + e];
  double up[8];
#pragma unroll
  for (int c = 0; c < 8; c++) up[c] = c < nu ? uprev[(size_t)c * n + e] : 0.0;
  wsync();
  // B_total = B + sum_j z0_j Hhat_j  (Hhat [j][(i nu + c)]: a load instruction reads 64
  // consecutive doubles); for nz <= 32 all of an output's loads are issued before its FMAs (the
  // same four chains, in the same order, as dotn)
  for (int o = lane; o < zu; o += 64) {
    const double* hr = Hh + o;
    double d;
    if (nz <= 32) {
      double h[32];
#pragma unroll
      for (int j = 0; j < 32; j++) h[j] = hr[(size_t)min(j, nz - 1) * zu];
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
      for (int j = 0; j < 32; j += 4)
        if (j + 4 <= nz) {
          s0 = fma(h[j], Zs[j], s0);
          s1 = fma(h[j + 1], Zs[j + 1], s1);
          s2 = fma(h[j + 2], Zs[j + 2], s2);
          s3 = fma(h[j + 3], Zs[j + 3], s3);
        }
#pragma unroll
      for (int j = 0; j < 32; j++)
        if (j >= (nz & ~3) && j < nz) s0 = fma(h[j], Zs[j], s0);
      d = (s0 + s1) + (s2 + s3);
    } else {
      d = dotn(hr, zu, Zs, nz);
    }
    const double s = Bm[o] + d;
    M[o] = s, X[o] = s;
  }
  wsync();
  // the reference window of the first 16 frames (lane < nz; clamped addresses, no guarded loads),
  // issued after B_total's loads so that its latency overlaps the M_k phase (no global loads there:
  // the load counter is waited on in order)
  double wv[16];
  {
    const int li = min(lane, nz - 1);
#pragma unroll
    for (int t = 0; t < 16; t++) wv[t] = win[((size_t)min(t, H - 1) * nz + li) * n + e];
  }
  BL_STAMP(1);
  // M_k = A M_{k-1}; X_k = M_k or X_{k-1} + M_k, on the f64 MFMA: A's 16-row tiles (A fragment:
  // lane l holds A[16 t + (l & 15)][4 ks + (l >> 4)]) times M_{k-1} padded to 16 columns (B: lane l
  // holds M[4 ks + (l >> 4)][l & 15]); C: lane l, register r = row 16 t + (l >> 4) + 4 r, column l & 15.
  // Column nu of the B operand carries A^{k-1} z0, so the same products give the free response
  // A^k z0 (k = 1..H; the last round computes only that column).
  {
    const int NTz = (nz + 15) >> 4, KSz = (nz + 3) >> 2, fr = lane >> 4, fc = lane & 15;
    // A's fragments for nz <= 32 (2 row tiles x 8 k-steps) stay in registers across the H steps
    double af[2][8];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int ks = 0; ks < 8; ks++) {
        const int ar = 16 * t + fc, jr = 4 * ks + fr;
        af[t][ks] = (ar < nz && jr < nz) ? As[ar * as + jr] : 0.0;
      }
    const double* zc = Zs;  // A^{k-1} z0
    auto bop = [&](int jr) {  // B operand of row jr (lane column fc)
      return jr < nz ? (fc < nu ? M[jr * nu + fc] : (fc == nu ? zc[jr] : 0.0)) : 0.0;
    };
    for (int k = 1; k <= H; k++) {
      d4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; t++) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
      if (nz <= 32) {
        double bm[8];
#pragma unroll
        for (int ks = 0; ks < 8; ks++) bm[ks] = bop(4 * ks + fr);
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {
          acc[0] = mfma(af[0][ks], bm[ks], acc[0]);
          if (NTz > 1) acc[1] = mfma(af[1][ks], bm[ks], acc[1]);
        }
      } else {
        for (int ks = 0; ks < KSz; ks++) {
          const int jr = 4 * ks + fr;
          const double bm = bop(jr);
#pragma unroll
          for (int t = 0; t < 4; t++) {
            const int ar = 16 * t + fc;
            if (t < NTz) acc[t] = mfma((ar < nz && jr < nz) ? As[ar * as + jr] : 0.0, bm, acc[t]);
          }
        }
      }
      wsync();  // (every lane has read M_{k-1})
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 16 * t + fr + 4 * r, o = row * nu + fc;
          if (t < NTz && row < nz) {
            if (fc < nu && k < H) {
              M[o] = acc[t][r];
              X[k * xs + o] = K.delta ? X[(k - 1) * xs + o] + acc[t][r] : acc[t][r];
            } else if (fc == nu) {
              Zs[k * nz + row] = acc[t][r];
            }
          }
        }
      zc = Zs + k * nz;
      wsync();
    }
  }
  BL_STAMP(2);
  // e_t = ref_t - A^{t+1} z0 - [delta] C_t u_prev (lane i < nz), in place over row t + 1 of Zs
  if (lane < nz) {
#pragma unroll 2
    for (int t = 0; t < H; t++) {
      double wt = 0.0;
#pragma unroll
      for (int s2 = 0; s2 < 16; s2++) wt = s2 == t ? wv[s2] : wt;
      if (t >= 16) wt = win[((size_t)t * nz + lane) * n + e];
      double ev = wt - Zs[(t + 1) * nz + lane];
      if (K.delta) {
#pragma unroll
        for (int c = 0; c < 8; c++)
          if (c < nu) ev = fma(-X[t * xs + lane * nu + c], up[c], ev);
      }
      Zs[(t + 1) * nz + lane] = ev;
    }
  }
  wsync();
  // rhs in the reversed order (lane a holds entry flip(a) = s nu + c, s = H-1 - a / nu):
  // rhs[s] = q sum_{t >= s} X_{t-s}' e_t.  For H <= 16 from Y = Xs' E (the Gram's MFMA loop below,
  // N x H); otherwise here, one dot product per (lane, t).
  double rhs = 0.0;
  const int ls = H - 1 - lane / nu, lc = lane % nu;
  if (H > 16 && lane < N) {
    for (int t = ls; t < H; t++) rhs = fma(K.q, dotn(X + (t - ls) * xs + lc, nu, Zs + (t + 1) * nz, nz), rhs);
  }
  BL_STAMP(3);
  // Gram G[a][b] = sum_i X[i][a] X[i][b] over the N = H nu columns a = k nu + c of the stacked X_k
  // (rows i < nz), on the f64 MFMA: the A fragment of (tile t, k-step ks) -- lane l holds
  // X[4 ks + (l >> 4)][16 t + (l & 15)] -- is also the B fragment of (t, ks), so 4 fragment loads
  // per k-step feed the <= 10 lower tiles (ta >= tb); C: lane l, register r = row (l >> 4) + 4 r,
  // column l & 15 of the tile.  Stored packed lower (row >= col) over X, once every lane has read X.
  double* G = X;
  {
    const int NT = (N + 15) >> 4, KS = (nz + 3) >> 2;
    const bool yk = H <= 16;  // Y = Xs' E here (B operand: lane l holds e_{l & 15}[4 ks + (l >> 4)])
    d4 acc[10], yacc[4];
#pragma unroll
    for (int q = 0; q < 10; q++) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; q++) yacc[q] = d4{0.0, 0.0, 0.0, 0.0};
    const int fr = lane >> 4, fc = lane & 15;
    for (int ks = 0; ks < KS; ks++) {
      double fg[4];
      const int i = 4 * ks + fr;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int a = 16 * t + fc, k = a / nu;
        fg[t] = (t < NT && a < N && i < nz) ? X[k * xs + i * nu + (a - k * nu)] : 0.0;
      }
#pragma unroll
      for (int ta = 0, q = 0; ta < 4; ta++)
#pragma unroll
        for (int tb = 0; tb <= ta; tb++, q++)
          if (ta < NT) acc[q] = mfma(fg[ta], fg[tb], acc[q]);
      if (yk) {
        const double eo = (fc < H && i < nz) ? Zs[(fc + 1) * nz + i] : 0.0;
#pragma unroll
        for (int ta = 0; ta < 4; ta++)
          if (ta < NT) yacc[ta] = mfma(fg[ta], eo, yacc[ta]);
      }
    }
    wsync();
    if (yk) {  // Y [a][t] over M's storage (M and E are dead), then each lane's diagonal sum
      double* Y = M;
#pragma unroll
      for (int ta = 0; ta < 4; ta++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int a = 16 * ta + fr + 4 * r;
          if (ta < NT && a < N && fc < H) Y[a * H + fc] = yacc[ta][r];
        }
      wsync();
      if (lane < N)
        for (int t = ls; t < H; t++) rhs = fma(K.q, Y[((t - ls) * nu + lc) * H + t], rhs);
    }
#pragma unroll
    for (int ta = 0, q = 0; ta < 4; ta++)
#pragma unroll
      for (int tb = 0; tb <= ta; tb++, q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 16 * ta + fr + 4 * r, col = 16 * tb + fc;
          if (ta < NT && row < N && col <= row) G[row * (row + 1) / 2 + col] = acc[q][r];
        }
  }
  wsync();
  BL_STAMP(4);
  // P = Pi Hess Pi' in place over G: lane (d, c1, c2) walks its block diagonal's entries
  // (a1, a2) = ((b + d) nu + c1, b nu + c2), b = 0, 1, ... (a1 >= a2: d > 0, or c1 >= c2), keeps the
  // running sum S of G there and writes q S + r [d = 0, c1 = c2] back.  Every entry has one owner.
  double* P = G;
  for (int tr = lane; tr < H * nu * nu; tr += 64) {
    const int d = tr / (nu * nu), c1 = (tr / nu) % nu, c2 = tr % nu;
    if (d == 0 && c1 < c2) continue;  // (upper triangle of a diagonal block: not stored)
    const double rd = (d == 0 && c1 == c2) ? K.r : 0.0;
    double S = 0.0;
    for (int b = 0; b + d < H; b++) {
      const int a1 = (b + d) * nu + c1, a2 = b * nu + c2, o = a1 * (a1 + 1) / 2 + a2;
      S += G[o];
      P[o] = fma(K.q, S, rd);
    }
  }
  wsync();
  BL_STAMP(5);
  // Cholesky P = L L' with the rows in registers: lane i holds row i (compile-time column index,
  // N <= 64), in blocks of 4 columns.  Inside a block, column j is updated by the block's earlier
  // columns with L[j][q] taken by readlane (uniform), then scaled by its pivot; the trailing
  // columns k >= jb + 4 are updated once per block from the 4 columns put in LDS (M's storage),
  // read as same-address broadcasts.  Every row entry sees the same FMAs in the same column order
  // as the column-by-column right-looking form.  Pivots: 1/sqrt(d) from v_rsq_f64 and two Newton
  // steps, L[j][j] = d / sqrt(d) by that.  Lane l keeps 1 / L[l][l].  (The entries right of a
  // lane's diagonal take junk updates and are never read.)
  double row[64];
#pragma unroll
  for (int k = 0; k < 64; k++) row[k] = (lane < N && k <= lane) ? P[lane * (lane + 1) / 2 + k] : 0.0;
  double idg = 0.0;
  double* colb = M;  // [64][4] (>= 256 doubles: M is dead once X is complete)
#pragma unroll
  for (int jb = 0; jb < 64; jb += 4) {
    if (jb < N) {
      double l[4];
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const int j = jb + m;
        l[m] = 0.0;
        if (j < N) {
          double v = row[j];
#pragma unroll
          for (int q = 0; q < m; q++) v = fma(-l[q], rdlane(l[q], j), v);
          const double dj = rdlane(v, j);
          double y = __builtin_amdgcn_rsq(dj);
          y = fma(0.5 * y, fma(-(dj * y), y, 1.0), y);
          y = fma(0.5 * y, fma(-(dj * y), y, 1.0), y);
          l[m] = lane > j ? v * y : (lane == j ? dj * y : 0.0);
          row[j] = l[m];
          if (lane == j) idg = y;
        }
      }
      if (jb + 4 < N) {
        *(d2*)(colb + 4 * lane) = d2{l[0], l[1]};
        *(d2*)(colb + 4 * lane + 2) = d2{l[2], l[3]};
        wsync();
#pragma unroll
        for (int k = jb + 4; k < 64; k++)
          if (k < N) {
            const d2 c01 = *(const d2*)(colb + 4 * k), c23 = *(const d2*)(colb + 4 * k + 2);
            double v = fma(-l[0], c01[0], row[k]);
            v = fma(-l[1], c01[1], v);
            v = fma(-l[2], c23[0], v);
            row[k] = fma(-l[3], c23[1], v);
          }
        wsync();
      }
    }
  }
  BL_STAMP(6);
  // L y = rhs from the register rows; then L' v' = y, of which only v'_a, a >= N - nu, is wanted
  // (u0's entries, in the reversed order): those are the back substitution's first nu steps, so
  // only rows a >= N - nu of L go back to LDS (lane i reads row j's entry i, contiguous over the
  // lanes).  Pivot values by readlane.
  double y = rhs;
#pragma unroll
  for (int j = 0; j < 64; j++) {
    if (j < N) {
      const double yj = rdlane(y, j) * rdlane(idg, j);
      if (lane == j) y = yj;
      if (lane > j && lane < N) y = fma(-row[j], yj, y);
    }
  }
  const int a0 = N - nu;
#pragma unroll
  for (int k = 0; k < 64; k++)
    if (lane < N && k <= lane && k >= a0) P[lane * (lane + 1) / 2 + k] = row[k];
  wsync();
  for (int j = N - 1; j >= a0; j--) {
    const double vj = rdlane(y, j) * rdlane(idg, j);
    if (lane == j) y = vj;
    if (lane >= a0 && lane < j) y = fma(-P[j * (j + 1) / 2 + lane], vj, y);
  }
  BL_STAMP(7);
  const int c0 = lane - a0;  // v_0's entry c sits in lane flip(c) = (H-1) nu + c
  if (c0 >= 0 && c0 < nu) {  // u0 = v_0 + u_prev (get_control, MPC_Controler.py:147-149)
    double upl = 0.0;
#pragma unroll
    for (int c = 0; c < 8; c++) upl = c0 == c ? up[c] : upl;
    const double u0 = y + upl;
    uprev[(size_t)c0 * n + e] = u0;
    action[(size_t)e * nu + c0] = (float)fmin(fmax(u0, -K.uclip), K.uclip);
  }
  BL_STAMP(8);
}

typedef void (*EncodeFn)(KDev, const double*, int, const float*, double*);
typedef void (*StepFn)(KDev, const double*, int, const float*, const double*, const double*, double*, float*);
const EncodeFn ENCODE[4] = {k_encode<1>, k_encode<2>, k_encode<3>, k_encode<4>};
const StepFn STEP[4] = {k_mpc_step<1>, k_mpc_step<2>, k_mpc_step<3>, k_mpc_step<4>};

}  // namespace

struct sim_koopman {
  int device = 0;
  sim_koopman_desc desc;
  KDev kd;
  double* d_frag = nullptr;    // encoder + [Gz | Gu] fragments, biases
  double* d_grfrag = nullptr;  // Gr fragments
  // DBKN (sim_koopman_set_bilinear): A [nz][nz], B [nz][nu], Hhat [j][(i nu + c)]
  BDev bd{};
  double *d_A = nullptr, *d_B = nullptr, *d_Hh = nullptr;
};

#define KCHECK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return soarm_set_error(SIM_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

extern "C" {

#ifdef SOARM_BL_PROF
// diagnostic build only: the k_bilinear phase cycles (9 values), reset after reading
int sim_koopman_bl_profile(double* out) {
  unsigned long long h[9];
  KCHECK(hipDeviceSynchronize());
  KCHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bl), sizeof(h)));
  for (int k = 0; k < 9; k++) out[k] = (double)h[k];
  const unsigned long long z[9] = {};
  KCHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_bl), z, sizeof(z)));
  return 0;
}
#endif

int sim_koopman_create(const sim_koopman_desc* d, const double* weights, const double* gain, int device,
                       sim_koopman** out) {
  if (!d || !weights || !gain || !out) return soarm_set_error(SIM_E_ARG, "null argument");
  *out = nullptr;
  const int xd = d->x_dim, ud = d->u_dim, nl = d->nlayer, H = d->horizon;
  if (xd < 1 || xd > SIM_KMAXX) return soarm_set_error(SIM_E_MODEL, "x_dim must be in 1..8");
  if (ud < 1 || ud > SIM_KMAXU) return soarm_set_error(SIM_E_MODEL, "u_dim must be in 1..8");
  if (nl < 2 || nl > SIM_KMAXLAYER) return soarm_set_error(SIM_E_MODEL, "nlayer must be in 2..6");
  if (H < 1 || H > SIM_KMAXH) return soarm_set_error(SIM_E_MODEL, "horizon must be in 1..32");
  if (d->width[0] != xd) return soarm_set_error(SIM_E_MODEL, "width[0] must equal x_dim");
  for (int l = 1; l <= nl; l++)
    if (d->width[l] < 1 || d->width[l] > SIM_KMAXW) return soarm_set_error(SIM_E_MODEL, "encoder widths must be in 1..64");
  KDev K{};
  K.xd = xd, K.ud = ud, K.nl = nl, K.H = H, K.outw = d->width[nl], K.nz = xd + d->width[nl];
  K.uclip = d->u_clip;
  if (K.H * K.nz > 1024) return soarm_set_error(SIM_E_MODEL, "horizon * nz must be <= 1024");
  // static kernel shapes: layer 0 = 4 tiles x 2 k-steps, hidden = 4 x 16, last = ntl x 16
  int off = 0;
  for (int l = 0; l < nl; l++) {
    K.ntile[l] = l == nl - 1 ? (d->width[l + 1] + 15) / 16 : 4;
    K.ks[l] = l == 0 ? 2 : 16;
    K.frag[l] = off;
    off += K.ntile[l] * K.ks[l] * 64;
  }
  K.bias = off;
  off += nl * SIM_KMAXW;
  K.gain = off;
  K.ks_gain = 2 + 4 * K.ntile[nl - 1] + 2;
  off += K.ks_gain * 64;
  K.total = off;
  K.gr_ks = 4 * ((K.H * K.nz + 15) / 16);  // a multiple of 4 k-steps (zero fragments past H nz)
  if ((size_t)K.total * 8 > 160 * 1024 || (size_t)K.gr_ks * 64 * 8 > 160 * 1024)
    return soarm_set_error(SIM_E_MODEL, "controller does not fit in LDS");

  // host packing: fragment order, zero padding
  std::vector<double> blob(K.total, 0.0), gr((size_t)K.gr_ks * 64, 0.0);
  const double* w = weights;
  for (int l = 0; l < nl; l++) {
    const int in = d->width[l], ou = d->width[l + 1];
    for (int T = 0; T < K.ntile[l]; T++)
      for (int s = 0; s < K.ks[l]; s++)
        for (int lane = 0; lane < 64; lane++) {
          const int row = 16 * T + (lane & 15), col = 4 * s + (lane >> 4);
          blob[K.frag[l] + (T * K.ks[l] + s) * 64 + lane] = (row < ou && col < in) ? w[(size_t)row * in + col] : 0.0;
        }
    w += (size_t)ou * in;
    for (int r = 0; r < ou; r++) blob[K.bias + l * SIM_KMAXW + r] = w[r];
    w += ou;
  }
  // gain columns: [Gr (H*nz) | Gz (nz) | Gu (ud)]; B-operand order of the step kernel:
  // x rows 0..7 (k-steps 0,1), feature rows (4 per k-step), u_prev rows 0..7
  const int gcols = K.H * K.nz + K.nz + ud;
  auto gz_col = [&](int kk) -> int {  // padded k index -> gain column (or -1)
    if (kk < 8) return kk < xd ? K.H * K.nz + kk : -1;
    kk -= 8;
    const int nfr = 16 * K.ntile[nl - 1];
    if (kk < nfr) return kk < K.outw ? K.H * K.nz + xd + kk : -1;
    kk -= nfr;
    return kk < ud ? K.H * K.nz + K.nz + kk : -1;
  };
  for (int s = 0; s < K.ks_gain; s++)
    for (int lane = 0; lane < 64; lane++) {
      const int row = lane & 15, c = gz_col(4 * s + (lane >> 4));
      blob[K.gain + s * 64 + lane] = (row < ud && c >= 0) ? gain[(size_t)row * gcols + c] : 0.0;
    }
  for (int s = 0; s < K.gr_ks; s++)
    for (int lane = 0; lane < 64; lane++) {
      const int row = lane & 15, c = 4 * s + (lane >> 4);
      gr[s * 64 + lane] = (row < ud && c < K.H * K.nz) ? gain[(size_t)row * gcols + c] : 0.0;
    }

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return soarm_set_error(SIM_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return soarm_set_error(SIM_E_ARG, "bad device ordinal");
  KCHECK(hipSetDevice(device));
  sim_koopman* k = new sim_koopman;
  k->device = device, k->desc = *d, k->kd = K;
  if (hipMalloc(&k->d_frag, blob.size() * sizeof(double)) != hipSuccess ||
      hipMalloc(&k->d_grfrag, gr.size() * sizeof(double)) != hipSuccess) {
    sim_koopman_free(k);
    return soarm_set_error(SIM_E_HIP, "hipMalloc failed");
  }
  KCHECK(hipMemcpy(k->d_frag, blob.data(), blob.size() * sizeof(double), hipMemcpyHostToDevice));
  KCHECK(hipMemcpy(k->d_grfrag, gr.data(), gr.size() * sizeof(double), hipMemcpyHostToDevice));
  const int ti = K.ntile[nl - 1] - 1;
  KCHECK(hipFuncSetAttribute((const void*)ENCODE[ti], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  KCHECK(hipFuncSetAttribute((const void*)STEP[ti], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  KCHECK(hipFuncSetAttribute((const void*)k_feedforward, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  *out = k;
  return SIM_OK;
}

void sim_koopman_free(sim_koopman* k) {
  if (!k) return;
  (void)hipSetDevice(k->device);
  (void)hipFree(k->d_frag);
  (void)hipFree(k->d_grfrag);
  (void)hipFree(k->d_A);
  (void)hipFree(k->d_B);
  (void)hipFree(k->d_Hh);
  delete k;
}

int sim_koopman_set_bilinear(sim_koopman* k, const double* A, const double* B, const double* Hhat, int delta,
                             double q, double r) {
  if (!k || !A || !B || !Hhat) return soarm_set_error(SIM_E_ARG, "null argument");
  const int nz = k->kd.nz, nu = k->kd.ud, H = k->kd.H, N = H * nu;
  if (nz > 64 || nu > 8 || N > 64) return soarm_set_error(SIM_E_MODEL, "bilinear MPC: nz <= 64, u_dim <= 8, H * u_dim <= 64");
  if (!(q > 0.0) || !(r > 0.0)) return soarm_set_error(SIM_E_ARG, "bilinear MPC: q and r must be positive");
  BDev b{};
  b.nz = nz, b.nu = nu, b.H = H, b.N = N, b.delta = delta ? 1 : 0, b.q = q, b.r = r, b.uclip = k->kd.uclip;
  b.xs = nz * nu + ((nu - nz * nu) % 32 + 32) % 32;
  b.xreg = (std::max(H * b.xs, N * (N + 1) / 2) + 1) & ~1;  // (even: M's column buffer is read as 16-B pairs)
  b.mreg = (std::max(std::max(nz * nu + (H + 1) * nz, N * H), 256) + 1) & ~1;
  b.per_env = b.xreg + b.mreg;
  // as many envs per workgroup as fit the CU's LDS with A (8 at nz 32, nu 5, H 10: 125 KB; the
  // kernel's 215 VGPRs allow 2 waves per SIMD, so 8 is also the register limit)
  b.epw = 0;
  for (int ep : {8, 6, 4, 2, 1})
    if (!b.epw && ((size_t)b.per_env * ep + (size_t)nz * (nz + 1)) * 8 <= 160 * 1024) b.epw = ep;
  if (!b.epw) return soarm_set_error(SIM_E_MODEL, "bilinear MPC does not fit in LDS");
  // Hhat [j][i][c] is already the kernel's layout [j][(i nu + c)]
  std::vector<double> hht(Hhat, Hhat + (size_t)nz * nz * nu);
  KCHECK(hipSetDevice(k->device));
  (void)hipFree(k->d_A), (void)hipFree(k->d_B), (void)hipFree(k->d_Hh);
  k->d_A = k->d_B = k->d_Hh = nullptr;
  KCHECK(hipMalloc(&k->d_A, (size_t)nz * nz * 8));
  KCHECK(hipMalloc(&k->d_B, (size_t)nz * nu * 8));
  KCHECK(hipMalloc(&k->d_Hh, hht.size() * 8));
  KCHECK(hipMemcpy(k->d_A, A, (size_t)nz * nz * 8, hipMemcpyHostToDevice));
  KCHECK(hipMemcpy(k->d_B, B, (size_t)nz * nu * 8, hipMemcpyHostToDevice));
  KCHECK(hipMemcpy(k->d_Hh, hht.data(), hht.size() * 8, hipMemcpyHostToDevice));
  for (const void* f : {(const void*)k_bilinear<8>, (const void*)k_bilinear<6>, (const void*)k_bilinear<4>,
                        (const void*)k_bilinear<2>, (const void*)k_bilinear<1>, (const void*)k_bilinear<8, 10, 5, 32>})
    KCHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  k->bd = b;
  return SIM_OK;
}

int sim_koopman_bilinear_step(sim_koopman* k, int n, const double* z0, const double* window, double* u_prev,
                              float* action, void* stream) {
  if (!k || !z0 || !window || !u_prev || !action || n < 0) return soarm_set_error(SIM_E_ARG, "bad argument");
  if (!k->d_A) return soarm_set_error(SIM_E_ARG, "sim_koopman_set_bilinear was not called");
  if (n == 0) return SIM_OK;
  const int ep = k->bd.epw;
  const bool ref_shape = k->bd.H == 10 && k->bd.nu == 5 && k->bd.nz == 32 && ep == 8;  // (static shapes)
  auto kern = ref_shape ? k_bilinear<8, 10, 5, 32>
              : ep == 8 ? k_bilinear<8>
              : ep == 6 ? k_bilinear<6>
              : ep == 4 ? k_bilinear<4>
              : ep == 2 ? k_bilinear<2>
                        : k_bilinear<1>;
  hipLaunchKernelGGL(kern, dim3((n + ep - 1) / ep), dim3(64 * ep),
                     ((size_t)k->bd.per_env * ep + (size_t)k->bd.nz * (k->bd.nz + 1)) * sizeof(double), (hipStream_t)stream,
                     k->bd, k->d_A, k->d_B,
                     k->d_Hh, n, z0, window, u_prev, action);
  KCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_koopman_encode(sim_koopman* k, int m, const float* x, double* z, void* stream) {
  if (!k || !x || !z || m < 0) return soarm_set_error(SIM_E_ARG, "bad argument");
  if (m == 0) return SIM_OK;
  hipLaunchKernelGGL(ENCODE[k->kd.ntile[k->kd.nl - 1] - 1], dim3((m + 63) / 64), dim3(256),
                     k->kd.total * sizeof(double), (hipStream_t)stream, k->kd, k->d_frag, m, x, z);
  KCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_koopman_feedforward(sim_koopman* k, int nframe, int nref, int n, const double* zref, double* ff,
                            void* stream) {
  if (!k || !zref || !ff || nframe < 0 || nref < 0 || n < 0) return soarm_set_error(SIM_E_ARG, "bad argument");
  if (nframe == 0 || n == 0) return SIM_OK;
  hipLaunchKernelGGL(k_feedforward, dim3((n + 63) / 64, (nframe + FR - 1) / FR), dim3(256),
                     k->kd.gr_ks * 64 * sizeof(double), (hipStream_t)stream, k->kd, k->d_grfrag, nframe, nref, n,
                     zref, ff);
  KCHECK(hipGetLastError());
  return SIM_OK;
}

int sim_koopman_mpc_step(sim_koopman* k, int n, const float* x, const double* z0, const double* ff,
                         double* u_prev, float* action, void* stream) {
  if (!k || (!x && !z0) || !u_prev || !action || n < 0) return soarm_set_error(SIM_E_ARG, "bad argument");
  if (n == 0) return SIM_OK;
  hipLaunchKernelGGL(STEP[k->kd.ntile[k->kd.nl - 1] - 1], dim3((n + 63) / 64), dim3(256),
                     k->kd.total * sizeof(double), (hipStream_t)stream, k->kd, k->d_frag, n, x, z0, ff, u_prev,
                     action);
  KCHECK(hipGetLastError());
  return SIM_OK;
}

}  // extern "C"
