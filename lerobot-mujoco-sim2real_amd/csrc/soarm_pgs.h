// soarm_pgs.h — constraint rows + projected Gauss-Seidel dual solve.
//
// Restates MuJoCo's mj_makeConstraint / mj_makeImpedance / mj_solPGS
//  for the rows the hot path creates: one
// frictionloss row per arm dof (always active), joint-limit rows when a
// hinge is past its range, and 4 pyramidal edges per contact.  Rows are
// visited in MuJoCo's order (friction rows, then limits joint by joint
// lower/upper, then contacts in candidate-pair order), so the sweep matches
// the oracle's.
//
// Where the rows live (one lane = one env, one wave per SIMD at 4096 envs, so
// every sweep is an issue-bound chain and nothing may come from global memory):
//  * dof-frictionloss rows: registers; J = e_i, W = M^-1 J' is a column of the
//    arm block's explicit inverse;
//  * joint-limit rows (rare): a compact list of active rows in LDS;
//  * contacts 0..LDS_CON-1: LDS, [field][lane] (conflict-free), one record per
//    contact holding the 12-dof J_n, J_t1, J_t2; the 4 pyramid edges
//    J_n +- mu J_tk are formed on the fly.  A contact that touches only the
//    free body (cube on table) is swept in its 3-D Gram form: the residuals of
//    its 4 edges are affine in (J_n v, J_t1 v, J_t2 v), so one sweep over the
//    contact costs three 6-dof dots, 4 scalar edge updates and one 6-dof
//    velocity update — the same Gauss-Seidel sequence as updating v per edge;
//  * contacts LDS_CON..SIM_MAXCON-1 (rare): per-edge J/W slab in global
//    scratch, [row][env] SoA.
// PGS on the resting cube's 16 redundant edges needs ~96 sweeps per substep
// (measured on the oracle with MuJoCo's improvement criterion), so the sweep
// body is the hot loop of the contact scene.
#pragma once
#include <type_traits>
#include <utility>

#include "soarm_collide.h"

namespace soarm {

#ifdef SOARM_PHASE_PROF
// diagnostic build only: per-env PGS start/end clock, sweep count, fast-path flag (env < 65536)
__device__ long long g_pgs_prof[65536 * 8];
// fine-grained per-env clock stamps of one k_substep (diagnostic build): see k_substep
__device__ long long g_stamp[65536 * 16];
#define PSTAMP(k) \
  if (e < 65536) g_stamp[16 * e + (k)] = clock64()
// per-wave accumulators of k_substep's phase profile (layout: soarm_substep.h g_phase; [77..81] the
// RS solve's split).  Lane 0 of each wave owns its row and launches are stream-ordered, so plain
// read-modify-writes: shared-address atomics from every wave queued behind the profiled kernel's own
// loads and inflated the phases after the solve ~15x (r05).  sim_phase_profile reduces the rows.
// [82..84]: RS-kernel waves that took the v-form fallback -- count, max and summed wave cycles;
// [85..91] lanes of such waves by cause (rs_why bits).
constexpr int WPH = 92, WPH_MAXW = 16384;
__device__ unsigned long long g_wphase[WPH_MAXW * WPH];
#define WPH_ID() (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6)
__device__ int g_rs_force11;  // (set from SOARM_RS_FORCE11 by the launch code)
#define WPH_ADD(k, v) g_wphase[WPH_ID() * WPH + (k)] += (unsigned long long)(v)
#define WPH_MAX(k, v) \
  g_wphase[WPH_ID() * WPH + (k)] = max(g_wphase[WPH_ID() * WPH + (k)], (unsigned long long)(v))
// contact-row build split: [0] loads + frame, [1] Jacobian, [2] Gram / M^-1 / velocities, [3] edges + LDS writes
__device__ long long g_rowprof[65536 * 4];
#define RP_INIT long long rp_acc[4] = {0, 0, 0, 0}, rp_t = clock64()
#define RP_MARK(k)                  \
  {                                 \
    const long long t_ = clock64(); \
    rp_acc[k] += t_ - rp_t;         \
    rp_t = t_;                      \
  }
#define RP_STORE \
  if (e < 65536) g_rowprof[4 * e] = rp_acc[0], g_rowprof[4 * e + 1] = rp_acc[1], g_rowprof[4 * e + 2] = rp_acc[2], g_rowprof[4 * e + 3] = rp_acc[3]
#else
#define PSTAMP(k)
#define RP_INIT
#define RP_MARK(k)
#define RP_STORE
#endif

constexpr int LDS_CON = 6;  // contacts whose rows stay in LDS
// Lanes per env of the contact substep kernel: 4 lanes run the same per-env code
// (identical values, so identical stores) and split the parts that fan out -- contact-row
// construction, the warm start, the next substep's geom poses -- and, in scenes with a
// free body, the contact-space sweep of the cube block gives lane k ownership of block
// contact k's residuals (its cross-Gram row), broadcast within the quad (DPP) on that
// contact's turn.  The arm-only scene has no block; its quad splits the other parts.
#ifndef SOARM_LPE
#define SOARM_LPE 4
#endif
#ifndef SOARM_LPE_ARM
#define SOARM_LPE_ARM 4
#endif
template <int NF>
constexpr int lpe() { return NF == 1 ? SOARM_LPE : SOARM_LPE_ARM; }
// value of lane J of each quad (DPP quad_perm broadcast); J is a compile-time 0..3
// projected Gauss-Seidel step of a pyramid edge, max(x, -f): one VOP3 max with a
// negated source.  fmaxf(x, -f) on a loop-carried f costs an extra canonicalising
// v_max(-f, -f) per edge (IEEE mode: the compiler cannot prove -f canonical); every
// operand here is a finite arithmetic result, so the plain instruction is exact.
// Used only in loops without memory reads: an inline asm is not known to return, so
// LICM keeps loads that follow it inside the loop.
// packed FP32 (v_pk_fma_f32 / v_pk_add_f32): one wave per SIMD issues a VALU op every
// ~4.7 cycles whether it is packed or not, so two independent FMAs on a register pair
// cost one issue slot (tools/mb_chain.hip)
typedef float f2 __attribute__((ext_vector_type(2)));
DEVI f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
DEVI f2 splat2(float x) { return f2{x, x}; }
// a * (b.y, b.y) + c: the high half of a pair splatted by op_sel (the compiler copies it to a
// low half first)
DEVI f2 fma2_hi(f2 a, f2 b, f2 c) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
DEVI float max_neg(float x, float f) {
  float r;
  asm("v_max_f32_e64 %0, %1, -%2" : "=v"(r) : "v"(x), "v"(f));
  return r;
}
// re-define a value in a VGPR (an empty asm): starts a new live range at this point
DEVI void vpin(float& x) { asm volatile("" : "+v"(x)); }
DEVI void vpin(f2& x) { asm volatile("" : "+v"(x)); }
DEVI float qbcast(float x, int j) {
  const int b = __float_as_int(x);
  switch (j) {
    case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xFF, 0xF, 0xF, false));
  }
}
// LDS written by other lanes of the (single-wave) workgroup is read after this
DEVI void wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
// sum over the quad, bit-identical in its 4 lanes (butterfly of commutative adds)
DEVI float qsum(float x) {
  const float t = x + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
  return t + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x4E, 0xF, 0xF, false));
}
constexpr int CF = 61;      // LDS floats per contact record
// record fields: [0, 3*12) J_n | J_t1 | J_t2 (12 slots each), 36..39 aref_e,
// 40..43 ARdiag_e / 2, 44..47 force_e, 48..51 1/ARdiag_e, 52 mu, 53 R (pyramid),
// 54 flags, 55..60 Gram matrix G = [J_n; J_t1; J_t2] M^-1 [..]' (nn, n1, n2, 11, 12, 22)
// of a contact that touches only the free body (diagonal M^-1)
enum { F_AREF = 36, F_HARD = 40, F_FRC = 44, F_IARD = 48, F_MU = 52, F_R = 53, F_FLAGS = 54, F_GRAM = 55 };
enum { TOUCH_ARM = 1, TOUCH_FREE = 2 };
// Sim state not used by the sweeps but needed after them (mass matrix blocks for the
// implicit-damping solve, smooth forces, observed site): parked in LDS so the sweep's
// register budget is not spent holding it.  Arm block packed (21) + free-body diagonals
// (6 per free body; the free block is diagonal, host-validated) + qfrc_smooth + ee.
template <int NA, int NF>
constexpr int keep_floats() { return NA * (NA + 1) / 2 + 6 * NF + (NA + 6 * NF) + 3; }
// joint-limit rows (rare): compact list, one record per active limit
constexpr int LF = 7;  // dof, sign, aref, R, ARdiag, 1/ARdiag, force
// PGS: the arm's rows are retired from the sweeps of a pure-block / uncoupled-extra solve once
// one sweep moves their forces by at most this much in total (N, N m); see ysweeps
constexpr float ARM_RETIRE = 1e-6f;
constexpr int XS_LIST = SIM_MAXCON;           // ext[0, XS_LIST): the env's contact list (quad build)
constexpr int XS_EXT = XS_LIST + 98;           // + extra-slot scratch beyond the limit list
enum { L_DOF = 0, L_SGN = 1, L_AREF = 2, L_R = 3, L_ARD = 4, L_IARD = 5, L_FRC = 6 };

// ---- Row-space PGS (the RS kernel: k_substep<..., RS>, 16 lanes per env, 4 envs per wave).
// MuJoCo's mj_solPGS sweeps the dual on the dense matrix AR = J M^-1 J' + R (efc_AR): row i's
// residual is AR_i f + b_i, its force steps by -res / AR_ii and is projected (frictionloss
// rows into [-fl, fl], limit rows and pyramid edges to f >= 0), rows in order.  The RS kernel
// holds that system directly: lane r of an env's 16-lane DPP row owns constraint rows r
// (slot A) and 16 + r (slot B) -- every frictionloss, limit and pyramid-edge row, from the
// first sweep to the last -- with the row's scaled residual s_r = -res_r / AR_rr and its row of
// the scaled matrix C[r][q] = -AR_rq / AR_rr (C[r][r] = -1) in registers.  Step q of a sweep:
// the projected step d = clamp(s_q, lo_q - f_q, hi_q - f_q) is formed from lane q's residual by
// a DPP row broadcast fused into the max (v_max_f32_dpp row_newbcast), every lane moves its
// residuals by C[r][q] d (one packed FMA per slot), and the step's bound registers (-f_q,
// kept broadcast in every lane of the env) take it: two dependent instructions per row.
// The improvement of mj_solPGS's stopping test is the sweep's exact cost change: with
// res = AR f + b, cost(f0) - cost(f1) = sum_r AR_rr / 2 (f1 - f0)_r (s0 + s1)_r, and each
// row's force change over the sweep is its own step, which a second accumulator beside s takes
// exactly (its coefficient is 1 at the row's own step, 0 elsewhere).
#ifndef SOARM_RS_SEQ
#define SOARM_RS_SEQ 0  // 1: the decoupled layouts' steps one at a time (A/B of the paired sweep)
#endif
constexpr int RS_MAXROW = 32;               // rows of one env (2 slots x 16 lanes)
constexpr int RS_WROW = 12;                 // floats per row of W = M^-1 J' in LDS (NV <= 12)
constexpr int RS_WENV = RS_MAXROW * RS_WROW + 4;  // per env (+4: the 4 envs of a wave on distinct banks)
constexpr int RS_EPW = 4;                   // envs per wave (workgroup)
template <int Q>
DEVI float rowbcast(float x) {  // lane Q of each 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x150 + Q, 0xF, 0xF, true));
}
// sum over the 16-lane row, bit-identical in all 16 lanes (the stop test must agree)
// (the permutes fused into the adds, v_add_f32_dpp; every stage adds two values that are equal
// bit for bit within each pair of partners -- quad xor 1, quad xor 2, the 8-lane mirror, the
// 16-lane mirror -- and fp addition is commutative, so all 16 lanes end with the same bits)
DEVI float rowsum16(float x) {
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(x));
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(x));
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x));
  return x;
}
// max(lane Q's x, b): the row broadcast fused into the max (VOP2 DPP).  A DPP read of a VGPR needs
// 2 wait states after the VALU write of it, and the compiler's hazard recognizer does not look into
// inline asm: the caller states how many instructions (NOPS = 2 - that count) must be padded.
template <int Q, int NOPS = 2>
DEVI float max_bcast(float x, float b) {
  float r;
  if constexpr (NOPS >= 2)
    asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x), "v"(b), "i"(Q));
  else if constexpr (NOPS == 1)
    asm volatile("s_nop 0\n\tv_max_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x), "v"(b), "i"(Q));
  else
    asm volatile("v_max_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x), "v"(b), "i"(Q));
  return r;
}
DEVI float vmin(float a, float b) {  // v_min without the IEEE-mode canonicalising of fminf
  float r;
  asm("v_min_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// f(std::integral_constant<int, i>) for i = 0 .. N-1 (compile-time lane / register indices)
template <class F, int... Is>
DEVI void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
DEVI void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}
// Row layout of one wave's RS solve (compile time).  Steps in mj_solPGS order: the NA dof
// frictionloss rows (F), then the edges of up to KAT arm-only contacts (AT: arm on the table /
// floor, arm self-contacts), of up to 4 contacts on the free body alone (CT: the cube on the
// table), of up to KAC contacts between the arm and the free body (AC) -- the order the pair
// list produces (arm-only pairs precede the free body's, its world pairs precede its arm pairs).
// Rows touching arm dofs (F, AT, AC) live in slot B, the CT edges in slot A: M is block diagonal,
// so an F / AT step moves slot B alone and a CT step slot A alone (and slot B's AC rows when the
// wave has an AC contact); a step therefore costs one residual update where the systems decouple.
// Steps an env has no row for are zero rows (exact no-ops).
template <int NA, int KAT, int KAC>
struct RsLayout {
  static_assert(NA + 4 * (KAT + KAC) <= 16, "slot B holds the F, AT and AC rows");
  static constexpr int CT0 = NA + 4 * KAT, AC0 = CT0 + 16, NS = AC0 + 4 * KAC;
  static constexpr bool decoupled = KAC == 0;  // no AC rows: the slot-B (arm) and slot-A (cube) steps never meet
  static constexpr int slot(int q) { return (q >= CT0 && q < AC0) ? 0 : 1; }
  static constexpr int lane(int q) { return q < CT0 ? q : q < AC0 ? q - CT0 : q - 16; }
  static constexpr bool upd_a(int q) { return q >= CT0; }                 // CT, AC
  static constexpr bool upd_b(int q) { return q < CT0 || q >= AC0 || KAC > 0; }
  // instructions after step q's write of slot sl before step q+1 (see rs_sweep's order)
  static constexpr int after_write(int q, int sl) {
    return (sl == 0 ? upd_a(q) : upd_b(q)) ? ((upd_a(q) && upd_b(q)) ? 1 : 0) + 1 + (q < NA ? 1 : 0) : 2;
  }
};
// one sweep of the row-space PGS (see above): s = (residual, own-step accumulator) per slot,
// C = (C, G) pairs per step, NF = lo - f of every row, NH = hi - f of the NA frictionloss rows (the
// others have hi = +inf).  Instruction order is pinned (sched_barrier): a DPP op waits for every
// VALU op in flight, so a step is its broadcast-max, the residual update of the slot the NEXT step
// broadcasts from, then the other slot's update and the bound updates -- which are also the 2 wait
// states the next broadcast needs after that write (padded with s_nop where a step has fewer)
//
// Layouts without AC rows (KAC = 0: no arm-cube contact in the wave, ~99.6% of the headline's waves)
// are two systems that never meet: the F / AT steps read and move slot B alone, the CT steps slot A
// alone (M is block diagonal).  Their steps then run paired -- B step i beside A step i, two
// independent chains in one instruction stream, each hiding the other's latency and DPP drain --
// and each slot still takes its own steps in mj_solPGS order, so every residual, force and
// accumulator is bit-identical to the sequential sweep.
template <int NA, class LY>
DEVI void rs_sweep(f2& sA, f2& sB, const f2 (&CA)[LY::NS], const f2 (&CB)[LY::NS], float (&NF)[LY::NS],
                   float (&NH)[NA]) {
  if constexpr (LY::decoupled && !SOARM_RS_SEQ) {
    constexpr int NB = LY::CT0, NAS = LY::NS - LY::CT0;  // slot-B steps (F, AT), slot-A steps (CT)
    static_assert(NB <= NAS, "slot A has at least as many steps as slot B");
    sfor<NAS>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      constexpr bool HB = I < NB;
      constexpr int QA = LY::CT0 + I;
      // wait states before this step's broadcasts (2 needed after the VALU write of the source):
      // B reads sB, written by step I-1's first update, with the sA update and >= 2 bound updates
      // after it; A reads sA, written by step I-1's second update, with step I-1's bound updates
      // (2 when it had a B step, else 1) and this step's B broadcast after it
      constexpr int waitA = I == 0 ? 0 : ((I - 1) < NB ? 2 + (HB ? 1 : 0) : 1 + (HB ? 1 : 0));
      float dB = 0.f, dA;
      if constexpr (HB) dB = max_bcast<LY::lane(I), (I == 0 ? 2 : 0)>(sB.x, NF[I]);
      dA = max_bcast<LY::lane(QA), (waitA >= 2 ? 0 : 2 - waitA)>(sA.x, NF[QA]);
      if constexpr (HB && I < NA) dB = vmin(dB, NH[I]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (HB) sB = __builtin_elementwise_fma(CB[I], f2{dB, dB}, sB);
      __builtin_amdgcn_sched_barrier(0);
      sA = __builtin_elementwise_fma(CA[QA], f2{dA, dA}, sA);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (HB) {
        NF[I] -= dB;
        if constexpr (I < NA) NH[I] -= dB;
      }
      NF[QA] -= dA;
      __builtin_amdgcn_sched_barrier(0);
    });
    return;
  }
  sfor<LY::NS>([&](auto qc) {
    constexpr int Q = decltype(qc)::value;
    constexpr int SL = LY::slot(Q), LN = LY::lane(Q);
    constexpr int after = Q == 0 ? 0 : LY::after_write(Q - 1, SL);
    float d = max_bcast<LN, (after >= 2 ? 0 : 2 - after)>(SL == 0 ? sA.x : sB.x, NF[Q]);
    if constexpr (Q < NA) d = vmin(d, NH[Q]);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int NSL = Q + 1 < LY::NS ? LY::slot(Q + 1) : SL;  // the next step's source slot
    auto upd = [&](auto slc) {
      if constexpr (decltype(slc)::value == 0) {
        if constexpr (LY::upd_a(Q)) sA = __builtin_elementwise_fma(CA[Q], f2{d, d}, sA);
      } else {
        if constexpr (LY::upd_b(Q)) sB = __builtin_elementwise_fma(CB[Q], f2{d, d}, sB);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    upd(std::integral_constant<int, NSL>{});
    upd(std::integral_constant<int, 1 - NSL>{});
    NF[Q] -= d;
    if constexpr (Q < NA) NH[Q] -= d;
    __builtin_amdgcn_sched_barrier(0);
  });
}

// Per-env LDS state, [field][column]: one column per env of the workgroup (64 / lanes per
// env); the lanes of an env share its column (identical values, or records written by the
// one lane that built them).
struct RowLds {
  float* a;     // [(LDS_CON + 1) * CF][cols] contact records + a zero record (null: contact-free kernel)
  float* lim;   // [NA * LF][cols] active joint-limit records
  float* keep;  // [KEEP][cols] state held in LDS across the PGS sweeps (null: kept in registers)
  float* ext;   // [XS_EXT][cols] scratch of the y sweep (contact list, extra contact slots)
  int lane;     // thread in the workgroup
  int col;      // this env's column
  int cols;     // columns (envs per workgroup)
  float* rsw = nullptr;  // RS kernel: [env column][RS_WENV] rows of W = M^-1 J' (row-space PGS), else null
  DEVI float& at(int c, int f) const { return a[(c * CF + f) * cols + col]; }
  DEVI float& lm(int l, int f) const { return lim[(l * LF + f) * cols + col]; }
  DEVI float& lraw(int k) const { return lim[k * cols + col]; }
  DEVI float& kp(int k) const { return keep[k * cols + col]; }
  DEVI float& ex(int k) const { return ext[k * cols + col]; }
};

// The env's pair-mask words, loaded at the top of the substep (they come from the previous
// collide launch) so their round trip overlaps the smooth dynamics instead of starting the
// contact-row build; `hold` pins them (the loads stay above, the registers are not sunk).
// Zero (no contacts) unless loaded.
// cw: the count word of the multi-contact pairs (DModel::pair_cq), so the contact list needs
// no per-pair count load.
struct PairMask {
  static constexpr int MAXW = (SIM_MAXPAIR + 31) / 32;
  uint32_t w[MAXW] = {}, cw = 0u;
  DEVI void load(const uint32_t* __restrict__ pmask, const DModel& m, int n, int e) {
    const int nw = (m.npair + 31) >> 5;
#pragma unroll
    for (int k = 0; k < MAXW; k++) w[k] = k < nw ? soa(pmask, k, n, e) : 0u;
    if (m.ncq > 0) cw = soa(pmask, nw, n, e);
  }
  DEVI void hold() {
#pragma unroll
    for (int k = 0; k < MAXW; k++) asm volatile("" : "+v"(w[k]));
    asm volatile("" : "+v"(cw));
  }
  DEVI int count(const DModel& m, int p) const {
    const int cq = m.pair_cq[p];
    return cq < 0 ? 1 : (int)((cw >> (2 * cq)) & 3u) + 1;
  }
  // the same for pair 32 w + b from the word's tables (w compile-time: no per-lane load)
  DEVI int count_w(const DModel& m, int w, int b) const {
    const uint32_t mu = m.pair_mw_multi[w], bit = 1u << b;
    if (!(mu & bit)) return 1;
    const int cq = m.pair_cqbase[w] + __popc(mu & (bit - 1u));
    return (int)((cw >> (2 * cq)) & 3u) + 1;
  }
};

// first row past the contact rows of the scratch slab (sim_batch d_scratch): Newton's zone history
template <int NA, int NF>
constexpr int zhist_row() { return 4 * SIM_MAXCON * (2 * (NA + 6 * NF) + 4); }
template <int NA, int NF>
struct ContactRows {
  static constexpr int NV = NA + 6 * NF;
  // overflow rows (edge r of contact c >= LDS_CON): J[NV], W[NV], aref, R, ARdiag, force
  float* base;  // = scratch + e
  int stride;   // = n envs
  DEVI float& J(int r, int i) const { return base[((size_t)r * (2 * NV + 4) + i) * stride]; }
  DEVI float& W(int r, int i) const { return base[((size_t)r * (2 * NV + 4) + NV + i) * stride]; }
  DEVI float& S(int r, int k) const { return base[((size_t)r * (2 * NV + 4) + 2 * NV + k) * stride]; }
};

// explicit inverse of the block-diagonal M: arm block + one 6x6 per free body
template <int NA, int NF>
struct MInv {
  static constexpr int NV = NA + 6 * NF;
  float A[NA * (NA + 1) / 2];     // arm block inverse, packed lower triangle (symmetric)
  float Fd[NF > 0 ? NF : 1][6];   // free bodies: diagonal mass block (host-validated) -> 1/M_ii
  DEVI float a(int i, int k) const { return i >= k ? A[i * (i + 1) / 2 + k] : A[k * (k + 1) / 2 + i]; }
  DEVI void build(const Sim<NA, NF>& S) {
#pragma unroll
    for (int i = 0; i < NA; i++) {
      float ei[NA], col[NA];
#pragma unroll
      for (int k = 0; k < NA; k++) ei[k] = (k == i) ? 1.f : 0.f;
      ldl_solve<NA>(S.LA, S.DAi, col, ei);
#pragma unroll
      for (int k = 0; k <= i; k++) A[i * (i + 1) / 2 + k] = col[k];
    }
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
      for (int i = 0; i < 6; i++) Fd[f][i] = 1.f / S.MF[f][i * (i + 1) / 2 + i];
  }
  // y = M^-1 x, restricted to the halves x can be nonzero on
  DEVI void mul(const float x[NV], float y[NV], bool arm, bool fr) const {
#pragma unroll
    for (int i = 0; i < NV; i++) y[i] = 0.f;
    if (arm) {
#pragma unroll
      for (int i = 0; i < NA; i++) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NA; k++) s += a(i, k) * x[k];
        y[i] = s;
      }
    }
    if (fr) {
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int i = 0; i < 6; i++) y[NA + 6 * f + i] = Fd[f][i] * x[NA + 6 * f + i];
    }
  }
};

// diagonal inverse mass of the (single) free body, dof i of its 6
#define S_FD(Mi, i) ((Mi).Fd[0][(i)])

template <int NA, int NF>
DEVI float dotv(const float a[], const float b[], bool arm, bool fr) {
  constexpr int NV = NA + 6 * NF;
  float s0 = 0.f, s1 = 0.f;
  if (arm) {
#pragma unroll
    for (int i = 0; i < NA; i++) s0 += a[i] * b[i];
  }
  if (fr) {
#pragma unroll
    for (int i = NA; i < NV; i++) s1 += a[i] * b[i];
  }
  return s0 + s1;
}

// pyramid edge e of a contact from its J_n, J_t1, J_t2:  J_n +- mu J_tk
template <int NV>
DEVI void edge_J(const float jn[NV], const float jt1[NV], const float jt2[NV], int e, float mu, float J[NV]) {
  const float s = (e & 1) ? -mu : mu;
  const float* jt = (e >> 1) ? jt2 : jt1;
#pragma unroll
  for (int i = 0; i < NV; i++) J[i] = jn[i] + s * jt[i];
}

// Lane-varying dof index i < N without dynamic register indexing (which would put
// the arrays in scratch): one-hot weights, then dots.
template <int N>
DEVI void one_hot(int i, float* oh) {
#pragma unroll
  for (int k = 0; k < N; k++) oh[k] = (i == k) ? 1.f : 0.f;
}
template <int N>
DEVI float pick(const float* v, const float* oh) {
  float r = 0.f;
#pragma unroll
  for (int k = 0; k < N; k++) r = fmaf(oh[k], v[k], r);
  return r;
}

// v_arm += M^-1 e_i * sgf for the one-hot dof oh
template <int NA, int NF>
DEVI void add_arm_col(const MInv<NA, NF>& Mi, float* v, const float* oh, float sgf) {
#pragma unroll
  for (int k = 0; k < NA; k++) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < NA; j++) a = fmaf(oh[j], Mi.a(k, j), a);
    v[k] = fmaf(a, sgf, v[k]);
  }
}

// Per edge e of a contact, the column of its Gram matrix for J_e = J_n + s J_tk
// (s = +-mu): how (J_n v, J_t1 v, J_t2 v) move per unit force on edge e.
DEVI void gram_coefs(const float G[6], float mu, float cf[12]) {
#pragma unroll
  for (int ed = 0; ed < 4; ed++) {
    const float s = (ed & 1) ? -mu : mu;
    const bool k2 = ed >> 1;
    cf[3 * ed + 0] = G[0] + s * (k2 ? G[2] : G[1]);
    cf[3 * ed + 1] = G[1] + s * (k2 ? G[4] : G[3]);
    cf[3 * ed + 2] = G[2] + s * (k2 ? G[5] : G[4]);
  }
}

// One Gauss-Seidel pass over the 4 pyramid edges of a free-body-only contact in
// Gram form: a, b, c = J_n v, J_t1 v, J_t2 v; each edge's residual is a + s b
// (or c) - aref + R f; its force step moves (a, b, c) by the Gram column; the
// free body's velocity block v6 is updated once at the end.  Same sequence as
// updating v after every edge.
DEVI void gram_step(float* v6, const float* jn, const float* j1, const float* j2, const float* cf,
                    const float* ar, const float* ia, const float* hd, float* fo, float mu, float Rp,
                    const float* Fd, float& improvement) {
  float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    a += jn[i] * v6[i];
    b += j1[i] * v6[i];
    cc += j2[i] * v6[i];
  }
  float df[4];
#pragma unroll
  for (int ed = 0; ed < 4; ed++) {
    const float s = (ed & 1) ? -mu : mu;
    const float res = (a + s * ((ed >> 1) ? cc : b)) - ar[ed] + Rp * fo[ed];
    const float fnew = fmaxf(fo[ed] - res * ia[ed], 0.f);
    df[ed] = fnew - fo[ed];
    a += cf[3 * ed] * df[ed];
    b += cf[3 * ed + 1] * df[ed];
    cc += cf[3 * ed + 2] * df[ed];
    improvement -= df[ed] * (res + hd[ed] * df[ed]);
    fo[ed] = fnew;
  }
  // sum_e J_e df_e = J_n (df0+df1+df2+df3) + mu J_t1 (df0-df1) + mu J_t2 (df2-df3)
  const float Dn = (df[0] + df[1]) + (df[2] + df[3]);
  const float D1 = mu * (df[0] - df[1]), D2 = mu * (df[2] - df[3]);
#pragma unroll
  for (int i = 0; i < 6; i++) v6[i] += Fd[i] * (jn[i] * Dn + j1[i] * D1 + j2[i] * D2);
}

}  // namespace soarm
#include "soarm_newton.h"
namespace soarm {

// Builds every constraint row, solves the dual by PGS (or, SOL = Newton, the primal by
// soarm_newton.h), sets S.qacc / S.fcon.
// Contacts are read straight from the collide output (pair mask + cbuf, pair
// order).  Returns the number of contacts used.
template <int NA, int NF, bool CON, int SOL = SIM_SOL_PGS, bool RS = false>
DEVI int solve_constraints(Sim<NA, NF>& S, const float* __restrict__ cbuf, const int* __restrict__ ccount,
                           const uint32_t* __restrict__ pmask, int n, int e, const RowLds& L,
                           const ContactRows<NA, NF>& cr, const PairMask& pm) {
  constexpr int NV = Sim<NA, NF>::NV;
  const DModel& m = *S.mp;
  // Newton needs neither M^-1 nor the rows' ARdiag (PGS's step sizes): its rows are J, aref, R
  constexpr bool NEWT = SOL == SIM_SOL_NEWTON;
  S.solve_m(S.qacc_s, S.fsmooth);
  MInv<NA, NF> Mi;
  if constexpr (!NEWT) Mi.build(S);
  PSTAMP(6);

  // RS kernel: whether every env of the wave takes the row-space solve (decided once the contacts
  // are listed: no overflow rows, at most RS_MAXROW rows); it then needs neither the records'
  // Gram blocks / edge ARdiag nor the warm start below (rs_solve builds its own)
  bool rs_fast = false;
  int rs_nat = 0, rs_nct = 0, rs_nac = 0;  // contacts per category (RsLayout): arm-only, free body alone, both
#ifdef SOARM_PHASE_PROF
  int rs_why = 0;  // why a wave takes the fallback (bits: limit, overflow, order, CT>4, AT>1, AC>1, AT+AC)
#endif
  // ---- dof frictionloss rows (MuJoCo row order: all of them first)
  float ff[NA], fa[NA], fR[NA], fhD[NA], fiD[NA];
#pragma unroll
  for (int i = 0; i < NA; i++) {
    fR[i] = m.dof_fricR[i];
    fa[i] = -m.dof_fricB[i] * S.qvel[i];
    if constexpr (!NEWT) {
      const float ard = Mi.a(i, i) + fR[i];
      fhD[i] = 0.5f * ard;
      fiD[i] = 1.f / ard;
    }
  }
  // ---- joint-limit rows: joint by joint, lower then upper; compact list in LDS
  int nlim = 0;
#pragma unroll
  for (int i = 0; i < NA; i++) {
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const float dist = side == 0 ? S.qpos[i] - m.jnt_range[i][0] : m.jnt_range[i][1] - S.qpos[i];
      if (m.jnt_limited[i] && dist < m.jnt_margin[i]) {
        const float imp = impedance(m.jnt_solimp[i], dist, m.jnt_margin[i]);
        const float R = fmaxf(MINVALF, (1.f - imp) * m.dof_invweight0[i] / imp);
        const float vel = side == 0 ? S.qvel[i] : -S.qvel[i];
        L.lm(nlim, L_DOF) = (float)i;
        L.lm(nlim, L_SGN) = side == 0 ? 1.f : -1.f;
        L.lm(nlim, L_AREF) = -m.jnt_KB[i][1] * vel - m.jnt_KB[i][0] * imp * (dist - m.jnt_margin[i]);
        L.lm(nlim, L_R) = R;
        if constexpr (!NEWT) {
          const float ard = Mi.a(i, i) + R;
          L.lm(nlim, L_ARD) = ard;
          L.lm(nlim, L_IARD) = 1.f / ard;
        } else {
          L.lm(nlim, L_IARD) = 1.f / R;  // Newton: the row's 1/R
        }
        nlim++;
      }
    }
  }

  PSTAMP(7);
  // ---- contact rows, straight from the collide output in pair order
  int ncon = 0;
  RP_INIT;
  // Contact row c from its collide output rw (dist, pos, normal geom1 -> geom2) and its pair's
  // constants: record c (LDS, c < LDS_CON) or the overflow slab.  split: lane-split build
  // (quad mode), the building lane writes the record into all 4 columns of its quad.
  auto wrec = [&](int c, int f, float x, bool split) {
    (void)split;  // the env's column is shared by its lanes: one store serves the quad
    L.at(c, f) = x;
  };
  auto build_row = [&](int c, const float* rw, int b1, int b2, float mu, float tran, float margin, float KB0,
                       float KB1, const float* si, bool split) {
      const float cdist = rw[0];
      const float cpos[3] = {rw[1], rw[2], rw[3]};
      float fr[9] = {rw[4], rw[5], rw[6], 0, 0, 0, 0, 0, 0};
      {  // contact frame (mju_makeFrame)
        float y[3];
        if (fabsf(fr[1]) < 0.5f)
          y[0] = 0, y[1] = 1, y[2] = 0;
        else
          y[0] = 0, y[1] = 0, y[2] = 1;
        const float dd = dot3(fr, y);
        y[0] -= dd * fr[0], y[1] -= dd * fr[1], y[2] -= dd * fr[2];
        const float inv = rsqrtf(dot3(y, y));
        fr[3] = y[0] * inv, fr[4] = y[1] * inv, fr[5] = y[2] * inv;
        cross(fr + 6, fr, fr + 3);
      }
      RP_MARK(0);
      // relative translational Jacobian (body2 - body1) at the contact point, contact frame
      float jd[3][NV];
#pragma unroll
      for (int i = 0; i < NV; i++) jd[0][i] = jd[1][i] = jd[2][i] = 0.f;
      int flags = 0;
#pragma unroll
      for (int side = 0; side < 2; side++) {
        const int b = side ? b2 : b1;
        const float sg = side ? 1.f : -1.f;
        if (b >= 2 && b < 2 + NA) flags |= TOUCH_ARM;
#pragma unroll
        for (int i = 0; i < NA; i++) {
          if (b >= i + 2 && b < 2 + NA) {  // hinge i moves chain bodies i+2.. (reference point: origin)
            float l[3];
            cross(l, S.cdof[i], cpos);
            const float jp[3] = {S.cdof[i][3] + l[0], S.cdof[i][4] + l[1], S.cdof[i][5] + l[2]};
#pragma unroll
            for (int q = 0; q < 3; q++) jd[q][i] += sg * dot3(fr + 3 * q, jp);
          }
        }
#pragma unroll
        for (int ff2 = 0; ff2 < NF; ff2++) {
          const int fb = 2 + NA + ff2, d0 = NA + 6 * ff2;
          if (b == fb) {
            flags |= TOUCH_FREE;
            const float off[3] = {cpos[0] - S.xpos[fb][0], cpos[1] - S.xpos[fb][1], cpos[2] - S.xpos[fb][2]};
#pragma unroll
            for (int i = 0; i < 6; i++) {
              float l[3];
              cross(l, S.cdof[d0 + i], off);
              const float jp[3] = {S.cdof[d0 + i][3] + l[0], S.cdof[d0 + i][4] + l[1], S.cdof[d0 + i][5] + l[2]};
#pragma unroll
              for (int q = 0; q < 3; q++) jd[q][d0 + i] += sg * dot3(fr + 3 * q, jp);
            }
          }
        }
      }
      const bool ta = flags & TOUCH_ARM;
      RP_MARK(1);
      const float imp = impedance(si, cdist, margin);
      const float diag = tran + mu * mu * tran;
      const float R0 = fmaxf(MINVALF, (1.f - imp) * diag / imp);
      const float Rpy = 2.f * mu * mu * R0 / m.impratio;
      const bool lds = c < LDS_CON;
      if (lds) {
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int i = 0; i < NV; i++) wrec(c, 12 * q + i, jd[q][i], split);
        wrec(c, F_MU, mu, split);
        wrec(c, F_R, Rpy, split);
        wrec(c, F_FLAGS, (float)flags, split);
        if constexpr (NEWT) wrec(c, F_IARD, 1.f / Rpy, split);  // Newton: the pyramid's 1/R
      }
      // Gram matrix G = [Jn; Jt1; Jt2] M^-1 [Jn; Jt1; Jt2]' and the three velocities:
      // every pyramid edge J_e = J_n + s J_tk (s = +-mu) follows from them.  Full
      // width (jd is zero on the halves the contact does not touch; branch-free code
      // avoids running both sides of a divergent flag test) unless no lane's contact
      // touches the arm: then the free-body half alone (diagonal M^-1).
      float W0[NV], W1[NV], W2[NV], G[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (!NEWT && !rs_fast) {
        const bool arm_any = NF == 0 || !__all(!ta);
        Mi.mul(jd[0], W0, arm_any, true);
        Mi.mul(jd[1], W1, arm_any, true);
        Mi.mul(jd[2], W2, arm_any, true);
        G[0] = dotv<NA, NF>(jd[0], W0, arm_any, true), G[1] = dotv<NA, NF>(jd[0], W1, arm_any, true);
        G[2] = dotv<NA, NF>(jd[0], W2, arm_any, true), G[3] = dotv<NA, NF>(jd[1], W1, arm_any, true);
        G[4] = dotv<NA, NF>(jd[1], W2, arm_any, true), G[5] = dotv<NA, NF>(jd[2], W2, arm_any, true);
      }
      float vq[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NV; i++)
        vq[0] += jd[0][i] * S.qvel[i], vq[1] += jd[1][i] * S.qvel[i], vq[2] += jd[2][i] * S.qvel[i];
      if (!NEWT && !rs_fast)
        if (lds) {
#pragma unroll
          for (int k2 = 0; k2 < 6; k2++) wrec(c, F_GRAM + k2, G[k2], split);
        }
      RP_MARK(2);
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
        const float s = (ed & 1) ? -mu : mu;
        const bool k2 = ed >> 1;
        const float vel = vq[0] + s * (k2 ? vq[2] : vq[1]);
        // J_e M^-1 J_e' = G_nn + 2 s G_nk + s^2 G_kk
        const float ard = NEWT ? 0.f : G[0] + s * (2.f * (k2 ? G[2] : G[1]) + s * (k2 ? G[5] : G[3])) + Rpy;
        const float ar = -KB1 * vel - KB0 * imp * (cdist - margin);
        if (lds) {
          wrec(c, F_AREF + ed, ar, split);
          if (!NEWT && !rs_fast) {
            wrec(c, F_HARD + ed, 0.5f * ard, split);
            wrec(c, F_IARD + ed, 1.f / ard, split);
          }
        } else {
          const int r = 4 * c + ed;
#pragma unroll
          for (int i = 0; i < NV; i++) {
            cr.J(r, i) = jd[0][i] + s * (k2 ? jd[2][i] : jd[1][i]);
            if constexpr (!NEWT) cr.W(r, i) = W0[i] + s * (k2 ? W2[i] : W1[i]);
          }
          cr.S(r, 0) = ar;
          cr.S(r, 1) = Rpy;
          cr.S(r, 2) = NEWT ? 1.f / Rpy : ard;  // (Newton: 1/R)
        }
      }
  };

  constexpr bool QUADR = lpe<NF>() == 4 && CON;
  if constexpr (CON && QUADR) {
    // per env (a soft reset's re-forward and the acc_bad retry list no contacts), so divergent
    const bool listed = ccount != nullptr;
    // (RS) whether this env's rows fit a row-space layout; without a contact list the layouts hold
    // the NA frictionloss rows only, so an active limit row sends the wave to the v-form sweeps
    bool rs_lane = nlim == 0;
    if (listed) {
      // lane-split build (quad mode): every lane lists the env's contacts (pair, slot) in
      // pair order, then lane k of the quad builds contacts k, k+4, ... of the LDS records
      // and writes each into the quad's 4 columns; overflow contacts (rare) are built by
      // every lane (identical values in the env's slab)
      const int nw = (m.npair + 31) >> 5;
      // (RS) the contact categories of the RS layout (RsLayout) in list order: AT* CT* AC*, from the
      // pair words' body tables as the list is made (no per-contact pass over the list)
      bool rs_ok = true;
      int rs_stage = 0;
#pragma unroll
      for (int w = 0; w < PairMask::MAXW; w++) {  // unrolled: pm->w[] stays in registers
        uint32_t bits = w >= nw ? 0u : pm.w[w];
        const uint32_t warm = RS && w < nw ? m.pair_mw_arm[w] : 0u, wfree = RS && w < nw ? m.pair_mw_free[w] : 0u;
        while (bits) {
          const int b = __builtin_ctz(bits);
          const int p = 32 * w + b;
          bits &= bits - 1;
          const int cnt = pm.count_w(m, w, b);
          const int cat = (wfree >> b) & 1u ? ((warm >> b) & 1u ? 2 : 1) : 0;
          for (int k = 0; k < cnt; k++) {
            if (ncon >= SIM_MAXCON) {
              S.status |= SIM_ST_CONOVERFLOW;
              break;
            }
            L.ex(ncon) = __int_as_float(p << 3 | k);
            ncon++;
            if constexpr (RS) {
              rs_ok = rs_ok && cat >= rs_stage;
              rs_stage = cat;
              rs_nat += cat == 0, rs_nct += cat == 1, rs_nac += cat == 2;
            }
          }
        }
      }
      if constexpr (RS) {  // the contact categories of the RS layout (RsLayout): AT* CT* AC* in list order
        const bool ok = nlim == 0 && ncon <= LDS_CON && rs_ok;
        // the layouts instantiated: (KAT, KAC) = (0, 0) the cube resting alone, (1, 0) plus one
        // arm-only contact, (0, 1) plus one arm-cube contact, (1, 1) both, in one env or in two envs
        // of the wave (without it those waves -- ~1 launch in 10 over steps 20-120 -- took the v-form
        // sweeps at ~4x the wave time); other waves take the v-form sweeps
#ifdef SOARM_PHASE_PROF
        rs_why = (nlim > 0) | ((ncon > LDS_CON) << 1) | ((!ok && nlim == 0 && ncon <= LDS_CON) << 2) |
                 ((rs_nct > 4) << 3) | ((rs_nat > 1) << 4) | ((rs_nac > 1) << 5);
#endif
        rs_lane = ok && rs_nct <= 4 && rs_nat <= 1 && rs_nac <= 1;
      }
    }
    if constexpr (RS) {
      // one vote of the whole wave, taken with every lane active (outside the per-env branch): the
      // solve's dispatch on rs_fast is wave-uniform
      rs_fast = __all(rs_lane);
#ifdef SOARM_PHASE_PROF
      if (listed) rs_why |= (!rs_fast && rs_lane) << 6;  // an env that fits, in a wave with one that does not
#endif
    }
    if (listed) {
      auto build_listed = [&](int c, bool split) {
        const int pk = __float_as_int(L.ex(c));
        const int p = pk >> 3, k = pk & 7;
        const int s0 = m.pair_slot[p];
        float rw[7];
#pragma unroll
        for (int f = 0; f < 7; f++) rw[f] = soa(cbuf, (s0 + k) * 7 + f, n, e);
        float si[5];
#pragma unroll
        for (int q = 0; q < 5; q++) si[q] = m.pair_solimp[p][q];
        build_row(c, rw, m.pair_body1[p], m.pair_body2[p], S.fric >= 0.f ? S.fric : m.pair_friction[p],
                  m.pair_tran[p], m.pair_margin[p], m.pair_KB[p][0], m.pair_KB[p][1], si, split);
      };
      const int nlds = ncon < LDS_CON ? ncon : LDS_CON;
      constexpr int SPL = RS ? 16 : 4;  // the RS kernel: the env's 16 lanes split the build
      for (int c0 = 0; c0 < nlds; c0 += SPL) {
        const int c = c0 + (L.lane & (SPL - 1));
        if (c < nlds) build_listed(c, true);
      }
      wave_sync();  // the quad's records, written by its 4 lanes
      for (int c = LDS_CON; c < ncon; c++) build_listed(c, false);
    }
  } else if constexpr (CON) {
    if (ccount != nullptr) {
      const int nw = (m.npair + 31) >> 5;
#pragma unroll
      for (int w = 0; w < PairMask::MAXW; w++) {  // unrolled: pm->w[] stays in registers
        uint32_t bits = w >= nw ? 0u : pm.w[w];
        while (bits) {
          const int p = 32 * w + __builtin_ctz(bits);
          bits &= bits - 1;
          // everything this pair needs, loaded once and all in flight together: the count,
          // the pair's constants and every slot it may fill (cap <= PAIR_MAXCON; a set mask
          // bit means at least one contact, and slots past the count are never used)
          RP_MARK(3);
          const int cnt = pm.count(m, p);
          const int s0 = m.pair_slot[p], cap = m.pair_cap[p];
          const int b1 = m.pair_body1[p], b2 = m.pair_body2[p];
          const float mu = S.fric >= 0.f ? S.fric : m.pair_friction[p];
          const float tran = m.pair_tran[p], margin = m.pair_margin[p];
          const float KB0 = m.pair_KB[p][0], KB1 = m.pair_KB[p][1];
          float si[5];
#pragma unroll
          for (int q = 0; q < 5; q++) si[q] = m.pair_solimp[p][q];
          float raw[PAIR_MAXCON][7];
#pragma unroll
          for (int k = 0; k < PAIR_MAXCON; k++)
#pragma unroll
            for (int f = 0; f < 7; f++) raw[k][f] = k < cap ? soa(cbuf, (s0 + k) * 7 + f, n, e) : 0.f;
#pragma unroll
          for (int k = 0; k < PAIR_MAXCON; k++) {
            if (k >= cnt) break;
            if (ncon >= SIM_MAXCON) {
              S.status |= SIM_ST_CONOVERFLOW;
              break;
            }
            build_row(ncon, raw[k], b1, b2, mu, tran, margin, KB0, KB1, si, false);
            ncon++;
          }
        }
      }
    }
  }
  RP_MARK(3);
  RP_STORE;
  const int nl = ncon < LDS_CON ? ncon : LDS_CON;
  if constexpr (SOL == SIM_SOL_NEWTON) {  // MuJoCo's default solver on the same rows (soarm_newton.h)
    float fiR[NA];
#pragma unroll
    for (int i = 0; i < NA; i++) fiR[i] = 1.f / fR[i];
    const NewtonRows<NA, NF, CON> nr{m, L, cr, fR, fiR, fa, nlim, nl, ncon};
#ifdef SOARM_PHASE_PROF
    if (e < 65536) g_pgs_prof[8 * e + 6] = g_pgs_prof[8 * e + 7] = g_pgs_prof[8 * e] = clock64();
    PSTAMP(8);
    PSTAMP(9);  // (no separate warm-start phase: the solve below is stamp 9's phase and "pgs")
#endif
    const int nit = newton_solve(S, nr);
#ifdef SOARM_PHASE_PROF
    if (e < 65536)
      g_pgs_prof[8 * e + 1] = clock64(), g_pgs_prof[8 * e + 2] = nit, g_pgs_prof[8 * e + 3] = 0,
                        g_pgs_prof[8 * e + 4] = nlim, g_pgs_prof[8 * e + 5] = ncon;
#else
    (void)nit;
#endif
    return ncon;
  }
#ifdef SOARM_PHASE_PROF
  if (e < 65536) g_pgs_prof[8 * e + 6] = clock64();  // rows built
  PSTAMP(8);
#endif

  // ---- warm start from qacc_warmstart (forces implied by the primal), keep if it beats f = 0
  // (a wave on the RS solve makes its warm start in row space instead, rs_solve)
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
  if (!(RS && rs_fast)) {
#pragma unroll
  for (int i = 0; i < NA; i++) {
    const float fl = m.dof_frictionloss[i];
    const float jar = S.warm[i] - fa[i];
    const float fs = (jar <= -fl * fR[i]) ? fl : (jar >= fl * fR[i]) ? -fl : -jar / fR[i];
    ff[i] = fl > 0.f ? fs : 0.f;
#pragma unroll
    for (int k = 0; k < NA; k++) v[k] += Mi.a(i, k) * ff[i];
  }
  for (int l = 0; l < nlim; l++) {
    float oh[NA];
    one_hot<NA>((int)L.lm(l, L_DOF), oh);
    const float sg = L.lm(l, L_SGN);
    const float jar = sg * pick<NA>(S.warm, oh) - L.lm(l, L_AREF);
    const float fs = jar < 0.f ? -jar / L.lm(l, L_R) : 0.f;
    L.lm(l, L_FRC) = fs;
    add_arm_col(Mi, v, oh, sg * fs);
  }
  // contacts (Gram form: J_e x = J_n x + s J_tk x; one M^-1 product per contact); quad mode:
  // lane k takes contacts k, k+4, ... and the quad sums the velocity changes
  float vw[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) vw[i] = 0.f;
  // (the RS kernel: the env's 16 lanes split the contacts, one each)
  const int cstep = RS ? 16 : QUADR ? 4 : 1, cfirst = RS ? (L.lane & 15) : QUADR ? (L.lane & 3) : 0;
  auto env_sum = [&](float x) { return RS ? rowsum16(x) : QUADR ? qsum(x) : x; };
  for (int c = cfirst; c < nl; c += cstep) {
    float jn[NV], jt1[NV], jt2[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) jn[i] = L.at(c, i), jt1[i] = L.at(c, 12 + i), jt2[i] = L.at(c, 24 + i);
    const float mu = L.at(c, F_MU), Rp = L.at(c, F_R);
    float jw[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NV; i++) jw[0] += jn[i] * S.warm[i], jw[1] += jt1[i] * S.warm[i], jw[2] += jt2[i] * S.warm[i];
    float fs[4];
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      const float s = (ed & 1) ? -mu : mu;
      const float jar = jw[0] + s * jw[1 + (ed >> 1)] - L.at(c, F_AREF + ed);
      fs[ed] = jar < 0.f ? -jar / Rp : 0.f;
      wrec(c, F_FRC + ed, fs[ed], QUADR);
    }
    const float Dn = (fs[0] + fs[1]) + (fs[2] + fs[3]), D1 = mu * (fs[0] - fs[1]), D2 = mu * (fs[2] - fs[3]);
    float u[NV], w[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) u[i] = jn[i] * Dn + jt1[i] * D1 + jt2[i] * D2;
    Mi.mul(u, w, true, true);
#pragma unroll
    for (int i = 0; i < NV; i++) vw[i] += w[i];
  }
#pragma unroll
  for (int i = 0; i < NV; i++) v[i] += env_sum(vw[i]);
  for (int c = nl; c < ncon; c++)
    for (int ed = 0; ed < 4; ed++) {
      const int r = 4 * c + ed;
      float jar = -cr.S(r, 0);
#pragma unroll
      for (int i = 0; i < NV; i++) jar += cr.J(r, i) * S.warm[i];
      const float fs = jar < 0.f ? -jar / cr.S(r, 1) : 0.f;
      cr.S(r, 3) = fs;
#pragma unroll
      for (int i = 0; i < NV; i++) v[i] += cr.W(r, i) * fs;
    }
  // dual cost of the warm start: sum_r 0.5 f_r (J_r v - aref_r + R_r f_r) + 0.5 f_r (J_r qacc_smooth - aref_r)
  float cost = 0.f;
#pragma unroll
  for (int i = 0; i < NA; i++)
    cost += 0.5f * ff[i] * (v[i] - fa[i] + fR[i] * ff[i]) + 0.5f * ff[i] * (S.qacc_s[i] - fa[i]);
  for (int l = 0; l < nlim; l++) {
    float oh[NA];
    one_hot<NA>((int)L.lm(l, L_DOF), oh);
    const float sg = L.lm(l, L_SGN), f = L.lm(l, L_FRC), ar = L.lm(l, L_AREF);
    cost += 0.5f * f * (sg * pick<NA>(v, oh) - ar + L.lm(l, L_R) * f) + 0.5f * f * (sg * pick<NA>(S.qacc_s, oh) - ar);
  }
  float ccost = 0.f;  // contacts' share (quad mode: lane k's contacts, summed over the quad)
  for (int c = cfirst; c < nl; c += cstep) {
    float jn[NV], jt1[NV], jt2[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) jn[i] = L.at(c, i), jt1[i] = L.at(c, 12 + i), jt2[i] = L.at(c, 24 + i);
    const float mu = L.at(c, F_MU), Rp = L.at(c, F_R);
    float jv[3] = {0.f, 0.f, 0.f}, jq[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NV; i++) {
      jv[0] += jn[i] * v[i], jv[1] += jt1[i] * v[i], jv[2] += jt2[i] * v[i];
      jq[0] += jn[i] * S.qacc_s[i], jq[1] += jt1[i] * S.qacc_s[i], jq[2] += jt2[i] * S.qacc_s[i];
    }
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      const float s = (ed & 1) ? -mu : mu;
      const float fr = L.at(c, F_FRC + ed), ar = L.at(c, F_AREF + ed);
      ccost += 0.5f * fr * (jv[0] + s * jv[1 + (ed >> 1)] - ar + Rp * fr) +
               0.5f * fr * (jq[0] + s * jq[1 + (ed >> 1)] - ar);
    }
  }
  cost += env_sum(ccost);
  if constexpr (QUADR) wave_sync();  // F_FRC of the quad's contacts, written by their lanes
  for (int c = nl; c < ncon; c++)
    for (int ed = 0; ed < 4; ed++) {
      const int r = 4 * c + ed;
      float jv = 0.f, jq = 0.f;
#pragma unroll
      for (int i = 0; i < NV; i++) {
        jv += cr.J(r, i) * v[i];
        jq += cr.J(r, i) * S.qacc_s[i];
      }
      const float fr = cr.S(r, 3), ar = cr.S(r, 0);
      cost += 0.5f * fr * (jv - ar + cr.S(r, 1) * fr) + 0.5f * fr * (jq - ar);
    }
  if (cost > 0.f) {
#pragma unroll
    for (int i = 0; i < NA; i++) ff[i] = 0.f;
    for (int l = 0; l < nlim; l++) L.lm(l, L_FRC) = 0.f;
    for (int c = 0; c < nl; c++)
#pragma unroll
      for (int ed = 0; ed < 4; ed++) L.at(c, F_FRC + ed) = 0.f;
    for (int r = 4 * nl; r < 4 * ncon; r++) cr.S(r, 3) = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = S.qacc_s[i];
  }
  }

#ifdef SOARM_PHASE_PROF
  if (e < 65536) g_pgs_prof[8 * e + 7] = clock64();  // warm start + cost done
#endif
  // ---- projected Gauss-Seidel sweeps (mj_solPGS's improvement criterion, scaled by the model
  // constant 1 / (meaninertia * max(1, nv)), meaninertia = trace(M(qpos0)) / nv)
  const float scale = m.pgs_scale;
  if constexpr (RS) {  // the RS kernel: the damped Euler step's factor instead (Sim::damp_factor)
    S.damp_factor();
    int k = 0;
#pragma unroll
    for (int i = 0; i < NA * (NA + 1) / 2; i++) L.kp(k++) = S.LH[i];
#pragma unroll
    for (int i = 0; i < NA; i++) L.kp(k++) = S.DHi[i];
#pragma unroll
    for (int i = 0; i < 6 * NF; i++) L.kp(k++) = S.kf[i / 6][i % 6];
#pragma unroll
    for (int i = 0; i < 3; i++) L.kp(k++) = S.ee[i];
  } else if (L.keep) {  // park what only the post-solve stages need (restored below)
    int k = 0;
#pragma unroll
    for (int i = 0; i < NA * (NA + 1) / 2; i++) L.kp(k++) = S.MA[i];
#pragma unroll
    for (int f2 = 0; f2 < NF; f2++)
#pragma unroll
      for (int i = 0; i < 6; i++) L.kp(k++) = S.MF[f2][i * (i + 1) / 2 + i];
#pragma unroll
    for (int i = 0; i < NV; i++) L.kp(k++) = S.fsmooth[i];
#pragma unroll
    for (int i = 0; i < 3; i++) L.kp(k++) = S.ee[i];
  }
#ifdef SOARM_PHASE_PROF
  if (e < 65536) g_pgs_prof[8 * e] = clock64();
  PSTAMP(9);
  int nsweep = m.iterations, armstop = 0;
#endif
  // dof-frictionloss rows (J = e_i): one pass.  Branch-free: a dof with frictionloss 0
  // (no row in MuJoCo) clamps to [0, 0] and stays an exact no-op.
  auto fric_rows = [&](float& improvement) {
#pragma unroll
    for (int i = 0; i < NA; i++) {
      const float fl = m.dof_frictionloss[i];
      const float res = v[i] - fa[i] + fR[i] * ff[i];
      const float fn = fminf(fmaxf(ff[i] - res * fiD[i], -fl), fl);
      const float df = fn - ff[i];
#pragma unroll
      for (int k = 0; k < NA; k++) v[k] += Mi.a(i, k) * df;
      ff[i] = fn;
      improvement -= df * (res + fhD[i] * df);
    }
  };
  // active joint-limit rows (LDS list; usually empty)
  auto limit_rows = [&](float& improvement) {
    for (int l = 0; l < nlim; l++) {
      float oh[NA];
      one_hot<NA>((int)L.lm(l, L_DOF), oh);
      const float sg = L.lm(l, L_SGN), fo = L.lm(l, L_FRC);
      const float res = sg * pick<NA>(v, oh) - L.lm(l, L_AREF) + L.lm(l, L_R) * fo;
      const float fn = fmaxf(fo - res * L.lm(l, L_IARD), 0.f);
      const float df = fn - fo;
      add_arm_col(Mi, v, oh, sg * df);
      L.lm(l, L_FRC) = fn;
      improvement -= df * (res + 0.5f * L.lm(l, L_ARD) * df);
    }
  };
  // arm-only contact c: NA-dof dots, the 4-edge chain, one arm-block M^-1 product
  auto arm_v = [&](int c, float mu, float Rp, const float* cf, float* fo, const float* ar, const float* ia,
                   const float* hd, float& improvement) {
    float jn[NA], j1[NA], j2[NA];
#pragma unroll
    for (int i = 0; i < NA; i++) jn[i] = L.at(c, i), j1[i] = L.at(c, 12 + i), j2[i] = L.at(c, 24 + i);
    float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
    for (int i = 0; i < NA; i++) a += jn[i] * v[i], b += j1[i] * v[i], cc += j2[i] * v[i];
    float df[4];
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      const float s = (ed & 1) ? -mu : mu;
      const float res = (a + s * ((ed >> 1) ? cc : b)) - ar[ed] + Rp * fo[ed];
      const float fnew = fmaxf(fo[ed] - res * ia[ed], 0.f);
      df[ed] = fnew - fo[ed];
      a += cf[3 * ed] * df[ed];
      b += cf[3 * ed + 1] * df[ed];
      cc += cf[3 * ed + 2] * df[ed];
      improvement -= df[ed] * (res + hd[ed] * df[ed]);
      fo[ed] = fnew;
    }
    const float Dn = (df[0] + df[1]) + (df[2] + df[3]);
    const float D1 = mu * (df[0] - df[1]), D2 = mu * (df[2] - df[3]);
    float u[NA];
#pragma unroll
    for (int i = 0; i < NA; i++) u[i] = jn[i] * Dn + j1[i] * D1 + j2[i] * D2;
#pragma unroll
    for (int i = 0; i < NA; i++) {
      float w = 0.f;
#pragma unroll
      for (int k = 0; k < NA; k++) w += Mi.a(i, k) * u[k];
      v[i] += w;
    }
#pragma unroll
    for (int ed = 0; ed < 4; ed++) L.at(c, F_FRC + ed) = fo[ed];
  };
  // contact c from its LDS record, in Gram form: a 6-dof free-body update when
  // (wave-uniformly) it touches only the free body, otherwise full-width dots and one
  // M^-1 product per sweep for the velocity update
  auto lds_contact = [&](int c, float& improvement) {
    const bool ta = (int)L.at(c, F_FLAGS) & TOUCH_ARM;
    float G[6], cf[12], fo[4], ar[4], ia[4], hd[4];
#pragma unroll
    for (int ed = 0; ed < 4; ed++)
      fo[ed] = L.at(c, F_FRC + ed), ar[ed] = L.at(c, F_AREF + ed), ia[ed] = L.at(c, F_IARD + ed),
      hd[ed] = L.at(c, F_HARD + ed);
#pragma unroll
    for (int k = 0; k < 6; k++) G[k] = L.at(c, F_GRAM + k);
    const float mu = L.at(c, F_MU), Rp = L.at(c, F_R);
    gram_coefs(G, mu, cf);
    if constexpr (NF == 1) {
      if (__all(!ta)) {
        float jn[6], j1[6], j2[6];
#pragma unroll
        for (int i = 0; i < 6; i++)
          jn[i] = L.at(c, NA + i), j1[i] = L.at(c, 12 + NA + i), j2[i] = L.at(c, 24 + NA + i);
        gram_step(v + NA, jn, j1, j2, cf, ar, ia, hd, fo, mu, Rp, Mi.Fd[0], improvement);
#pragma unroll
        for (int ed = 0; ed < 4; ed++) L.at(c, F_FRC + ed) = fo[ed];
        return;
      }
    }
    if (__all(!((int)L.at(c, F_FLAGS) & TOUCH_FREE))) {
      // arm-only contact (link vs table / floor / link): NA-dof dots, one arm-block
      // M^-1 product per sweep
      arm_v(c, mu, Rp, cf, fo, ar, ia, hd, improvement);
      return;
    }
    // the record holds zeros in the halves the contact does not touch: full-width,
    // branch-free dots (divergent half-selection would run both sides anyway)
    float jn[NV], j1[NV], j2[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) jn[i] = L.at(c, i), j1[i] = L.at(c, 12 + i), j2[i] = L.at(c, 24 + i);
    float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) a += jn[i] * v[i], b += j1[i] * v[i], cc += j2[i] * v[i];
    float df[4];
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      const float s = (ed & 1) ? -mu : mu;
      const float res = (a + s * ((ed >> 1) ? cc : b)) - ar[ed] + Rp * fo[ed];
      const float fnew = fmaxf(fo[ed] - res * ia[ed], 0.f);
      df[ed] = fnew - fo[ed];
      a += cf[3 * ed] * df[ed];
      b += cf[3 * ed + 1] * df[ed];
      cc += cf[3 * ed + 2] * df[ed];
      improvement -= df[ed] * (res + hd[ed] * df[ed]);
      fo[ed] = fnew;
    }
    const float Dn = (df[0] + df[1]) + (df[2] + df[3]);
    const float D1 = mu * (df[0] - df[1]), D2 = mu * (df[2] - df[3]);
    float u[NV], w[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) u[i] = jn[i] * Dn + j1[i] * D1 + j2[i] * D2;
    Mi.mul(u, w, true, true);
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] += w[i];
#pragma unroll
    for (int ed = 0; ed < 4; ed++) L.at(c, F_FRC + ed) = fo[ed];
  };
  // contacts beyond LDS_CON: per-edge J/W rows in global scratch (rare)
  auto scratch_rows = [&](float& improvement) {
    for (int r = 4 * nl; r < 4 * ncon; r++) {
      float res = -cr.S(r, 0) + cr.S(r, 1) * cr.S(r, 3);
#pragma unroll
      for (int i = 0; i < NV; i++) res += cr.J(r, i) * v[i];
      const float fo = cr.S(r, 3);
      const float fnew = fmaxf(fo - res / cr.S(r, 2), 0.f);
      const float df = fnew - fo;
      if (df != 0.f) {
#pragma unroll
        for (int i = 0; i < NV; i++) v[i] += cr.W(r, i) * df;
        cr.S(r, 3) = fnew;
        improvement -= df * res + 0.5f * cr.S(r, 2) * df * df;
      }
    }
  };

  // Register block: the first run of up to FC consecutive contacts that touch only
  // the free body (the cube's box-box contacts with the table) keeps all its row data
  // in registers for the whole solve, so the common sweep is straight-line code in
  // which the arm's friction chain and the cube's contact chain (independent: M is
  // block diagonal) interleave.  Contacts before / after the run go through their
  // LDS records in row order.  Slots beyond the run are zero rows (1/ARdiag = 0).
  constexpr int FC = (NF == 1 && CON) ? 4 : 1;
  int c0 = nl, nrun = 0;
  if constexpr (NF == 1 && CON) {
    for (int c = 0; c < nl; c++)
      if ((int)L.at(c, F_FLAGS) == TOUCH_FREE) {
        c0 = c;
        break;
      }
    while (nrun < FC && c0 + nrun < nl && (int)L.at(c0 + nrun, F_FLAGS) == TOUCH_FREE) nrun++;
  }
  // registers: the block's forces (updated every sweep) and Gram columns; the rest is
  // re-read from LDS each sweep — those loads are independent of the Gauss-Seidel
  // chains, so in straight-line code they issue ahead of use
  if constexpr (CON) {
#pragma unroll
    for (int f = 0; f < CF; f++) L.at(LDS_CON, f) = 0.f;  // the all-zero record (absent rows)
  }
  float cfo[FC][4], ccf[FC][12];
  int cslot[FC];
  if (NF == 1 && CON && !rs_fast) {
#pragma unroll
    for (int k = 0; k < FC; k++) {
      const bool on = k < nrun;
      cslot[k] = on ? c0 + k : LDS_CON;
#pragma unroll
      for (int ed = 0; ed < 4; ed++) cfo[k][ed] = on ? L.at(c0 + k, F_FRC + ed) : 0.f;
      float G[6];
#pragma unroll
      for (int i = 0; i < 6; i++) G[i] = L.at(cslot[k], F_GRAM + i);
      gram_coefs(G, L.at(cslot[k], F_MU), ccf[k]);
    }
  }
  const int c1 = c0 + nrun;
  // Contacts before the block that do not touch the free body commute with the block's
  // rows (disjoint dofs, block-diagonal M), so they may run after it: then one masked
  // loop covers every lane's non-block contacts (e.g. an arm-table contact, which
  // precedes the cube's rows in pair order, in one lane and an arm-cube contact, which
  // follows them, in another) instead of one loop before and one after the block.
  int npre = 0;
  for (int c = 0; c < c0; c++)
    if ((int)L.at(c, F_FLAGS) & TOUCH_FREE) npre = c0;
  const int npost = (c0 - npre) + (nl - c1);
#ifdef SOARM_PHASE_PROF
  bool npost_free = false;  // a non-block contact touches the free body
  int nfree_x = 0;
  for (int c = 0; c < nl; c++)
    if ((c < c0 || c >= c1) && ((int)L.at(c, F_FLAGS) & TOUCH_FREE)) npost_free = true, nfree_x++;
#endif
  // the block's sweep (straight-line: one basic block with the friction rows)
  auto block_rows = [&](float& improvement) {
    if constexpr (NF == 1 && CON) {
#pragma unroll
      for (int k = 0; k < FC; k++) {
        const int c = cslot[k];
        float jn[6], j1[6], j2[6], ar[4], ia[4], hd[4];
#pragma unroll
        for (int i = 0; i < 6; i++)
          jn[i] = L.at(c, NA + i), j1[i] = L.at(c, 12 + NA + i), j2[i] = L.at(c, 24 + NA + i);
#pragma unroll
        for (int ed = 0; ed < 4; ed++)
          ar[ed] = L.at(c, F_AREF + ed), ia[ed] = L.at(c, F_IARD + ed), hd[ed] = L.at(c, F_HARD + ed);
        const float mu = L.at(c, F_MU), Rp = L.at(c, F_R);
        gram_step(v + NA, jn, j1, j2, ccf[k], ar, ia, hd, cfo[k], mu, Rp, Mi.Fd[0], improvement);
      }
    }
  };
  // When no lane has a pre-block contact on the free body (always, for pair-ordered
  // scenes where the cube's world contacts come first), the block commutes with every
  // arm row before it: run it beside the friction rows so the two independent chains
  // share one straight-line region, then limits and the remaining contacts.
  const bool block_first = __all(npre == 0);
  // The single non-block contact of a lane (when it has one): an arm-only contact before
  // the block commutes with it (disjoint dofs), so it runs after the block, right where
  // the post-block ones run (lanes without one use the zero record).
  const int ca = npost == 1 ? (c0 - npre > 0 ? npre : c1) : LDS_CON;
  auto xidx = [&](int j) { return j < c0 - npre ? npre + j : c1 + j - (c0 - npre); };  // j-th non-block contact
  // ---- contact-space ("y") sweep of the register block, used when nothing else in the
  // wave touches the free body (every lane: no limits, no overflow rows, no non-block
  // contact other than at most one arm-only one).  Each block contact k keeps
  // y_k = (J_n v, J_t1 v, J_t2 v) of the free body's velocity, shifted by its reference
  // acceleration: a pyramid edge's aref is affine in the same directions,
  // aref_e = alpha + s_e beta_k (s_e = +-mu), so res_e = (a - alpha) + s_e (t_k - beta_k)
  // + R f_e.  A force step on contact j moves every other y_k by the 3x3 cross-Gram
  // block J_k M^-1 J_j' (the free block of M is diagonal, host-validated) — 27 FMAs per
  // contact instead of the three 6-dof dots and the 6-dof velocity update of the v form;
  // the velocity is rebuilt once from the force change after the sweeps.  Same
  // Gauss-Seidel sequence (MuJoCo's mj_solPGS row order) in exact arithmetic.
  // Extra contact slot E of the y variants (every lane: at most one non-block contact,
  // no limits, no overflow, at most 5 contacts): an arm-only contact, or one that touches
  // the arm and the free body ("coupled"), or the zero record.  Its y_E lives in registers;
  // its coefficients live in the LDS of records 5-6 (unused when no lane has more than 5
  // contacts): W_E = M_arm^-1 J_E,arm' (how a force step on E moves v_arm, and how a
  // frictionloss row moves y_E), the free-body cross-Gram blocks X_kE = J_k M^-1 J_E' with
  // the block contacts, the off-diagonal edge Gram, the 3x3 Gram, 1/ARdiag, ARdiag/2, mu, R.
  // Scratch of the extra slots (compile-time indices): the joint-limit list (no limit is
  // active in the y variants) and an array of its own.
  enum { E_W = 0, E_X = 18, E_A = 54, E_G = 60, E_IA = 66, E_HD = 70, E_MU = 74, E_RP = 75 };
  // second extra slot F (an arm-only contact before E in row order), v-form on the arm:
  // J_arm rows, W_F = M_arm^-1 J_F', edge Gram, 1/ARd, ARd/2, mu, R, aref shift, X_EF = J_E M^-1 J_F'
  enum { F_J = 76, F_W = 94, F_A = 112, F_IA = 118, F_HD = 122, F_MUX = 126, F_RPX = 127, F_SH = 128, F_XE = 131,
         XS_END = 140 };
  static_assert(XS_END <= NA * LF + XS_EXT - XS_LIST, "extra-slot scratch fits");
  auto EX = [&](int k) -> float& { return k < NA * LF ? L.lraw(k) : L.ex(XS_LIST + k - NA * LF); };
  float yE[3] = {0.f, 0.f, 0.f}, fE[4] = {0.f, 0.f, 0.f, 0.f}, fF[4] = {0.f, 0.f, 0.f, 0.f};
  // quad mode: the E/F coefficients preloaded into registers before the sweeps, in the
  // register pairs the packed loop consumes (no memory reads inside the sweep loop)
  struct ExtQ {
    float muo, eA10, eA32, fA10, fA32, eMu, eRp, fMu, fRp, fJ2[6], fX2[3], eG2[3], xo[9], fSh2;
    f2 eNia01, eNia23, fNia01, fNia23, eWp[9], eA2030, eA2131, fA2030, fA2131, eHD01, eHD23, fHD01, fHD23, fJp[6], fWp[9], fXp[3], eGp[3], qe01[3], qe23[3], fSh01;
  } xq;
  constexpr int NX = FC * (FC - 1) / 2;
  float yb[FC][3], xg[NX > 0 ? NX : 1][9];
  constexpr bool QUAD = lpe<NF>() == 4 && NF == 1 && CON && FC == 4;
  const int sub = QUAD ? (L.lane & 3) : 0;
  // quad mode: this lane's block contact (sub) — its y and its cross-Gram row X_sub,j
  // (j = sub: the contact's own 3x3 Gram block), full 3x3 per j
  float yo[3] = {0.f, 0.f, 0.f}, xr[QUAD ? FC : 1][9];
  // quad mode, packed: this lane's contact's 4 edge residuals r_e = y_0 + s_e y_t(e) + R f_e
  // (pairs (r0, r1), (r2, r3)), held scaled by -1/ARdiag_e (see sA10 below); the sweep
  // broadcasts them instead of y
  f2 ro01 = f2{0.f, 0.f}, ro23 = f2{0.f, 0.f};
  // rows of the arm block of M^-1 as dof pairs (packed v_arm updates of the friction rows)
  f2 Mp[NA][NA / 2];
  auto ypair = [](int j, int k) { return j * FC - j * (j + 1) / 2 + (k - j - 1); };  // j < k
  auto yblock_setup = [&]() {
    if constexpr (NF == 1 && CON) {
#pragma unroll
      for (int k = 0; k < FC; k++) {
        const int c = cslot[k];
        float ar[4];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) ar[ed] = L.at(c, F_AREF + ed);
        const float mu = L.at(c, F_MU);
        const float sh[3] = {0.5f * (ar[0] + ar[1]), mu > 0.f ? 0.5f * (ar[0] - ar[1]) / mu : 0.f,
                             mu > 0.f ? 0.5f * (ar[2] - ar[3]) / mu : 0.f};
#pragma unroll
        for (int q = 0; q < 3; q++) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < 6; i++) s = fmaf(L.at(c, 12 * q + NA + i), v[NA + i], s);
          yb[k][q] = s - sh[q];
        }
      }
      // cross-Gram blocks, one pair at a time (rows re-read from LDS: setup only)
#pragma unroll
      for (int j = 0; j < FC; j++)
#pragma unroll
        for (int k = j + 1; k < FC; k++) {
          float wk[3][6];
#pragma unroll
          for (int q = 0; q < 3; q++)
#pragma unroll
            for (int i = 0; i < 6; i++) wk[q][i] = Mi.Fd[0][i] * L.at(cslot[k], 12 * q + NA + i);
#pragma unroll
          for (int r = 0; r < 3; r++) {
            float jj[6];
#pragma unroll
            for (int i = 0; i < 6; i++) jj[i] = L.at(cslot[j], 12 * r + NA + i);
#pragma unroll
            for (int cc = 0; cc < 3; cc++) {
              float s = 0.f;
#pragma unroll
              for (int i = 0; i < 6; i++) s = fmaf(jj[i], wk[cc][i], s);
              xg[ypair(j, k)][3 * r + cc] = s;  // J_j[r] M^-1 J_k[cc]'
            }
          }
        }
      if constexpr (QUAD) {
#pragma unroll
        for (int q = 0; q < 3; q++) yo[q] = sub == 0 ? yb[0][q] : sub == 1 ? yb[1][q] : sub == 2 ? yb[2][q] : yb[3][q];
#pragma unroll
        for (int j = 0; j < FC; j++)
#pragma unroll
          for (int r = 0; r < 3; r++)
#pragma unroll
            for (int q = 0; q < 3; q++) {
              float cand[FC];
#pragma unroll
              for (int k = 0; k < FC; k++) {
                if (k == j) {  // own Gram block, symmetric packed (nn, n1, n2, 11, 12, 22)
                  const int lo = r < q ? r : q, hi = r < q ? q : r;
                  const int gi = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
                  cand[k] = L.at(cslot[k], F_GRAM + gi);
                } else {
                  cand[k] = k < j ? xg[ypair(k, j)][3 * r + q] : xg[ypair(j, k)][3 * q + r];
                }
              }
              xr[j][3 * r + q] = sub == 0 ? cand[0] : sub == 1 ? cand[1] : sub == 2 ? cand[2] : cand[3];
            }
      }
    }
  };
  // per-sweep constants of the block in registers: 1/ARdiag, ARdiag/2, mu, R, the
  // off-diagonal edge-Gram entries A_ed = J_e M^-1 J_d' (d < e) and the 3x3 Gram block
  float yia[FC][4], yhd[FC][4], ymu[FC], yRp[FC], yA[FC][6], yG[FC][6];
  // quad mode, packed: edge-Gram pairs (A20, A30), (A21, A31), ARdiag/2 pairs, and the own
  // residuals' update per edge of contact j: C_e'e = (1, s'_e' on t(e')) X_sub,j (1, s_e on
  // t(e)) + R delta (own contact), as pairs over e': r_own += C_.e df_e
  f2 qA2030[FC], qA2131[FC], qhd01[FC], qhd23[FC], C01[QUAD ? FC : 1][4], C23[QUAD ? FC : 1][4];
  // quad mode, packed: the residuals are carried scaled, s_e = -r_e / ARdiag_e, so the projected
  // step is df = max(s_e, -f_e) with no multiply on the chain; the edge-Gram entries that move
  // a later edge e' are pre-scaled by -1/ARdiag_e' (sA10 = -A10/ARdiag1, sA32, qA2030, qA2131)
  float sA10[FC], sA32[FC];
  // this lane's own block contact (quad mode): -1/ARdiag of its 4 edges as pairs
  auto own_nia01 = [&]() {
    return f2{-(sub == 0 ? yia[0][0] : sub == 1 ? yia[1][0] : sub == 2 ? yia[2][0] : yia[3][0]),
              -(sub == 0 ? yia[0][1] : sub == 1 ? yia[1][1] : sub == 2 ? yia[2][1] : yia[3][1])};
  };
  auto own_nia23 = [&]() {
    return f2{-(sub == 0 ? yia[0][2] : sub == 1 ? yia[1][2] : sub == 2 ? yia[2][2] : yia[3][2]),
              -(sub == 0 ? yia[0][3] : sub == 1 ? yia[1][3] : sub == 2 ? yia[2][3] : yia[3][3])};
  };
  auto yblock_consts = [&](auto pk) {
    if constexpr (NF == 1 && CON) {
#pragma unroll
      for (int k = 0; k < FC; k++) {
        const int c = cslot[k];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) yia[k][ed] = L.at(c, F_IARD + ed), yhd[k][ed] = L.at(c, F_HARD + ed);
        ymu[k] = L.at(c, F_MU), yRp[k] = L.at(c, F_R);
        float G[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
          G[i] = L.at(c, F_GRAM + i);
          if constexpr (!QUAD) yG[k][i] = G[i];  // quad mode: the own block sits in xr
        }
        // edge e = J_n + s_e J_t(e): s = +mu, -mu, +mu, -mu; t = 1, 1, 2, 2
        const float mu = ymu[k];
        auto gt = [&](int e) { return (e >> 1) ? G[2] : G[1]; };                  // G_n,t(e)
        auto gtt = [&](int e, int d) {                                          // G_t(e),t(d)
          const int te = e >> 1, td = d >> 1;
          return te == td ? (te ? G[5] : G[3]) : G[4];
        };
        auto sg = [&](int e) { return (e & 1) ? -mu : mu; };
        int q = 0;
#pragma unroll
        for (int ed = 1; ed < 4; ed++)
#pragma unroll
          for (int d = 0; d < ed; d++)
            yA[k][q++] = G[0] + sg(ed) * gt(ed) + sg(d) * gt(d) + sg(ed) * sg(d) * gtt(ed, d);
        if constexpr (QUAD && decltype(pk)::value) {
          sA10[k] = -yia[k][1] * yA[k][0], sA32[k] = -yia[k][3] * yA[k][5];
          qA2030[k] = f2{-yia[k][2] * yA[k][1], -yia[k][3] * yA[k][3]};
          qA2131[k] = f2{-yia[k][2] * yA[k][2], -yia[k][3] * yA[k][4]};
          qhd01[k] = f2{yhd[k][0], yhd[k][1]}, qhd23[k] = f2{yhd[k][2], yhd[k][3]};
        }
      }
      if constexpr (QUAD && decltype(pk)::value) {
        // own contact (sub): mu, R, forces; its residuals from y; the folded coefficients
        const float muo = sub == 0 ? ymu[0] : sub == 1 ? ymu[1] : sub == 2 ? ymu[2] : ymu[3];
        const float Rpo = sub == 0 ? yRp[0] : sub == 1 ? yRp[1] : sub == 2 ? yRp[2] : yRp[3];
        float fo[4];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) fo[ed] = sub == 0 ? cfo[0][ed] : sub == 1 ? cfo[1][ed] : sub == 2 ? cfo[2][ed] : cfo[3][ed];
        ro01 = f2{fmaf(Rpo, fo[0], fmaf(muo, yo[1], yo[0])), fmaf(Rpo, fo[1], fmaf(-muo, yo[1], yo[0]))};
        ro23 = f2{fmaf(Rpo, fo[2], fmaf(muo, yo[2], yo[0])), fmaf(Rpo, fo[3], fmaf(-muo, yo[2], yo[0]))};
        const f2 nio01 = own_nia01(), nio23 = own_nia23();
        ro01 = ro01 * nio01, ro23 = ro23 * nio23;  // scaled: s_e = -r_e / ARdiag_e
#pragma unroll
        for (int k = 0; k < FC; k++) {
          const float mu = ymu[k];
#pragma unroll
          for (int ed = 0; ed < 4; ed++) {
            const int t = 1 + (ed >> 1);
            const float se = (ed & 1) ? -mu : mu;
            // y_own moves by K = X_sub,k (1, s_e on t(e)) per unit step of edge ed of contact k
            const float K[3] = {fmaf(se, xr[k][t], xr[k][0]), fmaf(se, xr[k][3 + t], xr[k][3]),
                                fmaf(se, xr[k][6 + t], xr[k][6])};
            float c[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; e2++) {
              const float so = (e2 & 1) ? -muo : muo;
              c[e2] = fmaf(so, K[1 + (e2 >> 1)], K[0]) + ((k == sub && e2 == ed) ? Rpo : 0.f);
            }
            C01[k][ed] = f2{c[0], c[1]} * nio01, C23[k][ed] = f2{c[2], c[3]} * nio23;
          }
        }
      }
    }
  };
  // One sweep over the block.  Per contact the 4 edges are a 4x4 Gauss-Seidel on the
  // edge Gram matrix: every residual starts from the contact's y, and each force step
  // adds A_ed df_d to the later edges' residuals, so the dependent chain per edge is
  // mul -> max -> fma (df = max(-res/ARdiag, -f) is the projected step f' - f).
  auto yblock_contact = [&](const int j, float& improvement, f2& impq, float (&dsel)[4], auto coupled, auto pk) {
    if constexpr (QUAD && decltype(pk)::value) {  // packed residual form; contact j's residuals live in lane j
      const f2 c01 = f2{cfo[j][0], cfo[j][1]}, c23 = f2{cfo[j][2], cfo[j][3]};
      const f2 s01 = f2{qbcast(ro01.x, j), qbcast(ro01.y, j)};  // scaled residuals of contact j
      f2 s23 = f2{qbcast(ro23.x, j), qbcast(ro23.y, j)};
      // the steps are built in their pairs d01, d23 and splatted from a pair half (op_sel),
      // so no register copy sits between a step and the packed updates that consume it
      f2 d01, d23;
      d01.x = max_neg(s01.x, c01.x);
      const float s1 = fmaf(sA10[j], d01.x, s01.y);
      s23 = fma2(qA2030[j], d01.xx, s23);
      d01.y = max_neg(s1, c01.y);
      const f2 s23b = fma2_hi(qA2131[j], d01, s23);
      d23.x = max_neg(s23b.x, c23.x);
      const float s3 = fmaf(sA32[j], d23.x, s23b.y);
      d23.y = max_neg(s3, c23.y);
      const f2 n01 = c01 + d01, n23 = c23 + d23;
      cfo[j][0] = n01.x, cfo[j][1] = n01.y, cfo[j][2] = n23.x, cfo[j][3] = n23.y;
      // improvement -df (r + ARdiag df / 2) with r = -ARdiag s = -2 hd s: -(hd df)(df - 2 s)
      impq = fma2(-(qhd01[j] * d01), fma2(f2{s01.x, s1}, splat2(-2.f), d01), impq);
      impq = fma2(-(qhd23[j] * d23), fma2(f2{s23b.x, s3}, splat2(-2.f), d23), impq);
      const float dfs[4] = {d01.x, d01.y, d23.x, d23.y};
      // this lane's residuals take the 4 steps
      ro01 = fma2(C01[j][0], d01.xx, ro01), ro23 = fma2(C23[j][0], d01.xx, ro23);
      ro01 = fma2_hi(C01[j][1], d01, ro01), ro23 = fma2_hi(C23[j][1], d01, ro23);
      ro01 = fma2(C01[j][2], d23.xx, ro01), ro23 = fma2(C23[j][2], d23.xx, ro23);
      ro01 = fma2_hi(C01[j][3], d23, ro01), ro23 = fma2_hi(C23[j][3], d23, ro23);
      if constexpr (decltype(coupled)::value) {  // y_E moves by X_jE D_j: lane j keeps its own
#pragma unroll                                   // contact's steps, the quad sums them before E
        for (int ed = 0; ed < 4; ed++) dsel[ed] = sub == j ? dfs[ed] : dsel[ed];
      }
    } else if constexpr (NF == 1 && CON) {
      {
        float a, b, cc;
        if constexpr (QUAD) {  // contact j's y lives in lane j of the quad
          a = qbcast(yo[0], j), b = qbcast(yo[1], j), cc = qbcast(yo[2], j);
        } else {
          a = yb[j][0], b = yb[j][1], cc = yb[j][2];
        }
        const float mu = ymu[j], Rp = yRp[j];
        float r[4], df[4];
        r[0] = fmaf(Rp, cfo[j][0], fmaf(mu, b, a));
        r[1] = fmaf(Rp, cfo[j][1], fmaf(-mu, b, a));
        r[2] = fmaf(Rp, cfo[j][2], fmaf(mu, cc, a));
        r[3] = fmaf(Rp, cfo[j][3], fmaf(-mu, cc, a));
        int q = 0;
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
#pragma unroll
          for (int d = 0; d < ed; d++) r[ed] = fmaf(yA[j][q++], df[d], r[ed]);
          df[ed] = fmaxf(r[ed] * -yia[j][ed], -cfo[j][ed]);
        }
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          cfo[j][ed] += df[ed];
          improvement = fmaf(-df[ed], fmaf(yhd[j][ed], df[ed], r[ed]), improvement);
        }
        const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
        if constexpr (QUAD) {  // this lane's contact moves by its row of the cross-Gram
#pragma unroll
          for (int rr = 0; rr < 3; rr++)
            yo[rr] = fmaf(xr[j][3 * rr], D[0], fmaf(xr[j][3 * rr + 1], D[1], fmaf(xr[j][3 * rr + 2], D[2], yo[rr])));
        }
        if constexpr (!QUAD) {
          const float* G = yG[j];
          yb[j][0] = fmaf(G[0], D[0], fmaf(G[1], D[1], fmaf(G[2], D[2], a)));
          yb[j][1] = fmaf(G[1], D[0], fmaf(G[3], D[1], fmaf(G[4], D[2], b)));
          yb[j][2] = fmaf(G[2], D[0], fmaf(G[4], D[1], fmaf(G[5], D[2], cc)));
        }
#pragma unroll
        for (int k = 0; k < FC; k++) {
          if (QUAD || k == j) continue;
#pragma unroll
          for (int rr = 0; rr < 3; rr++) {
            float s = yb[k][rr];
#pragma unroll
            for (int qq = 0; qq < 3; qq++)
              s = fmaf(k < j ? xg[ypair(k, j)][3 * rr + qq] : xg[ypair(j, k)][3 * qq + rr], D[qq], s);
            yb[k][rr] = s;
          }
        }
        if constexpr (decltype(coupled)::value) {  // the extra contact shares the free body
#pragma unroll
          for (int q = 0; q < 3; q++) {
            float s = yE[q];
#pragma unroll
            for (int rr = 0; rr < 3; rr++) s = fmaf(EX(E_X + 9 * j + 3 * rr + q), D[rr], s);
            yE[q] = s;
          }
        }
      }
    }
  };
  // dof-frictionloss rows of the y variants, short-chain form: df = clamp(-res/ARdiag,
  // -fl - f, fl - f) (the projected step), v_arm += M^-1 e_i df
  auto fric_row_y = [&](const int i, float& improvement, auto ext, auto pk, float& famax) {
    {
      const float fl = m.dof_frictionloss[i];
      const float res = fmaf(fR[i], ff[i], v[i] - fa[i]);
      const float fn = fminf(fmaxf(fmaf(res, -fiD[i], ff[i]), -fl), fl);
      const float df = fn - ff[i];
      famax += fabsf(df);  // a NaN step keeps famax from passing the retire test
      if constexpr (decltype(pk)::value) {
#pragma unroll
        for (int k = 0; k + 1 < NA; k += 2) {  // v_arm += M^-1 e_i df, two dofs per packed FMA
          const f2 t = fma2(Mp[i][k >> 1], splat2(df), f2{v[k], v[k + 1]});
          v[k] = t.x, v[k + 1] = t.y;
        }
        if constexpr (NA & 1) v[NA - 1] = fmaf(Mi.a(i, NA - 1), df, v[NA - 1]);
      } else {
#pragma unroll
        for (int k = 0; k < NA; k++) v[k] = fmaf(Mi.a(i, k), df, v[k]);
      }
      if constexpr (decltype(ext)::value) {  // the extra contact's y: J_E M^-1 e_i = W_E[i]
#pragma unroll
        for (int q = 0; q < 3; q++)
          yE[q] = fmaf(decltype(pk)::value ? ((i & 1) ? xq.eWp[3 * q + (i >> 1)].y : xq.eWp[3 * q + (i >> 1)].x)
                                           : EX(E_W + 6 * q + i),
                       df, yE[q]);
      }
      ff[i] = fn;
      improvement = fmaf(-df, fmaf(fhD[i], df, res), improvement);
    }
  };
  // after the sweeps: the free body's velocity from the block's force change
  auto yblock_finish = [&]() {
    if constexpr (NF == 1 && CON) {
#pragma unroll
      for (int k = 0; k < FC; k++) {
        const int c = cslot[k];
        float d[4];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) d[ed] = k < nrun ? cfo[k][ed] - L.at(c, F_FRC + ed) : 0.f;
        const float mu = ymu[k];
        const float Dn = (d[0] + d[1]) + (d[2] + d[3]), D1 = mu * (d[0] - d[1]), D2 = mu * (d[2] - d[3]);
#pragma unroll
        for (int i = 0; i < 6; i++)
          v[NA + i] = fmaf(Mi.Fd[0][i],
                           fmaf(L.at(c, NA + i), Dn, fmaf(L.at(c, 12 + NA + i), D1, L.at(c, 24 + NA + i) * D2)),
                           v[NA + i]);
      }
    }
  };
  // edge Gram off-diagonals A_ed (d < e) of a contact from its 3x3 Gram block and mu
  auto edge_gram = [](const float G[6], float mu, float A[6]) {
    auto gt = [&](int e) { return (e >> 1) ? G[2] : G[1]; };
    auto gtt = [&](int e, int d) {
      const int te = e >> 1, td = d >> 1;
      return te == td ? (te ? G[5] : G[3]) : G[4];
    };
    auto sg = [&](int e) { return (e & 1) ? -mu : mu; };
    int q = 0;
#pragma unroll
    for (int ed = 1; ed < 4; ed++)
#pragma unroll
      for (int d = 0; d < ed; d++) A[q++] = G[0] + sg(ed) * gt(ed) + sg(d) * gt(d) + sg(ed) * sg(d) * gtt(ed, d);
  };
  // Set up E (record cE) and F (record cF); an absent slot is the zero record: 1/ARdiag = 0
  // and f = 0, so its steps are exact no-ops.
  auto yext_setup = [&](int cE, int cF) {
    if constexpr (NF == 1 && CON) {
      // ---- E: W_E, y_E, cross-Gram with the block, chain constants
#pragma unroll
      for (int q = 0; q < 3; q++) {
        float ja[NA], y = 0.f;
#pragma unroll
        for (int i = 0; i < NA; i++) ja[i] = L.at(cE, 12 * q + i);
#pragma unroll
        for (int i = 0; i < NA; i++) {
          float w = 0.f;
#pragma unroll
          for (int k = 0; k < NA; k++) w = fmaf(Mi.a(i, k), ja[k], w);
          EX(E_W + 6 * q + i) = w;
          y = fmaf(ja[i], v[i], y);
        }
#pragma unroll
        for (int i = 0; i < 6; i++) y = fmaf(L.at(cE, 12 * q + NA + i), v[NA + i], y);
        yE[q] = y;
      }
#pragma unroll
      for (int k = 0; k < FC; k++)
#pragma unroll
        for (int r = 0; r < 3; r++) {
          float jk[6];
#pragma unroll
          for (int i = 0; i < 6; i++) jk[i] = L.at(cslot[k], 12 * r + NA + i) * Mi.Fd[0][i];
#pragma unroll
          for (int q = 0; q < 3; q++) {
            float x = 0.f;
#pragma unroll
            for (int i = 0; i < 6; i++) x = fmaf(jk[i], L.at(cE, 12 * q + NA + i), x);
            EX(E_X + 9 * k + 3 * r + q) = x;
          }
        }
      {
        float ar[4], G[6], A[6];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          ar[ed] = L.at(cE, F_AREF + ed);
          fE[ed] = L.at(cE, F_FRC + ed);
          EX(E_IA + ed) = L.at(cE, F_IARD + ed);
          EX(E_HD + ed) = L.at(cE, F_HARD + ed);
        }
        const float mu = L.at(cE, F_MU);
        EX(E_MU) = mu;
        EX(E_RP) = L.at(cE, F_R);
        yE[0] -= 0.5f * (ar[0] + ar[1]);
        yE[1] -= mu > 0.f ? 0.5f * (ar[0] - ar[1]) / mu : 0.f;
        yE[2] -= mu > 0.f ? 0.5f * (ar[2] - ar[3]) / mu : 0.f;
#pragma unroll
        for (int i = 0; i < 6; i++) G[i] = EX(E_G + i) = L.at(cE, F_GRAM + i);
        edge_gram(G, mu, A);
#pragma unroll
        for (int i = 0; i < 6; i++) EX(E_A + i) = A[i];
      }
      // ---- F: J_arm, W_F, X_EF = J_E,arm W_F', chain constants, aref shift
#pragma unroll
      for (int r = 0; r < 3; r++) {
        float jf[NA], w[NA];
#pragma unroll
        for (int i = 0; i < NA; i++) jf[i] = EX(F_J + 6 * r + i) = L.at(cF, 12 * r + i);
#pragma unroll
        for (int i = 0; i < NA; i++) {
          float t = 0.f;
#pragma unroll
          for (int k = 0; k < NA; k++) t = fmaf(Mi.a(i, k), jf[k], t);
          w[i] = EX(F_W + 6 * r + i) = t;
        }
#pragma unroll
        for (int q = 0; q < 3; q++) {
          float x = 0.f;
#pragma unroll
          for (int i = 0; i < NA; i++) x = fmaf(L.at(cE, 12 * q + i), w[i], x);
          EX(F_XE + 3 * q + r) = x;
        }
      }
      {
        float ar[4], G[6], A[6];
#pragma unroll
        for (int ed = 0; ed < 4; ed++) {
          ar[ed] = L.at(cF, F_AREF + ed);
          fF[ed] = L.at(cF, F_FRC + ed);
          EX(F_IA + ed) = L.at(cF, F_IARD + ed);
          EX(F_HD + ed) = L.at(cF, F_HARD + ed);
        }
        const float mu = L.at(cF, F_MU);
        EX(F_MUX) = mu;
        EX(F_RPX) = L.at(cF, F_R);
        EX(F_SH + 0) = 0.5f * (ar[0] + ar[1]);
        EX(F_SH + 1) = mu > 0.f ? 0.5f * (ar[0] - ar[1]) / mu : 0.f;
        EX(F_SH + 2) = mu > 0.f ? 0.5f * (ar[2] - ar[3]) / mu : 0.f;
#pragma unroll
        for (int i = 0; i < 6; i++) G[i] = L.at(cF, F_GRAM + i);
        edge_gram(G, mu, A);
#pragma unroll
        for (int i = 0; i < 6; i++) EX(F_A + i) = A[i];
      }
    }
  };
  // one sweep step of F (arm-only, before E in row order): v-form on the arm (its y from
  // three NA-dof dots), the edge chain, v_arm += W_F D, and E's y by X_EF D
  auto yf_row = [&](float& improvement) {
    if constexpr (NF == 1 && CON) {
      const float mu = EX(F_MUX), Rp = EX(F_RPX);
      float y[3];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        float t = -EX(F_SH + q);
#pragma unroll
        for (int i = 0; i < NA; i++) t = fmaf(EX(F_J + 6 * q + i), v[i], t);
        y[q] = t;
      }
      float r[4], df[4];
      r[0] = fmaf(Rp, fF[0], fmaf(mu, y[1], y[0]));
      r[1] = fmaf(Rp, fF[1], fmaf(-mu, y[1], y[0]));
      r[2] = fmaf(Rp, fF[2], fmaf(mu, y[2], y[0]));
      r[3] = fmaf(Rp, fF[3], fmaf(-mu, y[2], y[0]));
      int q = 0;
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
#pragma unroll
        for (int d = 0; d < ed; d++) r[ed] = fmaf(EX(F_A + q++), df[d], r[ed]);
        df[ed] = fmaxf(r[ed] * -EX(F_IA + ed), -fF[ed]);
      }
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
        fF[ed] += df[ed];
        improvement = fmaf(-df[ed], fmaf(EX(F_HD + ed), df[ed], r[ed]), improvement);
      }
      const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
#pragma unroll
      for (int i = 0; i < NA; i++)
        v[i] = fmaf(EX(F_W + i), D[0], fmaf(EX(F_W + 6 + i), D[1], fmaf(EX(F_W + 12 + i), D[2], v[i])));
#pragma unroll
      for (int qq = 0; qq < 3; qq++)
        yE[qq] = fmaf(EX(F_XE + 3 * qq), D[0], fmaf(EX(F_XE + 3 * qq + 1), D[1], fmaf(EX(F_XE + 3 * qq + 2), D[2], yE[qq])));
    }
  };
  // quad mode, packed: the block's accumulated steps on y_E (lane-split X_kE D_k)
  auto yblock_to_e = [&](const float (&dsel)[4]) {
    const float mu = xq.muo;
    const float D[3] = {(dsel[0] + dsel[1]) + (dsel[2] + dsel[3]), mu * (dsel[0] - dsel[1]), mu * (dsel[2] - dsel[3])};
#pragma unroll
    for (int q = 0; q < 3; q++) {
      float p = 0.f;
#pragma unroll
      for (int rr = 0; rr < 3; rr++) p = fmaf(xq.xo[3 * rr + q], D[rr], p);
      yE[q] += qsum(p);
    }
  };
  // quad mode, packed: one edge chain (pyramid of 4 edges) from y = (a, b, c)
  // scaled residuals as in the block (s = -r / ARdiag; nia = -1/ARdiag per edge, the A's
  // pre-scaled by the -1/ARdiag of the edge they move), steps built in their pairs
  auto qchain = [&](float a, float b, float c, float (&f)[4], float mu, float Rp, f2 nia01, f2 nia23, float A10,
                    f2 A2030, f2 A2131, float A32, f2 hd01, f2 hd23, f2& imp, float (&df)[4]) {
    const f2 c01 = f2{f[0], f[1]}, c23 = f2{f[2], f[3]};
    const f2 s01 = fma2(splat2(Rp), c01, fma2(f2{mu, -mu}, splat2(b), splat2(a))) * nia01;
    f2 s23 = fma2(splat2(Rp), c23, fma2(f2{mu, -mu}, splat2(c), splat2(a))) * nia23;
    f2 d01, d23;
    d01.x = max_neg(s01.x, c01.x);
    const float s1 = fmaf(A10, d01.x, s01.y);
    s23 = fma2(A2030, d01.xx, s23);
    d01.y = max_neg(s1, c01.y);
    s23 = fma2_hi(A2131, d01, s23);
    d23.x = max_neg(s23.x, c23.x);
    const float s3 = fmaf(A32, d23.x, s23.y);
    d23.y = max_neg(s3, c23.y);
    df[0] = d01.x, df[1] = d01.y, df[2] = d23.x, df[3] = d23.y;
    const f2 n01 = c01 + d01, n23 = c23 + d23;
    f[0] = n01.x, f[1] = n01.y, f[2] = n23.x, f[3] = n23.y;
    imp = fma2(-(hd01 * d01), fma2(f2{s01.x, s1}, splat2(-2.f), d01), imp);
    imp = fma2(-(hd23 * d23), fma2(f2{s23.x, s3}, splat2(-2.f), d23), imp);
  };
  // v_arm += W D with W as dof pairs (W[q] row pairs)
  auto qvarm = [&](const f2 (&Wp)[9], const float (&D)[3]) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      f2 t = f2{v[2 * k], v[2 * k + 1]};
#pragma unroll
      for (int q = 0; q < 3; q++) t = fma2(Wp[3 * q + k], splat2(D[q]), t);
      v[2 * k] = t.x, v[2 * k + 1] = t.y;
    }
  };
  auto yf_row_q = [&](f2& imp, float& famax) {
    f2 y01 = xq.fSh01;
    float y2 = xq.fSh2;
#pragma unroll
    for (int i = 0; i < NA; i++) y01 = fma2(xq.fJp[i], splat2(v[i]), y01), y2 = fmaf(xq.fJ2[i], v[i], y2);
    float df[4];
    qchain(y01.x, y01.y, y2, fF, xq.fMu, xq.fRp, xq.fNia01, xq.fNia23, xq.fA10, xq.fA2030, xq.fA2131, xq.fA32, xq.fHD01, xq.fHD23,
           imp, df);
    famax += (fabsf(df[0]) + fabsf(df[1])) + (fabsf(df[2]) + fabsf(df[3]));
    const float mu = xq.fMu;
    const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
    qvarm(xq.fWp, D);
    f2 e01 = f2{yE[0], yE[1]};
#pragma unroll
    for (int rr = 0; rr < 3; rr++) e01 = fma2(xq.fXp[rr], splat2(D[rr]), e01), yE[2] = fmaf(xq.fX2[rr], D[rr], yE[2]);
    yE[0] = e01.x, yE[1] = e01.y;
  };
  // varm = false: v_arm is not read again during these sweeps (frictionloss rows retired, no F
  // slot), so E's v_arm update is deferred to one product with its total force change
  auto yext_row_q = [&](f2& imp, auto coupled, float& famax, auto varm) {
    float df[4];
    qchain(yE[0], yE[1], yE[2], fE, xq.eMu, xq.eRp, xq.eNia01, xq.eNia23, xq.eA10, xq.eA2030, xq.eA2131, xq.eA32, xq.eHD01, xq.eHD23,
           imp, df);
    if constexpr (!decltype(coupled)::value) famax += (fabsf(df[0]) + fabsf(df[1])) + (fabsf(df[2]) + fabsf(df[3]));
    const float mu = xq.eMu;
    const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
    if constexpr (decltype(varm)::value) qvarm(xq.eWp, D);
    if constexpr (decltype(coupled)::value) {  // this lane's block contact moves by X_own,E D
#pragma unroll
      for (int qq = 0; qq < 3; qq++) {
        ro01 = fma2(xq.qe01[qq], splat2(D[qq]), ro01);
        ro23 = fma2(xq.qe23[qq], splat2(D[qq]), ro23);
      }
    }
    f2 e01 = f2{yE[0], yE[1]};
    float e2 = yE[2];
#pragma unroll
    for (int qq = 0; qq < 3; qq++) e01 = fma2(xq.eGp[qq], splat2(D[qq]), e01), e2 = fmaf(xq.eG2[qq], D[qq], e2);
    yE[0] = e01.x, yE[1] = e01.y, yE[2] = e2;
  };
  // quad mode: preload the E/F coefficients (after yext_setup wrote them to LDS)
  auto yext_preload = [&]() {
#pragma unroll
    for (int q = 0; q < 3; q++)
#pragma unroll
      for (int k = 0; k < 3; k++) {
        xq.eWp[3 * q + k] = f2{EX(E_W + 6 * q + 2 * k), EX(E_W + 6 * q + 2 * k + 1)};
        xq.fWp[3 * q + k] = f2{EX(F_W + 6 * q + 2 * k), EX(F_W + 6 * q + 2 * k + 1)};
      }
    float eia[4], fia[4];  // -1/ARdiag of the E and F edges
#pragma unroll
    for (int ed = 0; ed < 4; ed++) eia[ed] = -EX(E_IA + ed), fia[ed] = -EX(F_IA + ed);
    xq.eNia01 = f2{eia[0], eia[1]}, xq.eNia23 = f2{eia[2], eia[3]};
    xq.fNia01 = f2{fia[0], fia[1]}, xq.fNia23 = f2{fia[2], fia[3]};
    xq.eA10 = eia[1] * EX(E_A + 0), xq.eA32 = eia[3] * EX(E_A + 5);
    xq.eA2030 = f2{eia[2] * EX(E_A + 1), eia[3] * EX(E_A + 3)}, xq.eA2131 = f2{eia[2] * EX(E_A + 2), eia[3] * EX(E_A + 4)};
    xq.fA10 = fia[1] * EX(F_A + 0), xq.fA32 = fia[3] * EX(F_A + 5);
    xq.fA2030 = f2{fia[2] * EX(F_A + 1), fia[3] * EX(F_A + 3)}, xq.fA2131 = f2{fia[2] * EX(F_A + 2), fia[3] * EX(F_A + 4)};
    xq.eHD01 = f2{EX(E_HD + 0), EX(E_HD + 1)}, xq.eHD23 = f2{EX(E_HD + 2), EX(E_HD + 3)};
    xq.fHD01 = f2{EX(F_HD + 0), EX(F_HD + 1)}, xq.fHD23 = f2{EX(F_HD + 2), EX(F_HD + 3)};
    xq.eMu = EX(E_MU), xq.eRp = EX(E_RP), xq.fMu = EX(F_MUX), xq.fRp = EX(F_RPX);
#pragma unroll
    for (int i = 0; i < NA; i++) xq.fJp[i] = f2{EX(F_J + i), EX(F_J + 6 + i)}, xq.fJ2[i] = EX(F_J + 12 + i);
#pragma unroll
    for (int rr = 0; rr < 3; rr++) xq.fXp[rr] = f2{EX(F_XE + rr), EX(F_XE + 3 + rr)}, xq.fX2[rr] = EX(F_XE + 6 + rr);
    xq.eGp[0] = f2{EX(E_G + 0), EX(E_G + 1)}, xq.eGp[1] = f2{EX(E_G + 1), EX(E_G + 3)}, xq.eGp[2] = f2{EX(E_G + 2), EX(E_G + 4)};
    xq.eG2[0] = EX(E_G + 2), xq.eG2[1] = EX(E_G + 4), xq.eG2[2] = EX(E_G + 5);
#pragma unroll
    for (int t = 0; t < 9; t++) xq.xo[t] = EX(E_X + 9 * sub + t);
    xq.muo = sub == 0 ? ymu[0] : sub == 1 ? ymu[1] : sub == 2 ? ymu[2] : ymu[3];
#pragma unroll
    for (int qq = 0; qq < 3; qq++) {  // residual form of X_own,E: rows (1, s_e on t(e)) of the own
                                      // contact, scaled by its -1/ARdiag as the residuals are
      xq.qe01[qq] = f2{fmaf(xq.muo, xq.xo[3 + qq], xq.xo[qq]), fmaf(-xq.muo, xq.xo[3 + qq], xq.xo[qq])} * own_nia01();
      xq.qe23[qq] = f2{fmaf(xq.muo, xq.xo[6 + qq], xq.xo[qq]), fmaf(-xq.muo, xq.xo[6 + qq], xq.xo[qq])} * own_nia23();
    }
    xq.fSh01 = f2{-EX(F_SH + 0), -EX(F_SH + 1)}, xq.fSh2 = -EX(F_SH + 2);
  };
  // one sweep step of the extra contact (after the friction rows and the block)
  auto yext_row = [&](float& improvement, auto coupled) {
    if constexpr (NF == 1 && CON) {
      const float mu = EX(E_MU), Rp = EX(E_RP);
      float r[4], df[4];
      r[0] = fmaf(Rp, fE[0], fmaf(mu, yE[1], yE[0]));
      r[1] = fmaf(Rp, fE[1], fmaf(-mu, yE[1], yE[0]));
      r[2] = fmaf(Rp, fE[2], fmaf(mu, yE[2], yE[0]));
      r[3] = fmaf(Rp, fE[3], fmaf(-mu, yE[2], yE[0]));
      int q = 0;
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
#pragma unroll
        for (int d = 0; d < ed; d++) r[ed] = fmaf(EX(E_A + q++), df[d], r[ed]);
        df[ed] = fmaxf(r[ed] * -EX(E_IA + ed), -fE[ed]);
      }
#pragma unroll
      for (int ed = 0; ed < 4; ed++) {
        fE[ed] += df[ed];
        improvement = fmaf(-df[ed], fmaf(EX(E_HD + ed), df[ed], r[ed]), improvement);
      }
      const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
#pragma unroll
      for (int i = 0; i < NA; i++)
        v[i] = fmaf(EX(E_W + i), D[0], fmaf(EX(E_W + 6 + i), D[1], fmaf(EX(E_W + 12 + i), D[2], v[i])));
      if constexpr (decltype(coupled)::value) {
        if constexpr (QUAD) {
#pragma unroll
          for (int rr = 0; rr < 3; rr++) {
            float s = yo[rr];
#pragma unroll
            for (int qq = 0; qq < 3; qq++) s = fmaf(EX(E_X + 9 * sub + 3 * rr + qq), D[qq], s);
            yo[rr] = s;
          }
        } else {
#pragma unroll
          for (int k = 0; k < FC; k++)
#pragma unroll
            for (int rr = 0; rr < 3; rr++) {
              float s = yb[k][rr];
#pragma unroll
              for (int qq = 0; qq < 3; qq++) s = fmaf(EX(E_X + 9 * k + 3 * rr + qq), D[qq], s);
              yb[k][rr] = s;
            }
        }
      }
      const float y0 = yE[0], y1 = yE[1], y2 = yE[2];
      yE[0] = fmaf(EX(E_G + 0), D[0], fmaf(EX(E_G + 1), D[1], fmaf(EX(E_G + 2), D[2], y0)));
      yE[1] = fmaf(EX(E_G + 1), D[0], fmaf(EX(E_G + 3), D[1], fmaf(EX(E_G + 4), D[2], y1)));
      yE[2] = fmaf(EX(E_G + 2), D[0], fmaf(EX(E_G + 4), D[1], fmaf(EX(E_G + 5), D[2], y2)));
    }
  };
  // after the sweeps: E's forces back to its record; its free-body part moves v6
  auto yext_finish = [&](int c, bool hasE, int cF, bool hasF, auto coupled) {
    if constexpr (NF == 1 && CON) {
      if (hasF) {
#pragma unroll
        for (int ed = 0; ed < 4; ed++) L.at(cF, F_FRC + ed) = fF[ed];
      }
      float d[4];
#pragma unroll
      for (int ed = 0; ed < 4; ed++) d[ed] = hasE ? fE[ed] - L.at(c, F_FRC + ed) : 0.f;
      if constexpr (decltype(coupled)::value) {
        const float mu = L.at(c, F_MU);
        const float Dn = (d[0] + d[1]) + (d[2] + d[3]), D1 = mu * (d[0] - d[1]), D2 = mu * (d[2] - d[3]);
#pragma unroll
        for (int i = 0; i < 6; i++)
          v[NA + i] = fmaf(Mi.Fd[0][i],
                           fmaf(L.at(c, NA + i), Dn, fmaf(L.at(c, 12 + NA + i), D1, L.at(c, 24 + NA + i) * D2)),
                           v[NA + i]);
      }
      if (hasE) {
#pragma unroll
        for (int ed = 0; ed < 4; ed++) L.at(c, F_FRC + ed) = fE[ed];
      }
    }
  };
  // extras in row order: F = the first of two (arm-only), E = the last one
  const int cE = npost >= 1 ? xidx(npost - 1) : LDS_CON, cF = npost == 2 ? xidx(0) : LDS_CON;
  const bool hasE = npost >= 1, hasF = npost == 2;
  auto ysweeps = [&](auto ext, auto coupled, auto ext2) {
    yblock_setup();
    using PK = std::integral_constant<bool, QUAD>;
    yblock_consts(PK{});
    if constexpr (PK::value) {
#pragma unroll
      for (int i = 0; i < NA; i++)
#pragma unroll
        for (int k = 0; k + 1 < NA; k += 2) Mp[i][k >> 1] = f2{Mi.a(i, k), Mi.a(i, k + 1)};
    }
    if constexpr (decltype(ext)::value) {
      yext_setup(cE, cF);
      if constexpr (PK::value) yext_preload();
    }
    // one sweep; ARM = false leaves out the arm's rows, FRIC = false only its frictionloss
    // rows (see below).  Returns the improvement; famax gets the sum of |df| over the arm's
    // rows (ffmax: over its frictionloss rows).
    auto sweep = [&](auto arm, auto fric, float& famax, float& ffmax) {
      // the arm's frictionloss rows and the cube block touch disjoint dofs (M is block
      // diagonal): the two Gauss-Seidel chains commute, so their rows are interleaved in
      // program order to give the (latency-bound) issue stream independent work; the
      // improvement terms go to one accumulator per chain
      float improvement = 0.f, imp_b = 0.f;
      f2 impq = f2{0.f, 0.f};
      float dsel[4] = {0.f, 0.f, 0.f, 0.f};
      // (NA = 6, FC = 4: rows {0,1} c0 {2} c1 {3,4} c2 {5} c3)
#pragma unroll
      for (int j = 0; j < FC; j++) {
        if constexpr (decltype(arm)::value && decltype(fric)::value) {
#pragma unroll
          for (int i = (j * NA + FC - 1) / FC; i < ((j + 1) * NA + FC - 1) / FC; i++)
            fric_row_y(i, improvement, ext, PK{}, ffmax);
        }
        yblock_contact(j, imp_b, impq, dsel, coupled, PK{});
      }
      if constexpr (FC == 0) {
#pragma unroll
        for (int i = 0; i < NA; i++) fric_row_y(i, improvement, ext, PK{}, ffmax);
      }
      if constexpr (PK::value) {
        if constexpr (decltype(ext)::value && decltype(coupled)::value) yblock_to_e(dsel);
        if constexpr (decltype(arm)::value && decltype(ext2)::value) yf_row_q(impq, famax);
        if constexpr (decltype(arm)::value && decltype(ext)::value)
          yext_row_q(impq, coupled, famax, std::integral_constant<bool, decltype(fric)::value || decltype(ext2)::value>{});
        improvement += impq.x + impq.y;
      } else {
        improvement += imp_b;
        if constexpr (decltype(ext2)::value) yf_row(improvement);
        if constexpr (decltype(ext)::value) yext_row(improvement, coupled);
      }
      return improvement;
    };
    // Arm retirement.  Unless an extra contact touches the cube, the arm's rows (its dof
    // frictionloss rows and the arm-only extra slots E/F) and the cube block share no dof:
    // two Gauss-Seidel systems that only meet in the stopping test.  Once a sweep moves the
    // arm's forces by at most ARM_RETIRE in total (N, N m) on every lane of the wave, the
    // remaining sweeps run the block alone (the pure block converges ~95 sweeps slower than
    // the arm, which settles in ~3).  The threshold sits an order below what MuJoCo's own
    // stopping test resolves: a row's step df lowers the cost by >= ARdiag df^2 / 2, and the
    // solve stops at improvement / trace(M) < tolerance (1e-8), which for the arm's rows
    // (ARdiag ~ 30, trace(M) ~ 0.3) leaves steps of order 1e-5.  Exactly-zero steps (the
    // common case: frictionloss rows saturated at +-frictionloss) leave the result bit for
    // bit equal to sweeping all rows.
    constexpr bool RETIRE = PK::value && FC > 0 && !decltype(coupled)::value;
    // Frictionloss retirement (the extra-slot variants).  The arm's 6 frictionloss rows settle
    // within a few sweeps (saturated at +-frictionloss, or holding), while an extra contact E
    // (arm on the table, or the gripper on the cube) keeps its Gauss-Seidel chain going for
    // tens of sweeps -- all ~95 of them when it touches the cube, which rules out the arm
    // retirement above.  Once one sweep moves the frictionloss forces by at most ARM_RETIRE in
    // total on every lane, the remaining sweeps leave those rows out and run E (and F) with
    // the block: the same threshold argument as the arm retirement, applied to the rows that
    // have settled.
    constexpr bool FRETIRE = PK::value && FC > 0 && decltype(ext)::value;
    int it = 0;
    bool done = false, fret = false;
    for (; it < m.iterations; it++) {
      float famax = 0.f, ffmax = 0.f;
      if (sweep(std::true_type{}, std::true_type{}, famax, ffmax) * scale < m.tolerance) {
        done = true;
        break;
      }
      if constexpr (RETIRE) {
        if (__all(famax + ffmax <= ARM_RETIRE)) {
#ifdef SOARM_PHASE_PROF
          armstop = it + 1;
#endif
          it++;
          break;
        }
      }
      if constexpr (FRETIRE) {
        if (__all(ffmax <= ARM_RETIRE)) {
          fret = true;
          it++;
          break;
        }
      }
    }
    if constexpr (FRETIRE) {
      // without F, nothing reads v_arm in these sweeps: E's steps move it once afterwards
      float fE0[4];
#pragma unroll
      for (int ed = 0; ed < 4; ed++) fE0[ed] = fE[ed];
      if (fret && !done)
        for (; it < m.iterations; it++) {
          float famax = 0.f, ffmax = 0.f;
          if (sweep(std::true_type{}, std::false_type{}, famax, ffmax) * scale < m.tolerance) {
            done = true;
            break;
          }
          if constexpr (RETIRE) {
            if (__all(famax <= ARM_RETIRE)) {
#ifdef SOARM_PHASE_PROF
              armstop = it + 1;
#endif
              it++;
              break;
            }
          }
        }
      if constexpr (!decltype(ext2)::value) {
        if (fret) {
          float df[4];
#pragma unroll
          for (int ed = 0; ed < 4; ed++) df[ed] = fE[ed] - fE0[ed];
          const float mu = xq.eMu;
          const float D[3] = {(df[0] + df[1]) + (df[2] + df[3]), mu * (df[0] - df[1]), mu * (df[2] - df[3])};
          qvarm(xq.eWp, D);
        }
      }
      // (no re-check of the retired frictionloss rows against the v_arm E / F kept moving
      // (ADVICE r03): holding their 24 values through the retired sweeps for a check costs the
      // kernel ~15 spilled VGPRs and 9% of its time (r04, measured; an applied verification
      // sweep also takes the result one sweep past mj_solPGS's stopping point).  The effect of
      // retiring them is bounded against the oracle's full-sweep PGS on envs with an extra
      // contact by test_gpu_parity.test_one_substep_extra_contact_sweeps.)
    }
    if constexpr (RETIRE) {
      // the block-only sweeps hold far fewer values than the sweeps with the arm's rows:
      // re-define the block's loop constants here (an empty asm per value) so they get
      // registers of their own for this loop instead of the AGPR homes they were given
      // under the first loop's pressure (one copy here, not an AGPR read per sweep)
      if constexpr (PK::value) {
#pragma unroll
        for (int k = 0; k < FC; k++) {
          vpin(qA2030[k]), vpin(qA2131[k]), vpin(qhd01[k]), vpin(qhd23[k]), vpin(sA10[k]), vpin(sA32[k]);
#pragma unroll
          for (int ed = 0; ed < 4; ed++) vpin(C01[k][ed]), vpin(C23[k][ed]), vpin(cfo[k][ed]);
        }
        vpin(ro01), vpin(ro23);
      }
      if (!done)
        for (; it < m.iterations; it++) {
          float unused = 0.f, unused2 = 0.f;
          if (sweep(std::false_type{}, std::false_type{}, unused, unused2) * scale < m.tolerance) {
            done = true;
            break;
          }
        }
    }
#ifdef SOARM_PHASE_PROF
    nsweep = done ? it + 1 : m.iterations;
#endif
    (void)done;
    yblock_finish();
    if constexpr (decltype(ext)::value) yext_finish(cE, hasE, cF, hasF, coupled);
  };
  const bool ypure = CON && NF == 1 && block_first && __all(nlim == 0 && nl == ncon && npost == 0);
  // up to two extras: the first of two must be arm-only (arm-only pairs precede the cube's
  // in pair order, so that is the common case), the last may touch the cube
  const bool yext = CON && NF == 1 && !ypure && block_first &&
                    __all(nlim == 0 && nl == ncon && npost <= 2 &&
                          (npost < 2 || (int)L.at(xidx(0), F_FLAGS) == TOUCH_ARM));
  const bool ycoupled = yext && __any(npost >= 1 && ((int)L.at(cE, F_FLAGS) & TOUCH_FREE));
  const bool yext2 = yext && __any(npost == 2);
  auto sweeps = [&](auto first) {
    for (int it = 0; it < m.iterations; it++) {
      float improvement = 0.f;
      if constexpr (decltype(first)::value) {
        fric_rows(improvement);  // same basic block as the register block: they interleave
        block_rows(improvement);
        limit_rows(improvement);
        for (int j = 0; j < npost; j++) lds_contact(j < c0 - npre ? npre + j : c1 + j - (c0 - npre), improvement);
        scratch_rows(improvement);
      } else {
        fric_rows(improvement);
        limit_rows(improvement);
        for (int c = 0; c < npre; c++) lds_contact(c, improvement);
        block_rows(improvement);
        for (int j = 0; j < npost; j++) lds_contact(j < c0 - npre ? npre + j : c1 + j - (c0 - npre), improvement);
        scratch_rows(improvement);
      }
      if (improvement * scale < m.tolerance) {
#ifdef SOARM_PHASE_PROF
        nsweep = it + 1;
#endif
        break;
      }
    }
  };
  // ---- row-space PGS (RS kernel; see RS_MAXROW above).  Rows in mj_solPGS order: the NA dof
  // frictionloss rows, the active limits, 4 pyramid edges per contact; NRB (compile time) bounds
  // the rows of every env of the wave (rows past an env's own are zero rows: J = 0, so C's row and
  // column are 0 and their steps are exact no-ops).  Lane r16 holds rows r16 (slot A) and 16 + r16
  // (slot B, when NRB > 16).  v: the velocity after the warm start; on return, qacc.
  auto rs_solve = [&](auto kat_c, auto kac_c) {
    if constexpr (RS && NF == 1 && CON) {
      using LY = RsLayout<NA, decltype(kat_c)::value, decltype(kac_c)::value>;
      constexpr int NS = LY::NS, KAT = decltype(kat_c)::value, KAC = decltype(kac_c)::value;
      const int r16 = L.lane & 15;
      float* const Wl = L.rsw + L.col * RS_WENV;
      // this lane's rows: slot A = CT edge r16, slot B = frictionloss row / AT edge / AC edge r16;
      // kind 0 frictionloss, 1 pyramid edge, -1 none; c, ed: the edge's contact and edge index;
      // qA / qB: the rows' step indices (their W rows in LDS)
      const int cA = rs_nat + (r16 >> 2), qA = LY::CT0 + r16;
      const int kindA = (r16 >> 2) < rs_nct ? 1 : -1;
      int kindB = -1, cB = 0;
      if (r16 < NA) {
        kindB = 0;
      } else if (r16 < LY::CT0) {
        cB = (r16 - NA) >> 2, kindB = cB < rs_nat ? 1 : -1;
      } else if (r16 < LY::CT0 + 4 * KAC) {
        const int k = (r16 - LY::CT0) >> 2;
        cB = rs_nat + rs_nct + k, kindB = k < rs_nac ? 1 : -1;
      }
      const int qB = r16 < LY::CT0 ? r16 : r16 + 16;
      // row data: J (NV), aref, R, the warm-start force (the warm start above)
      auto row_of = [&](int kind, int c, int ed, float (&J)[NV], float& ar, float& R, float& f) {
#pragma unroll
        for (int i = 0; i < NV; i++) J[i] = 0.f;
        ar = 0.f, R = 1.f, f = 0.f;
        if (kind == 0) {  // dof frictionloss row ed: J = e_ed
#pragma unroll
          for (int i = 0; i < NA; i++)
            if (ed == i) {
              J[i] = 1.f, ar = fa[i], R = fR[i];
              // warm-start force (the Gram-form warm start's frictionloss branch)
              const float fl = m.dof_frictionloss[i], jar = S.warm[i] - fa[i];
              const float fs = (jar <= -fl * R) ? fl : (jar >= fl * R) ? -fl : -jar / R;
              f = fl > 0.f ? fs : 0.f;
            }
        } else if (kind == 1) {  // pyramid edge J_n +- mu J_t of contact c
          const float mu = L.at(c, F_MU), s = (ed & 1) ? -mu : mu;
          const int t = 12 * (1 + (ed >> 1));
#pragma unroll
          for (int i = 0; i < NV; i++) J[i] = fmaf(s, L.at(c, t + i), L.at(c, i));
          ar = L.at(c, F_AREF + ed), R = L.at(c, F_R);
          float jar = -ar;  // warm-start force: the edge's J qacc_warmstart - aref, if negative
#pragma unroll
          for (int i = 0; i < NV; i++) jar = fmaf(J[i], S.warm[i], jar);
          f = jar < 0.f ? -jar / R : 0.f;
        }
      };
      float JA[NV], JB[NV], WA[NV], WB[NV], arA, arB, RA, RB, fA, fB;
      row_of(kindA, cA, r16 & 3, JA, arA, RA, fA);
      row_of(kindB, cB, kindB == 0 ? r16 : (r16 - NA) & 3, JB, arB, RB, fB);
      Mi.mul(JA, WA, false, true);  // (CT rows touch the free body alone)
      Mi.mul(JB, WB, true, KAC > 0);
      // W rows to LDS, by step (the 4 copies of a quad write identical values)
#pragma unroll
      for (int i = 0; i < NV; i++) Wl[qA * RS_WROW + i] = WA[i];
      if (qB < NS)
#pragma unroll
        for (int i = 0; i < NV; i++) Wl[qB * RS_WROW + i] = WB[i];
      // AR_rr = J_r W_r + R_r
      float ardA = RA, ardB = RB;
#pragma unroll
      for (int i = 0; i < NV; i++) ardA = fmaf(JA[i], WA[i], ardA), ardB = fmaf(JB[i], WB[i], ardB);
      const float iA = 1.f / ardA, iB = 1.f / ardB;
      const float hdA = 0.5f * ardA, hdB = 0.5f * ardB;
      wave_sync();
      // the bound registers, broadcast over the env's row: -f_q (edges) and the frictionloss
      // rows' lo - f, hi - f
      float NF_[NS], NH_[NA];
      auto bounds = [&]() {
        sfor<NS>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          const float fq = -rowbcast<LY::lane(q)>(LY::slot(q) == 0 ? fA : fB);
          if constexpr (q < NA) {
            const float fl = m.dof_frictionloss[q];
            NF_[q] = fq - fl, NH_[q] = fq + fl;
          } else {
            NF_[q] = fq;
          }
        });
      };
      // v = qacc_smooth + sum_q W_q f_q (lane i < NV sums dof i, the row broadcasts it); f_q from the
      // bound registers (NH_ = fl - f on the frictionloss rows, NF_ = -f on the others)
      auto vel = [&]() {
        float acc = 0.f;
        const int di = r16 < NV ? r16 : 0;
#pragma unroll
        for (int q = 0; q < NS; q++)
          acc = fmaf(Wl[q * RS_WROW + di], q < NA ? m.dof_frictionloss[q] - NH_[q] : -NF_[q], acc);
        sfor<NV>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          v[i] = S.qacc_s[i] + rowbcast<i>(acc);
        });
      };
      // the warm start in row space (the Gram-form block above is skipped on these waves): every
      // row's warm force (row_of), v, and the dual cost against f = 0, summed over the env's rows
      bounds();
      vel();
      float jvA = -arA, jvB = -arB, jqA = -arA, jqB = -arB;
#pragma unroll
      for (int i = 0; i < NV; i++) {
        jvA = fmaf(JA[i], v[i], jvA), jvB = fmaf(JB[i], v[i], jvB);
        jqA = fmaf(JA[i], S.qacc_s[i], jqA), jqB = fmaf(JB[i], S.qacc_s[i], jqB);
      }
      // dual cost: sum_r 0.5 f_r (J_r v - aref_r + R_r f_r) + 0.5 f_r (J_r qacc_smooth - aref_r)
      const float wcost = rowsum16(0.5f * fA * (jvA + RA * fA) + 0.5f * fA * jqA +
                                   (0.5f * fB * (jvB + RB * fB) + 0.5f * fB * jqB));
      const bool rej = wcost > 0.f;  // worse than no warm start: f = 0, v = qacc_smooth
      if (__any(rej)) {              // (wave-uniform: the broadcasts run on every row)
        fA = rej ? 0.f : fA, fB = rej ? 0.f : fB;
        bounds();
#pragma unroll
        for (int i = 0; i < NV; i++) v[i] = rej ? S.qacc_s[i] : v[i];
        jvA = rej ? jqA : jvA, jvB = rej ? jqB : jvB;
      }
      f2 sA = f2{-fmaf(RA, fA, jvA) * iA, 0.f}, sB = f2{-fmaf(RB, fB, jvB) * iB, 0.f};
      // the scaled matrix: C[r][q] = -J_r W_q / AR_rr, C[r][r] = -1, as (C, G) pairs: G is the row's
      // own-step indicator, so the second accumulator takes the row's force step exactly (the stop
      // test's Delta f_r; it was u_r - Delta s_r from an off-diagonal accumulator, whose fp32
      // cancellation stopped an ill-conditioned env 22 sweeps early, 3.3e-3 m/s off -- r05); only
      // the blocks a step updates
      f2 CA[NS], CB[NS];
      sfor<NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr bool UA = LY::upd_a(q), UB = LY::upd_b(q);
        f2 a = f2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NV; i++)
          a = fma2(f2{UA ? JA[i] : 0.f, UB ? JB[i] : 0.f}, splat2(Wl[q * RS_WROW + i]), a);
        const float ca = -a.x * iA, cb = -a.y * iB;
        CA[q] = qA == q ? f2{-1.f, 1.f} : f2{ca, 0.f};
        CB[q] = qB == q ? f2{-1.f, 1.f} : f2{cb, 0.f};
        // (the W rows of two steps in flight at a time: hoisting every step's 12 LDS loads to
        // the top would hold hundreds of values)
        if constexpr (q & 1) __builtin_amdgcn_sched_barrier(0);
      });
      float scale = m.pgs_scale, tol = m.tolerance;
      int iters = m.iterations;
      // (loaded once: the sweeps' asm statements keep LICM from hoisting the model loads, which would
      // otherwise be re-issued and waited for in every sweep)
      asm volatile("" : "+s"(iters), "+s"(scale), "+s"(tol));
      bool done = false;
#ifdef SOARM_PHASE_PROF
      // (the RS solve's split, in the Newton profiler's slots: PGS builds leave them unused)
      // [8] setup, [9] sweeps, [10] final qacc, summed over waves; [11] waves; [16] sum of wave sweeps
      const long long rp0 = clock64();
      int wsw = 0;
#endif
      for (int it = 0; it < iters; it++) {
#ifdef SOARM_PHASE_PROF
        wsw = it + 1;
#endif
        if (!done) {
#ifdef SOARM_PHASE_PROF
          nsweep = it + 1;
#endif
          const float s0A = sA.x, s0B = sB.x;
          sA.y = 0.f, sB.y = 0.f;
          rs_sweep<NA, LY>(sA, sB, CA, CB, NF_, NH_);
          // improvement = sum_r AR_rr / 2 Delta f_r (s0 + s1)_r, Delta f_r = the row's own step (y)
          float P = hdA * sA.y * (s0A + sA.x);
          P = fmaf(hdB * sB.y, s0B + sB.x, P);
          done = rowsum16(P) * scale < tol;
        }
        if (__all(done)) break;
      }
#ifdef SOARM_PHASE_PROF
      const long long rp1 = clock64();
#endif
      // qacc = qacc_smooth + sum_q W_q f_q (NH_ = fl - f on the frictionloss rows, NF_ = -f on the
      // others): lane i < NV sums dof i, then the row broadcasts it
      vel();
#ifdef SOARM_PHASE_PROF
      if ((threadIdx.x & 63) == 0 && WPH_ID() < WPH_MAXW) {
        const long long rp2 = clock64();
        WPH_ADD(77, rp0 - g_pgs_prof[8 * e]);
        WPH_ADD(78, rp1 - rp0);
        WPH_ADD(79, rp2 - rp1);
        WPH_ADD(80, 1);
        WPH_ADD(81, wsw);
      }
#endif
    }
  };
  // wave-uniform choice: separate copies of the loop, no branch inside the sweep
  if constexpr (RS) {
    if (rs_fast) {
      using Z = std::integral_constant<int, 0>;
      using O = std::integral_constant<int, 1>;
      int kat = __any(rs_nat >= 1) ? 1 : 0, kac = __any(rs_nac >= 1) ? 1 : 0;
#ifdef SOARM_PHASE_PROF
      if (g_rs_force11) kat = kac = 1;  // (diagnostic: every RS wave in the (1, 1) layout)
#endif
      if (kac == 1 && kat == 1)
        rs_solve(O{}, O{});
      else if (kac == 1)
        rs_solve(Z{}, O{});
      else if (kat == 1)
        rs_solve(O{}, Z{});
      else
        rs_solve(Z{}, Z{});
    } else {
      sweeps(std::false_type{});
    }
  } else if (ypure) {
    ysweeps(std::false_type{}, std::false_type{}, std::false_type{});
  } else if (yext && yext2 && ycoupled) {
    ysweeps(std::true_type{}, std::true_type{}, std::true_type{});
  } else if (yext && yext2) {
    ysweeps(std::true_type{}, std::false_type{}, std::true_type{});
  } else if (yext && ycoupled) {
    ysweeps(std::true_type{}, std::true_type{}, std::false_type{});
  } else if (yext) {
    ysweeps(std::true_type{}, std::false_type{}, std::false_type{});
  } else if (block_first) {
    sweeps(std::true_type{});
  } else {
    sweeps(std::false_type{});
  }
  if (NF == 1 && CON && !rs_fast) {  // the block's forces back to their records (for J' f)
#pragma unroll
    for (int k = 0; k < FC; k++)
      if (k < nrun)
#pragma unroll
        for (int ed = 0; ed < 4; ed++) L.at(c0 + k, F_FRC + ed) = cfo[k][ed];
  }
  if constexpr (RS) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < NA * (NA + 1) / 2; i++) S.LH[i] = L.kp(k++);
#pragma unroll
    for (int i = 0; i < NA; i++) S.DHi[i] = L.kp(k++);
#pragma unroll
    for (int i = 0; i < 6 * NF; i++) S.kf[i / 6][i % 6] = L.kp(k++);
#pragma unroll
    for (int i = 0; i < 3; i++) S.ee[i] = L.kp(k++);
  } else if (L.keep) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < NA * (NA + 1) / 2; i++) S.MA[i] = L.kp(k++);
#pragma unroll
    for (int f2 = 0; f2 < NF; f2++)
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) S.MF[f2][i * (i + 1) / 2 + j] = (i == j) ? L.kp(k++) : 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) S.fsmooth[i] = L.kp(k++);
#pragma unroll
    for (int i = 0; i < 3; i++) S.ee[i] = L.kp(k++);
  }
#ifdef SOARM_PHASE_PROF
  if (e < 65536)
    g_pgs_prof[8 * e + 1] = clock64(), g_pgs_prof[8 * e + 2] = nsweep,
    g_pgs_prof[8 * e + 3] = (ypure ? 0 : yext ? 1 : block_first ? 2 : 3) | (npost > 0 && npost_free ? 16 : 0) |
                            (min(npost, 3) << 8) | (min(nfree_x, 3) << 12) | ((nl > 5) << 16) | ((nlim > 0) << 17) |
                            ((nl != ncon) << 18) | ((long long)min(armstop, 255) << 20) |
                            ((long long)(yext ? 4 + 2 * yext2 + ycoupled : 0) << 28) | ((long long)(RS && !rs_fast) << 40) | ((long long)rs_why << 41),
    g_pgs_prof[8 * e + 4] = nlim, g_pgs_prof[8 * e + 5] = ncon;
#endif

  // ---- qacc and qfrc_constraint = J' f
#pragma unroll
  for (int i = 0; i < NV; i++) {
    S.qacc[i] = v[i];
    S.fcon[i] = 0.f;
  }
  if constexpr (CON && RS) return ncon;  // (the RS kernel's Euler step needs qacc alone: integrate_qacc)
  if constexpr (CON) {
    // qacc = qacc_smooth + M^-1 J' f, so J' f = M qacc - qfrc_smooth (M qacc_smooth = qfrc_smooth):
    // the Euler step's right-hand side qfrc_smooth + qfrc_constraint is M qacc.  One 6x6 product
    // (+ the free bodies' diagonal blocks) instead of J' f over every contact row; equal in exact
    // arithmetic, fp32 rounding apart (the oracle keeps J' f).
#pragma unroll
    for (int i = 0; i < NA; i++) {
      float sacc = -S.fsmooth[i];
#pragma unroll
      for (int k = 0; k < NA; k++) sacc = fmaf(S.MA[i >= k ? i * (i + 1) / 2 + k : k * (k + 1) / 2 + i], v[k], sacc);
      S.fcon[i] = sacc;
    }
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const int d = NA + 6 * f + i;
        S.fcon[d] = fmaf(S.MF[f][i * (i + 1) / 2 + i], v[d], -S.fsmooth[d]);
      }
    return ncon;
  }
#pragma unroll
  for (int i = 0; i < NA; i++) S.fcon[i] += ff[i];
  for (int l = 0; l < nlim; l++) {
    float oh[NA];
    one_hot<NA>((int)L.lm(l, L_DOF), oh);
    const float t = L.lm(l, L_SGN) * L.lm(l, L_FRC);
#pragma unroll
    for (int k = 0; k < NA; k++) S.fcon[k] = fmaf(oh[k], t, S.fcon[k]);
  }
  for (int c = 0; c < nl; c++) {
    float jn[NV], jt1[NV], jt2[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) jn[i] = L.at(c, i), jt1[i] = L.at(c, 12 + i), jt2[i] = L.at(c, 24 + i);
    const float mu = L.at(c, F_MU);
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      float J[NV];
      edge_J<NV>(jn, jt1, jt2, ed, mu, J);
      const float fr = L.at(c, F_FRC + ed);
#pragma unroll
      for (int i = 0; i < NV; i++) S.fcon[i] += J[i] * fr;
    }
  }
  for (int r = 4 * nl; r < 4 * ncon; r++) {
    const float fr = cr.S(r, 3);
#pragma unroll
    for (int i = 0; i < NV; i++) S.fcon[i] += cr.J(r, i) * fr;
  }
  return ncon;
}

}  // namespace soarm
