// HIP kernels of the batched HSDDP solve for gfx950 (MI355X).
//
// One solve = a fixed host schedule of five kernels per DDP iteration (see
// mhpc_runtime.cpp), every kernel working on the whole batch and skipping problems whose
// per-problem state machine (ProbState) says they are done -- the divergent control flow
// of MultiPhaseDDP::solve (MultiPhaseDDP.cpp:154-289) lives in device memory, not on the
// host:
//   k_rollout  lane = (problem, line-search candidate).  forward_sweep(0) (FULL) or all
//              Armijo trials of forward_iteration (LS) at once, each lane a serial
//              multi-phase rollout with costs, barrier, AL and phase transitions; the
//              first accepted trial is selected in-wave (MultiPhaseDDP.cpp:130-151).
//   k_partials lane = (problem, WB knot, direction group): the knot's forward dynamics once,
//              then every column of A,B,C,D by implicit differentiation of the contact KKT
//              system (forward_sweep_partials_only, SinglePhase.cpp:147-180); the impact
//              Jacobian Px by dual numbers (k_partials_impact).
//   k_bws      one wavefront per problem: the backward Riccati sweep over all phases with
//              impact-aware steps and the regularisation-retry loop
//              (MultiPhaseDDP.cpp:100-127,196-241, SinglePhase.cpp:183-216,
//              MHPC_CompoundTypes.h:117-144).  Knot blocks (<= 14x14) are staged in LDS,
//              the 64 lanes split each product; no MFMA (blocks far below MFMA shapes).
//   k_al_end   AL / ReB parameter update and outer-loop exit (MultiPhaseDDP.cpp:273-284).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "mhpc_device.h"
#include "mhpc_model_pair.h"

namespace MHPC_NS {

// ============================================================================================
// k_rollout: forward_iteration (MultiPhaseDDP.cpp:130-151) -- every Armijo trial at once.
// Block = two waves working as a pipeline on the same 64 (problem, candidate) lanes:
//   wave 0  the serial multi-phase rollout u = (u_nom + eps du) + K (x - x_nom),
//           x+ = x + dt f(x, u), phase transitions (MultiPhaseDDP.cpp:351-379); each knot's
//           (x, u, y) goes to a two-deep LDS ring;
//   wave 1  one knot behind: running cost (summed in knot order, exactly the serial
//           association), terminal cost / AL / touchdown constraint, and the coalesced store
//           of every candidate's knot record to its trajectory slot.
// One barrier per knot hands the ring over; the cost and the scattered stores leave the
// dynamics chain.  At the end the first accepted trial of each problem is selected in-block.
// ============================================================================================
constexpr int RING_W = 22;  // reals per ring record (x 14, u 4, y 4)
#ifdef MHPC_FP32
using real2 = float2;
#else
using real2 = double2;
#endif

// Feedback term K[i] (x - x_nom) of the line-search control (SinglePhase.cpp forward sweep,
// u = u_nom + eps du + K dx), summed in column order.  (Summing the two halves of the row
// separately -- a chain half as long -- measured no faster: profiles/r02_ab_wt_layout.txt.)
template <int N>
__device__ __forceinline__ real fb_dot(const real* Kr, const real* x, const real* nk) {
  MHPC_NO_FMA_F32  // as in the kernels that call it (fp32 line search uncontracted)
  real fb = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) fb += Kr[c] * (x[c] - nk[c]);
  return fb;
}

// Line-search trials whose running knot records are stored (j < RO_STORE_FIRST, and the last
// trial, which the reference adopts when none is accepted); every trial stores its terminal
// states.  The Armijo test accepts an early trial almost always (CPU oracle, C3 x512: trial
// 1-4 or none; C5 x128: trial 2-5), and the record stores are a large part of a launch
// (MHPC_RO_STORE_FIRST=4 A/B: -25 % k_rollout per launch at batch 4096, -4 % at 1024).  An
// accepted trial without records is rolled out again into its slot right after the line
// search (k_rollout mode 2, same arithmetic: bit for bit).  The handle's sp.ro_store
// (mhpc_set_kernel_variant(MHPC_VARIANT_RO_STORE)) overrides it.
#ifndef MHPC_RO_STORE_FIRST
#define MHPC_RO_STORE_FIRST 4
#endif
constexpr int RO_STORE_FIRST = MHPC_RO_STORE_FIRST;
int ro_store_default() { return RO_STORE_FIRST; }

// Problems per block of the pair variant (at most 32 / n_cand = 3 with 10 candidates).
#ifndef MHPC_RO_PAIR_PPB
#define MHPC_RO_PAIR_PPB 3
#endif
constexpr int RO_PAIR_PPB = MHPC_RO_PAIR_PPB;

// Ring depth of the pair variant's dynamics -> cost hand-over: a barrier per RD / 2 records
// (2: per record; 4: per two; 8: per four -- the cost wave takes every record handed over
// since the last barrier, in knot order.  8 vs 4: line search 0.399 -> 0.394 ms per launch at
// batch 1024, equal at batch 1, interleaved A/B round 5)
#ifndef MHPC_RO_RING_PAIR
#define MHPC_RO_RING_PAIR 8
#endif
constexpr int RO_RING_PAIR = MHPC_RO_RING_PAIR;
#ifndef MHPC_RO_PREFETCH
#define MHPC_RO_PREFETCH 1
#endif
// The line search's dynamics keeps the sin / cos constants in registers (SinCosK)
#ifndef MHPC_RO_VCONST
#define MHPC_RO_VCONST 1
#endif

// native 2-wide vector (HIP's double2 class defeats register promotion of arrays of it)
typedef real sreal2 __attribute__((ext_vector_type(2)));
constexpr int ST_PPW = 6;      // problems per staged wave (64 lanes / 10 candidates)
constexpr int ST_PAIRS = 193;   // staged pairs per problem (192 + 1: problems on distinct LDS banks)

// Line-search staging (ST): the 10 candidates of a problem share its nominal, gains and
// references, so each wave loads them once per problem, cooperatively, one chunk of CH
// knots ahead into registers (3 coalesced 2-wide loads per lane and problem) and drops
// them into LDS at the next chunk boundary -- the serial knot chain then reads LDS instead
// of waiting on a global-load round trip per knot (measured ~1.4k cycles per WB knot and
// ~5k per SRB knot before, tools/ro_timing.py).  Per problem the stage holds 192 pairs:
// [0, 128) the gain rows K (4 nx reals per knot), [128, ...) the nominal x, u (nx + 4
// reals per knot) followed by du (4 reals per knot).  Load slots A / B (K) and C
// (nominal + du) fill pairs [0, 64), [64, 128) and [128, 192) lane-linearly.
template <bool WB>
struct Stage {
  static constexpr int NX = WB ? 14 : 6;
  static constexpr int KP = 2 * NX;            // K pairs per knot: 28 / 12
  static constexpr int TP = (NX + 4) / 2;      // nominal x,u pairs per knot: 9 / 5
  static constexpr int CH = WB ? 4 : 8;        // knots per chunk
  static constexpr int T0 = 128;               // first nominal pair
  static constexpr int D0 = T0 + CH * TP;      // first du pair: 164 / 168
  static_assert(CH * KP <= 128 && D0 + 2 * CH <= 192, "stage layout");
};

// Per-lane part of the stage addresses (reals from the problem's chunk base of each array)
// and the chunk knot of each load slot; -1: the lane has no item in that slot.
struct StageLane {
  int offA, offB, offC, kcA, kcB, kcC;
  bool trajC;
};
template <bool WB>
__device__ __forceinline__ StageLane stage_lane(int lane) {
  using S = Stage<WB>;
  StageLane L;
  const int pa = lane, pb = 64 + lane;
  L.kcA = pa / S::KP; L.offA = L.kcA * 56 + 2 * (pa - L.kcA * S::KP);
  L.kcB = pb / S::KP; L.offB = L.kcB * 56 + 2 * (pb - L.kcB * S::KP);
  if (pb >= S::CH * S::KP) L.kcB = -1;
  L.trajC = lane < S::CH * S::TP;
  if (L.trajC) {
    L.kcC = lane / S::TP; L.offC = L.kcC * KS + 2 * (lane - L.kcC * S::TP);
  } else {
    const int e = lane - S::CH * S::TP;
    L.kcC = e < 2 * S::CH ? e / 2 : -1;
    L.offC = 2 * e;
  }
  return L;
}

// Issue the loads of chunk [k0, k0 + CH) of phase (ko, nr rollout knots) into pf (pbv: the
// problem of each staged slot).  Every load is unconditional (lanes without an item re-read
// the chunk base, absent problems problem 0's): a masked load would merge with the register's old value and make the
// compiler wait for it on the spot, which is exactly the round trip the stage hides.
// NP: problem slots of the wave (ST_PPW; 3 in the pair variant, whose dynamics wave holds
// 3 problems x 10 candidates) -- slots past NP would only load problem 0's data again.
template <bool WB, int NP>
__device__ __forceinline__ void stage_issue(const SolveParams& sp, const DevBufs& d,
                                            const StageLane& L, const int (&pbv)[ST_PPW], int ko,
                                            int k0, int nr, const int (&nomv)[ST_PPW],
                                            sreal2 (&pf)[ST_PPW * 3]) {
  const int lim = nr - k0;  // chunk knots that exist
  const int oA = L.kcA < lim ? L.offA : 0;
  const int oB = L.kcB >= 0 && L.kcB < lim ? L.offB : 0;
  const int oC = L.kcC >= 0 && L.kcC < lim ? L.offC : 0;
#pragma unroll
  for (int lp = 0; lp < NP; ++lp) {
    const int nom = nomv[lp];  // < 0: problem absent or not iterating (uniform)
    const int bb = nom >= 0 ? pbv[lp] : 0;
    const size_t kk = (size_t)bb * sp.NK + ko + k0;
    const real* Kb = d.K + kk * 56;
    const real* Tb = traj_ptr(sp, d, bb, nom >= 0 ? nom : 0, ko + k0);
    const real* Db = d.du + kk * 4;
    pf[3 * lp] = *reinterpret_cast<const sreal2*>(Kb + oA);
    pf[3 * lp + 1] = *reinterpret_cast<const sreal2*>(Kb + oB);
    pf[3 * lp + 2] = *reinterpret_cast<const sreal2*>((L.trajC ? Tb : Db) + oC);
  }
}

// Drop a loaded chunk into the LDS stage (lane-linear per slot).
template <int NP>
__device__ __forceinline__ void stage_drop(int lane, const sreal2 (&pf)[ST_PPW * 3],
                                           sreal2* stage2) {
#pragma unroll
  for (int i = 0; i < NP * 3; ++i) stage2[(i / 3) * ST_PAIRS + (i % 3) * 64 + lane] = pf[i];
}

// Optional cycle accounting of the rollout's knot loop (build with -DMHPC_RO_TIMING, read
// with mhpc_dbg_ro_cycles; lane 0 of the dynamics wave of every block): 0 WB feedback u,
// 1 WB dynamics, 2 WB record hand-over (ring + barrier), 3 SRB knot, 4 / 5 WB / SRB knots.
#ifdef MHPC_RO_TIMING
__device__ unsigned long long g_ro_cyc[11];
#define RO_T(v) const unsigned long long v = (lane == 0 && w0) ? clock64() : 0ull
#define RO_ADD(i, v) do { if (lane == 0 && w0) ro_cyc[i] += (v); } while (0)
#else
#define RO_T(v) do { } while (0)
#define RO_ADD(i, v) do { } while (0)
#endif

// PIPE = false: the same wave plays both roles (no ring, registers hand over) -- better
// once the batch fills the chip, when a second wave per block only competes for issue.
// full = 1: forward_sweep(0) as a real rollout (one lane per problem, eps = 0, always
// adopted) -- needed when the nominal is not a rollout of its own controls from x0, i.e.
// after mhpc_update_problem (receding horizon); otherwise k_cost replaces it.
// full = 2: the line search's accepted trial again (eps of st->reroll_j from the nominal the
// line search started from, into the new nominal slot), records only, for the problems whose
// trial stored none (RO_STORE_FIRST).
// ST = true: the line search reads nominal / gains / references through the LDS stage
// (requires n_cand >= 10, i.e. <= ST_PPW problems per wave).
// PAIR (with PIPE and ST): the dynamics wave gives each candidate a lane pair (even lane
// front leg, odd lane back leg, mhpc_model_pair.h), 3 problems per block; the cost wave keeps
// one lane per candidate.  cl = the candidate's lane in the cost wave and in the ring.
template <bool PIPE, bool ST, bool PAIR>
__global__ __launch_bounds__(PIPE ? 128 : 64) void k_rollout(SolveParams sp, DevBufs d,
                                                             int al_iter, int ddp_iter,
                                                             int max_ddp, int full) {
  MHPC_NO_FMA_F32
  const int nc = full ? 1 : sp.n_cand;
  // (a staged re-roll, mode 2: one lane per problem and the stage's ST_PPW problems a block)
  const int ppw = PAIR ? min(32 / nc, RO_PAIR_PPB) : (ST && full == 2) ? ST_PPW : 64 / nc;
  constexpr int SNP = PAIR ? RO_PAIR_PPB : ST_PPW;  // staged problem slots (ppw <= SNP when staged)
  constexpr bool PF = PAIR && ST && MHPC_RO_PREFETCH;  // register prefetch of the next knot
  const int t = threadIdx.x, lane = t & 63;
  const bool w0 = PIPE ? (t >> 6) == 0 : true, w1 = PIPE ? (t >> 6) == 1 : true;
  const int cl = (PAIR && w0) ? (lane >> 1) : lane;
  const bool back = PAIR && (lane & 1);  // the dynamics lane's leg
  const int lp = cl / nc, j = cl - lp * nc;
  // the block's layout group and problems (a block never mixes layouts)
  const GrpBlk gb = block_group(sp, blockIdx.x, ppw);
  if (gb.g < 0) return;  // (uniform; the grid has no such block)
  const Layout& L = layout_of(d, gb.g);
  const bool in = lp < ppw && gb.p0 + lp < gb.p1;
  const int b = in ? prob_at(sp, d, gb.p0 + lp) : 0;

  // ring of RD knot records; the waves meet at a barrier every RD / 2 records
  constexpr int RD = PIPE ? (PAIR ? RO_RING_PAIR : 2) : 1;
  constexpr int RG = PIPE ? RD / 2 : 1;  // records per barrier
  static_assert(RG >= 1 && (RG & (RG - 1)) == 0, "ring depth");
  // (the pair variant's records belong to its <= 32 candidates: half the columns suffice; a
  // deeper ring takes them, the four-deep one keeps 64 -- with its LDS cut to 52 KB a third
  // block fits a CU and the line search measured 0.5 % slower)
  constexpr int RCOL = (PAIR && RD > 4) ? 32 : 64;
  __shared__ real ring[RD][RING_W][RCOL];
  __shared__ acc sJ[64], sViol[64], sV[MAXP][64];
  __shared__ real sH[MAXP][64];
  __shared__ int sAny;
  __shared__ int sNom[ST ? ST_PPW : 1], sProb[ST ? ST_PPW : 1];
  __shared__ sreal2 stage2[ST ? SNP * ST_PAIRS : 1];
  __shared__ real sRef[ST ? SNP : 1][ST ? ST_RMAX + 1 : 1];  // +1: distinct banks
#ifdef MHPC_RO_TIMING
  unsigned long long ro_cyc[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif

  if (t == 0) sAny = 0;
  if (ST && t < ST_PPW) { sNom[t] = -1; sProb[t] = 0; }
  __syncthreads();
  bool run = false;
  int nom = 0, slot = 0;
  ProbState* st = nullptr;
  if (in) {
    st = &d.st[b];
    if (full == 2) {  // re-roll of the accepted trial into the new nominal slot
      run = st->active && st->reroll_j >= 0;
      nom = st->reroll_nom;
      slot = st->nom_slot;
    } else {
      run = st->active && (full || st->ddp_active);
      nom = st->nom_slot;
      slot = j < nom ? j : j + 1;
    }
  }
  if (w0 && run) sAny = 1;
  if (ST && w0 && run && j == 0) { sNom[lp] = nom; sProb[lp] = b; }
  __syncthreads();
  int nomv[ST_PPW];  // nominal slot of each staged problem, -1 if absent / not iterating
  int pbv[ST_PPW];   // its problem index
#pragma unroll
  for (int i = 0; i < ST_PPW; ++i) {
    nomv[i] = ST ? __builtin_amdgcn_readfirstlane(sNom[i]) : -1;
    pbv[i] = ST ? __builtin_amdgcn_readfirstlane(sProb[i]) : 0;
  }
  if (!sAny) return;  // uniform: no problem of this block is still iterating
  if (full == 1 && run && w0) {  // top of the AL iteration (MultiPhaseDDP.cpp:172-190)
    if (al_iter == 1) { st->cap_reb = st->opt_reb; st->cap_pen = st->opt_pen; }
    const bool reb_off = (st->viol > real(0.05)) || al_iter == 1;
    st->reb_active = (st->cap_reb && !reb_off) ? 1 : 0;
    st->opt_reb = st->reb_active;
  }
  if (full) __syncthreads();

  // (mode 2 reads its step size from the state: a per-lane index into the parameter block
  // here made the compiler copy the whole block to scratch)
  const real eps = run && !full ? sp.eps[j] : run && full == 2 ? st->reroll_eps : real(0.0);
  const bool reb = run && st->reb_active;
  real x[14];
  if (w0 && run) {
    const real* x0 = d.x0 + (size_t)b * 14;
    for (int i = 0; i < 14; ++i) x[i] = x0[i];
  }
  acc J = 0, viol2 = 0;
  // wave 1: store the lane's ring record (n reals, n even) to knot kk of its slot with
  // 2-wide stores (records are aligned to them: KS * sizeof(real))
  auto store_rec = [&](const real* r, int n, int kk, bool running) __attribute__((always_inline)) {
#ifdef MHPC_RO_NOSTORE  // timing experiments only: results are wrong
#if MHPC_RO_NOSTORE == 1
    if (kk >= 0) return;
#else
    n = n < 2 * MHPC_RO_NOSTORE ? n : 2 * MHPC_RO_NOSTORE;  // the first pieces only
#endif
#endif
    if (running && !full && j >= sp.ro_store && j != nc - 1) return;  // see RO_STORE_FIRST
    real2* o = reinterpret_cast<real2*>(traj_ptr(sp, d, b, slot, kk));
#pragma unroll
    for (int i = 0; i < RING_W / 2; ++i)
      if (2 * i < n) o[i] = real2{r[2 * i], r[2 * i + 1]};
  };
  real f[4] = {0, 0, 0, 0}, sc[2] = {0, 0};  // SRB phase: foothold, contact flags
  sreal2 pf[ST_PPW * 3];                    // the next chunk's stage loads in flight
  // PF (pair variant): the feedback operands of knot k+1 (own K rows, nominal x / u, du) are
  // read from the stage into registers at the end of knot k, so their LDS latency overlaps
  // the hand-over instead of heading the next knot's dependent chain; the next chunk is
  // dropped into the stage right after the last knot of a chunk has read it.
  real pK[28], pX[14], pU[4], pD[4];
  // sin / cos constants: VGPR copies (opaque to the compiler, so it keeps them live instead of
  // rematerialising each with two s_mov per use in the knot loop)
  SinCosK scK = kSinCosK;
#if MHPC_RO_VCONST && !defined(MHPC_FP32)
#pragma unroll
  for (int i = 0; i < 15; ++i) asm volatile("" : "+v"(scK.c[i]));
#endif
  auto prefetch = [&](bool wb, int kk) __attribute__((always_inline)) {
    const int kcc = kk & ((wb ? Stage<true>::CH : Stage<false>::CH) - 1);
    const int KP = wb ? Stage<true>::KP : Stage<false>::KP, TP = wb ? Stage<true>::TP : Stage<false>::TP;
    const int D0 = wb ? Stage<true>::D0 : Stage<false>::D0;
    const real* sgp = reinterpret_cast<const real*>(stage2 + lp * ST_PAIRS);
    const real* nk = sgp + 2 * (Stage<true>::T0 + kcc * TP);
    const real* Kk = sgp + 2 * kcc * KP;
    const real* duk = sgp + 2 * (D0 + 2 * kcc);
    if (wb) {
      const int r0 = back ? 2 : 0;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
        for (int c = 0; c < 14; ++c) pK[ii * 14 + c] = Kk[(r0 + ii) * 14 + c];
        pU[ii] = nk[14 + r0 + ii];
        pD[ii] = duk[r0 + ii];
      }
#pragma unroll
      for (int c = 0; c < 14; ++c) pX[c] = nk[c];
    } else if (PAIR) {  // SRB: the pair splits the four control rows (even u0, u1; odd u2, u3)
      const int r0 = back ? 2 : 0;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
        for (int c = 0; c < 6; ++c) pK[ii * 6 + c] = Kk[(r0 + ii) * 6 + c];
        pU[ii] = nk[6 + r0 + ii];
        pD[ii] = duk[r0 + ii];
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) pX[c] = nk[c];
    } else {
#pragma unroll
      for (int i = 0; i < 24; ++i) pK[i] = Kk[i];
#pragma unroll
      for (int c = 0; c < 6; ++c) pX[c] = nk[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) { pU[i] = nk[6 + i]; pD[i] = duk[i]; }
    }
  };
  // drop the loaded chunk (knots k1..) into the stage and fetch the next one (all lanes of
  // the dynamics wave: the loads are cooperative)
  auto chunk_turn = [&](bool wb, int ko, int N, int k1) __attribute__((always_inline)) {
    const int CH = wb ? Stage<true>::CH : Stage<false>::CH;
    stage_drop<SNP>(lane, pf, stage2);
    if (k1 + CH < N - 1) {
      const StageLane SL = wb ? stage_lane<true>(lane) : stage_lane<false>(lane);
      if (wb) stage_issue<true, SNP>(sp, d, SL, pbv, ko, k1 + CH, N - 1, nomv, pf);
      else stage_issue<false, SNP>(sp, d, SL, pbv, ko, k1 + CH, N - 1, nomv, pf);
    }
  };
  // dynamics side, phase start: SRB foothold / contact, first chunk of the stage
  // (the phase kind WBc is a compile-time argument of every per-phase / per-knot helper: each
  // knot loop is specialised per kind, and a run-time p < n_wb here would make the compiler
  // keep both kinds' code inside each loop)
  auto dyn_phase_begin = [&](auto WBc, int p) __attribute__((always_inline)) {
    const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    constexpr bool wb = decltype(WBc)::value;
    if (run && !wb) {
      plan_foothold(x, L.dt[p] * N, mode, f);
      srb_contact(mode, sc);
    }
    if (ST) {
      const StageLane SL = wb ? stage_lane<true>(lane) : stage_lane<false>(lane);
      if (wb) stage_issue<true, SNP>(sp, d, SL, pbv, ko, 0, N - 1, nomv, pf);
      else stage_issue<false, SNP>(sp, d, SL, pbv, ko, 0, N - 1, nomv, pf);
    }
    if (PF) {
      chunk_turn(wb, ko, N, 0);
      if (run) prefetch(wb, 0);
    }
  };
  // dynamics side, knot k of phase p: u = (u_nom + eps du) + K (x - x_nom), x+ = x + dt f(x, u);
  // rr = the knot's record (x, u, y) as the ring / the cost side takes it
  auto dyn_knot = [&](auto WBc, int p, int k, real* rr) __attribute__((always_inline)) {
    const int mode = L.mode[p], ko = L.ko[p];
    const real dt = L.dt[p];
    constexpr bool wb = decltype(WBc)::value;
    const int kc = k & ((wb ? Stage<true>::CH : Stage<false>::CH) - 1);
    const int KP = wb ? Stage<true>::KP : Stage<false>::KP, TP = wb ? Stage<true>::TP : Stage<false>::TP;
    const int D0 = wb ? Stage<true>::D0 : Stage<false>::D0;
    const real* sgp = reinterpret_cast<const real*>(stage2 + lp * ST_PAIRS);
    const real* nk = ST ? sgp + 2 * (Stage<true>::T0 + kc * TP) : traj_ptr(sp, d, b, nom, ko + k);
    const real* Kk = ST ? sgp + 2 * kc * KP : d.K + ((size_t)b * sp.NK + ko + k) * 56;
    const real* duk = ST ? sgp + 2 * (D0 + 2 * kc) : d.du + ((size_t)b * sp.NK + ko + k) * 4;
    if (wb && PAIR) {
      // the state-only part of the dynamics first: the feedback operands (prefetched from the
      // LDS stage at the end of the previous knot) land meanwhile
      WbPairPrep P;
      wb_pair_prep(x, back, P, scK);
      // the own leg's two torques (rows 2 back, 2 back + 1 of K)
      real u2[2];
      if (PF) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const real fb = fb_dot<14>(pK + ii * 14, x, pX);
          u2[ii] = (pU[ii] + eps * pD[ii]) + fb;
        }
      } else {
        const int r0 = back ? 2 : 0;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const real fb = fb_dot<14>(Kk + (r0 + ii) * 14, x, nk);
          u2[ii] = (nk[14 + r0 + ii] + eps * duk[r0 + ii]) + fb;
        }
      }
      real xd[14], y[4];
      wb_pair_finish(x, u2, mode, back, P, xd, y);
      // ring record split over the pair: x[7 back .. 7 back + 6], own u, own-slot y
#pragma unroll
      for (int i = 0; i < 7; ++i) rr[i] = back ? x[7 + i] : x[i];
      rr[7] = u2[0]; rr[8] = u2[1];
      rr[9] = back ? y[2] : y[0];
      rr[10] = back ? y[3] : y[1];
#pragma unroll
      for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
    } else if (wb) {
      real u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const real fb = fb_dot<14>(Kk + i * 14, x, nk);
        u[i] = (nk[14 + i] + eps * duk[i]) + fb;
      }
      real xd[14], y[4];
      wb_dynamics<real>(x, u, mode, xd, y, scK);
#pragma unroll
      for (int i = 0; i < 14; ++i) rr[i] = x[i];
#pragma unroll
      for (int i = 0; i < 4; ++i) { rr[14 + i] = u[i]; rr[18 + i] = y[i]; }
#pragma unroll
      for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
    } else {
      real u[4];
      if (PF && PAIR) {  // own two control rows, then the partner's by in-pair broadcasts
        real uo[2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const real fb = fb_dot<6>(pK + ii * 6, x, pX);
          uo[ii] = (pU[ii] + eps * pD[ii]) + fb;
        }
        u[0] = pair_from<0>(uo[0]);
        u[1] = pair_from<0>(uo[1]);
        u[2] = pair_from<1>(uo[0]);
        u[3] = pair_from<1>(uo[1]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const real fb = PF ? fb_dot<6>(pK + i * 6, x, pX) : fb_dot<6>(Kk + i * 6, x, nk);
          u[i] = PF ? (pU[i] + eps * pD[i]) + fb : (nk[6 + i] + eps * duk[i]) + fb;
        }
      }
      real xd[6];
      srb_dynamics(x, u, f, sc, xd);
#pragma unroll
      for (int i = 0; i < 6; ++i) rr[i] = x[i];
#pragma unroll
      for (int i = 0; i < 4; ++i) { rr[6 + i] = u[i]; rr[10 + i] = real(0.0); }
      if (PAIR) {  // the pair splits the 14 record entries: 0..6 even lane, 7..13 odd
#pragma unroll
        for (int i = 0; i < 7; ++i) rr[i] = back ? rr[7 + i] : rr[i];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) x[i] = x[i] + xd[i] * dt;
    }
  };
  // phase transition after the phase's terminal state (MultiPhaseDDP.cpp:351-379)
  auto transition = [&](auto WBc, int p) __attribute__((always_inline)) {
    const int mode = L.mode[p];
    if (decltype(WBc)::value && p + 1 < L.P) {
      if (mode == 2 || mode == 4) {
        real xp[14], lam[2];
        wb_impact<real>(x, mode == 2 ? kFront : kBack, xp, lam);
        for (int i = 0; i < 14; ++i) x[i] = xp[i];
      }
      if (p + 1 >= L.n_wb) {
        const real t0 = x[0], t1 = x[1], t2 = x[2], t7 = x[7], t8 = x[8], t9 = x[9];
        x[0] = t0; x[1] = t1; x[2] = t2; x[3] = t7; x[4] = t8; x[5] = t9;
      }
    }
  };
  // cost side, phase constants: ReB parameters and the staged position references
  struct CostPhase {
    real delta, etq, egr, refT;
    const __attribute__((address_space(1))) real* refpos;  // global (not a flat pointer)
  };
  // Position references of phase (N, ko) into the LDS stage (cost side: one wave writes and
  // reads them).  The staged variants read every knot's reference from LDS and run only when
  // every phase fits the stage (launch_rollout): a global load in the cost loop would be a
  // VM-counter wait, and on gfx950's single in-order counter that wait also covers every
  // record store issued before it -- which was most of the stores' cost in the line search.
  auto stage_ref = [&](int N, int ko) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < SNP * ST_RMAX / 64; ++i) {
      const int fi = lane + 64 * i, rl = fi / ST_RMAX, rk = fi - rl * ST_RMAX;
      if (rk < N && sNom[rl] >= 0) sRef[rl][rk] = d.refpos[(size_t)sProb[rl] * sp.NK + ko + rk];
    }
  };
  auto cost_phase_begin = [&](auto WBc, int p) __attribute__((always_inline)) {
    CostPhase c;
    const int N = L.N[p], ko = L.ko[p];
    constexpr bool wb = decltype(WBc)::value;
    c.delta = c.etq = c.egr = real(0.0);
    if (run && wb) { c.delta = st->delta[p]; c.etq = st->eps_tq[p]; c.egr = st->eps_grf[p]; }
    c.refpos = (const __attribute__((address_space(1))) real*)(d.refpos + (size_t)(in ? b : 0) * sp.NK + ko);
    c.refT = run ? c.refpos[N - 1] : real(0.0);
    if (ST) stage_ref(N, ko);
    return c;
  };
  // cost side: the running cost of knot kk from record r (knot order: the serial rollout's
  // association) and the record's store
  auto cost_knot = [&](auto WBc, int p, const CostPhase& c, int kk, const real* r, acc& V) __attribute__((always_inline)) {
    MHPC_NO_FMA_COST
    const int mode = L.mode[p], ko = L.ko[p];
    const real dt = L.dt[p];
    constexpr bool wb = decltype(WBc)::value;
    const real pos = ST ? sRef[lp][kk] : c.refpos[kk];
    if (full != 2)  // (a re-roll only writes the records)
      V += wb ? wb_running_cost(sp, mode, dt, pos, r, r + 14, r + 18, reb, c.delta, c.etq, c.egr)
              : fb_running_cost(sp, mode, dt, pos, r, r + 6);
    store_rec(r, wb ? RING_W : 14, ko + kk, true);
  };
  auto ring_rec = [&](int sl, real* r, int n) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < RING_W; ++i) r[i] = i < n ? ring[sl][i][lane] : real(0.0);
  };
  // terminal cost of an SRB phase (CostBase.cpp:37-47): 0.5 (x - xr)' Qf (x - xr)
  auto srb_terminal_cost = [&](int mode, real refT, const real* xe) __attribute__((always_inline)) {
    MHPC_NO_FMA_COST
    real rx[6];
    fb_term_ref(sp, refT, rx);
    acc Phi = 0;
    for (int i = 0; i < 6; ++i) { const real e = xe[i] - rx[i]; Phi += e * sp.cw.fQf[mode - 1][i] * e; }
    return Phi * acc(0.5);
  };
  // cost side, phase end: terminal cost, touchdown constraint, AL term (SinglePhase.cpp
  // :251-275), the phase value into sV / sH and the terminal record's store
  auto cost_terminal = [&](auto WBc, int p, const CostPhase& c, const real* xe, acc V) __attribute__((always_inline)) {
    MHPC_NO_FMA_COST
    const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    constexpr bool wb = decltype(WBc)::value;
    if (full == 2) {
      store_rec(xe, wb ? 14 : 6, ko + N - 1, false);
      return;
    }
    real h = 0;
    if (wb) {
      real rx[14];
      wb_term_ref(sp, mode, c.refT, rx);
      acc Phi = 0;
      for (int i = 0; i < 14; ++i) { const real e = xe[i] - rx[i]; Phi += e * sp.cw.wQf[mode - 1][i] * e; }
      Phi = Phi * acc(0.5);
      if (ntc_of(mode, true)) {
        h = mode == 2 ? wb_touchdown_value<kFront>(xe) : wb_touchdown_value<kBack>(xe);
        if (sp.AL_active) {
          const acc sg = st->sigma[p], lam = st->lambda[p];
          const acc sh2 = sg * h / 2;
          Phi += 50 * (sh2 * sh2 + lam * h);
        }
      }
      V += Phi;
    } else {
      V += srb_terminal_cost(mode, c.refT, xe);
    }
    J += V;
    viol2 += acc(h) * h;
    sV[p][lane] = V;
    sH[p][lane] = h;
    store_rec(xe, wb ? 14 : 6, ko + N - 1, false);
  };

  if constexpr (PIPE) {
    // Two waves on the same (problem, candidate) lanes, each in its own loop (disjoint
    // register live ranges): wave 0 rolls out and hands each knot record over through a
    // ring of RD records, wave 1 takes them RG at a time after a barrier.  Both loops walk the
    // same record sequence, so their barriers pair up.
    int q = 0;
    if (w0) {
      // one copy of the knot loop per phase kind (WB / SRB): no joins of the two kinds'
      // registers inside the loop (those forced the prefetched operands to land early)
      auto dyn_phase = [&](auto WBc, int p) __attribute__((always_inline)) {
        constexpr bool wb = decltype(WBc)::value;
        const int N = L.N[p], ko = L.ko[p];
        constexpr int nx = wb ? 14 : 6;
        dyn_phase_begin(WBc, p);
        for (int k = 0; k < N - 1; ++k, ++q) {
          const int s = q & (RD - 1);
          const bool bar = (q & (RG - 1)) == RG - 1;
          real rr[RING_W];
          const int CH = wb ? Stage<true>::CH : Stage<false>::CH;
          RO_T(tk0);
          if (ST && !PF && (k & (CH - 1)) == 0) chunk_turn(wb, ko, N, k);
          RO_T(tkc);
          if (run) dyn_knot(WBc, p, k, rr);
          RO_T(tk2);
          if (PF && k + 1 < N - 1) {
            if (((k + 1) & (CH - 1)) == 0) chunk_turn(wb, ko, N, k + 1);
            if (run) prefetch(wb, k + 1);
          }
          if (run) {
            if (PAIR) {
              // WB: x half (7), u pair (2), y pair (2); SRB: half of the 14 entries
              if (wb) {
#pragma unroll
                for (int i = 0; i < 7; ++i) ring[s][(back ? 7 : 0) + i][cl] = rr[i];
                ring[s][back ? 16 : 14][cl] = rr[7];
                ring[s][back ? 17 : 15][cl] = rr[8];
                ring[s][back ? 20 : 18][cl] = rr[9];
                ring[s][back ? 21 : 19][cl] = rr[10];
              } else {
#pragma unroll
                for (int i = 0; i < 7; ++i) ring[s][(back ? 7 : 0) + i][cl] = rr[i];
              }
            } else {
#pragma unroll
              for (int i = 0; i < RING_W; ++i)
                if (i < (wb ? RING_W : 14)) ring[s][i][lane] = rr[i];
            }
          }
          if (bar) __syncthreads();
#ifdef MHPC_RO_TIMING
          if (lane == 0 && run) {
            const unsigned long long tk3 = clock64();
            ro_cyc[wb ? 1 : 7] += tk2 - tkc;
            ro_cyc[wb ? 2 : 8] += tk3 - tk2;
            ro_cyc[9] += tkc - tk0;
            if (wb) ro_cyc[4]++; else { ro_cyc[5]++; ro_cyc[3] += tk3 - tk0; }
          }
#endif
        }
        // the phase's terminal state into the ring, then the transition
        const int s = q & (RD - 1);
        ++q;
        if (run) {
          if (PAIR) {
#pragma unroll
            for (int i = 0; i < 7; ++i) {
              const int e = (back ? 7 : 0) + i;
              if (e < nx) ring[s][e][cl] = back ? x[7 + i] : x[i];
            }
          } else {
            for (int i = 0; i < nx; ++i) ring[s][i][lane] = x[i];
          }
          transition(WBc, p);
        }
        __syncthreads();
      };
      for (int p = 0; p < L.P; ++p) {
        if (p < L.n_wb) dyn_phase(std::true_type{}, p);
        else dyn_phase(std::false_type{}, p);
      }
    } else {
      auto cost_phase = [&](auto WBc, int p) __attribute__((always_inline)) {
        constexpr bool wb = decltype(WBc)::value;
        const int N = L.N[p];
        constexpr int nrec = wb ? RING_W : 14;
        const CostPhase c = cost_phase_begin(WBc, p);
        acc V = 0;
        int npend = 0;  // knot records handed over since the last barrier, not consumed yet
        for (int k = 0; k < N - 1; ++k, ++q) {
          const int s = q & (RD - 1);
          const bool bar = (q & (RG - 1)) == RG - 1;
          if (bar) {
#ifdef MHPC_RO_TIMING
            const unsigned long long ta = lane == 0 ? clock64() : 0ull;
#endif
            __syncthreads();
#ifdef MHPC_RO_TIMING
            const unsigned long long tb = lane == 0 ? clock64() : 0ull;
#endif
            if (run) {
              real r[RING_W];
              for (int i = npend; i >= 1; --i) {  // (knot order: the serial rollout's sum)
                ring_rec((s - i) & (RD - 1), r, nrec);
                cost_knot(WBc, p, c, k - i, r, V);
              }
              ring_rec(s, r, nrec);
              cost_knot(WBc, p, c, k, r, V);
            }
#ifdef MHPC_RO_TIMING
            if (lane == 0 && run) {  // cost wave: barrier wait, consume time per WB / SRB record
              const unsigned long long tc = clock64() + (unsigned long long)(V != V);
              ro_cyc[10] += tb - ta;
              ro_cyc[wb ? 0 : 6] += tc - tb;
            }
#endif
          }
          npend = bar ? 0 : npend + 1;  // (< RG)
        }
        const int s = q & (RD - 1);
        ++q;
        __syncthreads();
        if (run) {
          real r[RING_W];
          for (int i = npend; i >= 1; --i) {  // the phase's last knot records still waiting
            ring_rec((s - i) & (RD - 1), r, nrec);
            cost_knot(WBc, p, c, N - 1 - i, r, V);
          }
          ring_rec(s, r, wb ? 14 : 6);
          cost_terminal(WBc, p, c, r, V);
        }
      };
      for (int p = 0; p < L.P; ++p) {
        if (p < L.n_wb) cost_phase(std::true_type{}, p);
        else cost_phase(std::false_type{}, p);
      }
    }
  } else {
    // one wave: the rollout and the costs of each knot in turn (records in registers), one
    // copy of the knot loop per phase kind
    auto fused_phase = [&](auto WBc, int p) __attribute__((always_inline)) {
      constexpr bool wb = decltype(WBc)::value;
      const int N = L.N[p], ko = L.ko[p];
      constexpr int CH = wb ? Stage<true>::CH : Stage<false>::CH;
      dyn_phase_begin(WBc, p);
      const CostPhase c = cost_phase_begin(WBc, p);
      acc V = 0;
      for (int k = 0; k < N - 1; ++k) {
        if (ST && (k & (CH - 1)) == 0) chunk_turn(wb, ko, N, k);
        if (run) {
          real rr[RING_W];
          dyn_knot(WBc, p, k, rr);
          if (!wb) {
#pragma unroll
            for (int i = 6; i < RING_W; ++i) rr[i] = i < 14 ? rr[i] : real(0.0);
          }
          cost_knot(WBc, p, c, k, rr, V);
        }
      }
      if (run) {
        real xe[RING_W];
#pragma unroll
        for (int i = 0; i < RING_W; ++i) xe[i] = i < (wb ? 14 : 6) ? x[i] : real(0.0);
        transition(WBc, p);
        cost_terminal(WBc, p, c, xe, V);
      }
    };
    for (int p = 0; p < L.P; ++p) {
      if (p < L.n_wb) fused_phase(std::true_type{}, p);
      else fused_phase(std::false_type{}, p);
    }
  }
  if (w1 && run) {
    sJ[lane] = J;
    sViol[lane] = sqrt(viol2);
  }
  __syncthreads();
#ifdef MHPC_RO_TIMING
  if (lane == 0)
    for (int i = 0; i < 11; ++i) atomicAdd(&g_ro_cyc[i], ro_cyc[i]);
#endif
  if (full == 2) {
    if (w1 && run) st->reroll_j = -1;
    return;
  }
  if (full) {
    if (w1 && run) {
      st->J = J;
      st->viol = sqrt(viol2);
      for (int p = 0; p < L.P; ++p) { st->V[p] = sV[p][lane]; st->h[p] = sH[p][lane]; }
      st->nom_slot = slot;
      st->par_slot = slot;
      st->par_al = sp.AL_active ? 1 : 0;
      st->ls_nt = 0;
      for (int p = 0; p < L.P; ++p) { st->par_sigma[p] = st->sigma[p]; st->par_lambda[p] = st->lambda[p]; }
      st->al_iter = al_iter;
      st->reg = 0;
      st->ddp_active = 1;
      st->al_partials = 1;
      st->cnt[C_FWD]++;
      st->cnt[C_PAR_RUN]++;
    }
    return;
  }
  if (w1 && run && j == 0) {
    const acc cost_prev = st->J;
    int sel = nc - 1, nls = nc + 1;
    for (int c = 0; c < nc; ++c) {
      const real e = sp.eps[c];
      const acc rhs = cost_prev + sp.gamma * e * (1 - e / 2) * st->dV_exp;
      if (sJ[lane + c] <= rhs) { sel = c; nls = c + 1; break; }
    }
    const int sl = lane + sel;
    st->reroll_j = (sel >= sp.ro_store && sel != nc - 1) ? sel : -1;
    st->reroll_nom = nom;
    st->reroll_eps = sp.eps[sel];
    st->J = sJ[sl];
    st->viol = sViol[sl];
    for (int p = 0; p < L.P; ++p) { st->V[p] = sV[p][sl]; st->h[p] = sH[p][sl]; }
    st->nom_slot = sel < nom ? sel : sel + 1;
    const bool conv = cost_prev - st->J < sp.DDP_thresh;
    if (st->ntrace < TRACE)
      st->trace[st->ntrace++] = (al_iter << 24) | (st->reb_active << 23) | ((conv ? 1 : 0) << 22) |
                                ((nls & 0xff) << 8) | (st->bws_iter & 0xff);
    st->cnt[C_LS] += nls < nc ? nls : nc;
    st->cnt[C_LS_RUN] += nc;
    st->cnt[C_LS_LAUNCH]++;
    if (conv) {
      st->ddp_active = 0;
      st->ls_nt = nls < nc ? nls : nc;  // trials whose AL terms stay in Phix (see ProbState)
      st->ls_nom = nom;
      for (int p = 0; p < L.P; ++p) { st->ls_sigma[p] = st->sigma[p]; st->ls_lambda[p] = st->lambda[p]; }
    } else {
      st->cnt[C_PAR]++;
      st->al_partials = 0;
      st->par_slot = st->nom_slot;  // forward_sweep_partials_only (no AL terms, B1)
      st->par_al = 0;
      st->ls_nt = 0;
      if (ddp_iter < max_ddp) st->cnt[C_PAR_RUN]++;
      else st->ddp_active = 0;
    }
  }
}

// ============================================================================================
// k_eps_rollout: forward_sweep_dynamics_only (SinglePhase.cpp:117-144) at an arbitrary list
// of step sizes from the current nominal, gains and AL / ReB state, costs only (no stores,
// no selection): the trial rollouts of forward_iteration without the Armijo stop -- the
// C2 workload (256 concurrent rollouts of one nominal).  Lane = (problem, step size).
// ============================================================================================
__global__ __launch_bounds__(64) void k_eps_rollout(SolveParams sp, DevBufs d, int n_eps,
                                                    const real* eps_v, real* Jo,
                                                    real* vo) {
  // blocks by layout group, lanes = (problem of the group, step size)
  long t0 = 0;
  const int g = block_group_items(sp, nullptr, n_eps, blockIdx.x, 64, &t0);
  if (g < 0) return;
  const Layout& L = layout_of(d, g);
  const long tg = t0 + threadIdx.x;  // item within the group
  if (tg >= (long)(sp.go[g + 1] - sp.go[g]) * n_eps) return;
  const int pos = sp.go[g] + (int)(tg / n_eps), e = (int)(tg % n_eps);
  const int b = prob_at(sp, d, pos);
  const long t = (long)b * n_eps + e;  // output index [problem][step size]
  const ProbState* st = &d.st[b];
  const int nom = st->nom_slot;
  const real eps = eps_v[e];
  const bool reb = st->reb_active != 0;
  real x[14];
  const real* x0 = d.x0 + (size_t)b * 14;
  for (int i = 0; i < 14; ++i) x[i] = x0[i];
  acc J = 0, viol2 = 0;
  for (int p = 0; p < L.P; ++p) {
    const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    const real dt = L.dt[p];
    const real* refpos = d.refpos + (size_t)b * sp.NK + ko;
    acc V = 0;
    real h = 0;
    if (p < L.n_wb) {
      const real delta = st->delta[p], etq = st->eps_tq[p], egr = st->eps_grf[p];
      for (int k = 0; k < N - 1; ++k) {
        const real* nk = traj_ptr(sp, d, b, nom, ko + k);
        const real* Kk = d.K + ((size_t)b * sp.NK + ko + k) * 56;
        const real* duk = d.du + ((size_t)b * sp.NK + ko + k) * 4;
        real u[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const real fb = fb_dot<14>(Kk + i * 14, x, nk);
          u[i] = (nk[14 + i] + eps * duk[i]) + fb;
        }
        real xd[14], y[4];
        wb_dynamics<real>(x, u, mode, xd, y);
        V += wb_running_cost(sp, mode, dt, refpos[k], x, u, y, reb, delta, etq, egr);
#pragma unroll
        for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
      }
      {
        MHPC_NO_FMA_COST
        real rx[14];
        wb_term_ref(sp, mode, refpos[N - 1], rx);
        acc Phi = 0;
        for (int i = 0; i < 14; ++i) { const real ee = x[i] - rx[i]; Phi += ee * sp.cw.wQf[mode - 1][i] * ee; }
        Phi = Phi * acc(0.5);
        if (ntc_of(mode, true)) {
          h = mode == 2 ? wb_touchdown_value<kFront>(x) : wb_touchdown_value<kBack>(x);
          if (sp.AL_active) {
            const acc sg = st->sigma[p], lam = st->lambda[p];
            const acc sh2 = sg * h / 2;
            Phi += 50 * (sh2 * sh2 + lam * h);
          }
        }
        V += Phi;
      }
      if (p + 1 < L.P) {
        if (mode == 2 || mode == 4) {
          real xp[14], lam[2];
          wb_impact<real>(x, mode == 2 ? kFront : kBack, xp, lam);
          for (int i = 0; i < 14; ++i) x[i] = xp[i];
        }
        if (p + 1 >= L.n_wb) {
          const real t0 = x[0], t1 = x[1], t2 = x[2], t7 = x[7], t8 = x[8], t9 = x[9];
          x[0] = t0; x[1] = t1; x[2] = t2; x[3] = t7; x[4] = t8; x[5] = t9;
        }
      }
    } else {
      real f[4], sc[2];
      plan_foothold(x, dt * N, mode, f);
      srb_contact(mode, sc);
      for (int k = 0; k < N - 1; ++k) {
        const real* nk = traj_ptr(sp, d, b, nom, ko + k);
        const real* Kk = d.K + ((size_t)b * sp.NK + ko + k) * 56;
        const real* duk = d.du + ((size_t)b * sp.NK + ko + k) * 4;
        real u[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const real fb = fb_dot<6>(Kk + i * 6, x, nk);
          u[i] = (nk[6 + i] + eps * duk[i]) + fb;
        }
        real xd[6];
        srb_dynamics(x, u, f, sc, xd);
        V += fb_running_cost(sp, mode, dt, refpos[k], x, u);
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = x[i] + xd[i] * dt;
      }
      real rx[6];
      fb_term_ref(sp, refpos[N - 1], rx);
      acc Phi = 0;
      for (int i = 0; i < 6; ++i) { const real ee = x[i] - rx[i]; Phi += ee * sp.cw.fQf[mode - 1][i] * ee; }
      V += Phi * acc(0.5);
    }
    J += V;
    viol2 += acc(h) * h;
  }
  Jo[t] = real(J);
  vo[t] = real(sqrt(viol2));
}

// ============================================================================================
// k_cost_grad: the running-cost gradient lx of every knot and the terminal-cost gradient
// Phix of phase p as the last partials evaluation left them (rcost[k].lx, tcost.Phix;
// CostBase.cpp:19-31,49-60 + the AL term of SinglePhase.cpp:257-275 when it was a
// forward_sweep(0)), for print_debugInfo's cost.txt.  The constraint terms added to lx are
// exact zeros (joint limits carry eps_ReB = 0; torque / GRF limits do not depend on x).
// Problems [b0, b0 + nb), all of layout g; lane = (problem, knot); lx [nb][N-1][n], phix [nb][n].
// ============================================================================================
__global__ void k_cost_grad(SolveParams sp, DevBufs d, int g, int p, int b0, int nb, real* lx,
                            real* phix) {
  const Layout& L = layout_of(d, g);
  const int N = L.N[p], ko = L.ko[p], mode = L.mode[p];
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)nb * N) return;
  const int i0 = (int)(t / N), k = (int)(t - (long)i0 * N), b = b0 + i0;
  const ProbState* st = &d.st[b];
  const bool wb = p < L.n_wb;
  const int n = wb ? 14 : 6;
  const real dt = L.dt[p];
  const real* x = traj_ptr(sp, d, b, st->par_slot, ko + k);
  const real pos = d.refpos[(size_t)b * sp.NK + ko + k];
  if (k < N - 1) {
    real* o = lx + ((size_t)i0 * (N - 1) + k) * n;
    for (int i = 0; i < n; ++i) {
      real rxi, w2;
      if (wb) {
        rxi = i == 0 ? pos : i == 1 ? sp.height : i == 2 ? real(0.0)
              : i < 7 ? cQjointBias[i - 3] : i == 7 ? sp.vel : real(0.0);
        w2 = 2 * dt * sp.cw.wQ[mode - 1][i];
      } else {
        rxi = i == 0 ? pos : i == 1 ? sp.height : i == 3 ? sp.vel : real(0.0);
        w2 = 2 * dt * sp.cw.fQ[mode - 1][i];
      }
      o[i] = w2 * (x[i] - rxi);
    }
  } else {
    real* o = phix + (size_t)i0 * n;
    if (wb) {
      real rx[14];
      wb_term_ref(sp, mode, pos, rx);
      const bool al = ntc_of(mode, true) && st->par_al;
      real h = 0, hx[14], Hs[3][3];
      if (al) {
        if (mode == 2) wb_touchdown_compact<kFront>(x, &h, hx, Hs);
        else wb_touchdown_compact<kBack>(x, &h, hx, Hs);
      }
      const real s = st->par_sigma[p], lam = st->par_lambda[p];
      real v[14];
      for (int i = 0; i < 14; ++i) {
        v[i] = sp.cw.wQf[mode - 1][i] * (x[i] - rx[i]);
        if (al) v[i] += 50 * (s * s / 2 * hx[i] * h + lam * hx[i]);
      }
      if (ntc_of(mode, true) && sp.AL_active) {  // trials of the last line search
        const real s2 = st->ls_sigma[p], lam2 = st->ls_lambda[p];
        for (int j = 0; j < st->ls_nt; ++j) {
          const int slot = j < st->ls_nom ? j : j + 1;
          const real* xt = traj_ptr(sp, d, b, slot, ko + k);
          real ht, hxt[14], Hst[3][3];
          if (mode == 2) wb_touchdown_compact<kFront>(xt, &ht, hxt, Hst);
          else wb_touchdown_compact<kBack>(xt, &ht, hxt, Hst);
          for (int i = 0; i < 14; ++i) v[i] += 50 * (s2 * s2 / 2 * hxt[i] * ht + lam2 * hxt[i]);
        }
      }
      for (int i = 0; i < 14; ++i) o[i] = v[i];
    } else {
      real rx[6];
      fb_term_ref(sp, pos, rx);
      for (int i = 0; i < 6; ++i) o[i] = sp.cw.fQf[mode - 1][i] * (x[i] - rx[i]);
    }
  }
}

// ============================================================================================
// Phase buffers of the receding-horizon loop (MHPCLocomotion::update_problem,
// MHPCLocomotion.cpp:107-158): the reference keeps one N_TIMESTEPS_MAX-knot buffer per WB
// and per SRB phase slot (nominal x,u,y and cost-to-go) and rotates which buffer each phase
// uses.  store [B][spmax][nbk][SREC]: x,u,y (a traj record), K 56, du 4, G 14.  Phase p of a
// problem's layout lives in its buffer L.buf[p]; k_store_save runs with the layouts before
// an update, k_store_load with those after it.
// ============================================================================================
constexpr int SREC = KS + 56 + 4 + 14;

__global__ void k_store_save(SolveParams sp, DevBufs d, real* store, int nbk, int spmax) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)sp.B * sp.NK) return;
  const int b = (int)(t / sp.NK), kk = (int)(t - (long)b * sp.NK);
  const Layout& L = d.lay[d.lid[b]];  // the problem's layout (per lane: not a hot kernel)
  if (kk >= L.NK) return;
  int p = 0;
  while (p + 1 < L.P && kk >= L.ko[p + 1]) ++p;
  const int k = kk - L.ko[p];
  real* o = store + (((size_t)b * spmax + L.buf[p]) * nbk + k) * SREC;
  const real* r = traj_ptr(sp, d, b, d.st[b].nom_slot, kk);
  for (int i = 0; i < KS; ++i) o[i] = r[i];
  const size_t rec = (size_t)b * sp.NK + kk;
  for (int i = 0; i < 56; ++i) o[KS + i] = d.K[rec * 56 + i];
  for (int i = 0; i < 4; ++i) o[KS + 56 + i] = d.du[rec * 4 + i];
  for (int i = 0; i < 14; ++i) o[KS + 60 + i] = d.G[rec * 14 + i];
}

__global__ void k_store_load(SolveParams sp, DevBufs d, const real* store, int nbk, int spmax) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)sp.B * sp.NK) return;
  const int b = (int)(t / sp.NK), kk = (int)(t - (long)b * sp.NK);
  const Layout& L = d.lay[d.lid[b]];  // the problem's layout (per lane: not a hot kernel)
  if (kk >= L.NK) return;
  int p = 0;
  while (p + 1 < L.P && kk >= L.ko[p + 1]) ++p;
  const int k = kk - L.ko[p];
  const real* o = store + (((size_t)b * spmax + L.buf[p]) * nbk + k) * SREC;
  real* r = traj_ptr(sp, d, b, 0, kk);  // k_init(warm = 0) sets nom_slot = 0
  for (int i = 0; i < KS; ++i) r[i] = o[i];
  if (k == L.N[p] - 1)  // u, y of the last knot are never rewritten by a sweep (B11): the
    for (int sl = 1; sl < sp.nslot; ++sl) {  // buffer's stale tail must follow any trial
      real* q = traj_ptr(sp, d, b, sl, kk);
      for (int i = 0; i < KS; ++i) q[i] = o[i];
    }
  const size_t rec = (size_t)b * sp.NK + kk;
  for (int i = 0; i < 56; ++i) d.K[rec * 56 + i] = o[KS + i];
  for (int i = 0; i < 4; ++i) d.du[rec * 4 + i] = o[KS + 56 + i];
  for (int i = 0; i < 14; ++i) d.G[rec * 14 + i] = o[KS + 60 + i];
}

hipError_t launch_store(const SolveParams& sp, const DevBufs& d, real* store, int nbk, int spmax,
                        int save, hipStream_t s) {
  const long n = (long)sp.B * sp.NK;
  if (save)
    hipLaunchKernelGGL(k_store_save, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, sp, d,
                       store, nbk, spmax);
  else
    hipLaunchKernelGGL(k_store_load, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, sp, d,
                       store, nbk, spmax);
  return hipGetLastError();
}

// ============================================================================================
// k_partials: forward_sweep_partials_only (SinglePhase.cpp:147-180) -- the dynamics
// Jacobians of every WB knot of the nominal, by implicit differentiation of the contact KKT
// system at the knot's solution (mhpc_model.h, WbKnot): the lane solves the knot's forward
// dynamics once and then, per tangent direction, evaluates the inverse-dynamics residual in
// dual numbers and solves with the knot's own factorisation.  One launch over the knot grid,
// a lane per (problem, WB knot): the configuration directions 2..6, the velocity directions
// 9..13, the controls 14..17 and the knot's control / force cost derivatives; directions 0, 1,
// 7, 8 (base position / velocity) are exact zeros written once at create.  k_partials_impact: the impact Jacobian Px at the end of the touchdown
// phases, one lane per (problem, impact, direction), dual numbers through wb_impact.
// ============================================================================================
// Direction groups, one launch each: [d0, d1) of the record's 18 columns (the controls'
// columns need no residual, just a solve).  1 (default, round 6): every direction in one lane,
// the knot's forward dynamics once.  2: G = 0 the configuration directions (+ the cost
// derivatives), G = 1 the velocity and control directions, on two streams (rounds 3-5: more
// lanes with shorter chains, the forward dynamics repeated per group); 4 splits both in two.
// 1 vs 2, interleaved A/B (profiles/r06_partials_groups_ab.txt): C3 +0.6 % at 1024 (SRB half
// beside them 0.186 -> 0.180 ms per launch), +1.1 % at 4096, C5 +1 %, mixed +0.5 %, C5 fp32
// -0.2 %; bitwise equal in fp64.  The fp32 build keeps two groups: its kernels are built with
// contraction, and the one-group code contracts differently (the float-sweep C5 errors of
// tests/test_gpu_fp32.py moved: X 95th percentile 1.09e-2), for no speed.
#ifndef MHPC_PAR_GROUPS
#ifdef MHPC_FP32
#define MHPC_PAR_GROUPS 2
#else
#define MHPC_PAR_GROUPS 1
#endif
#endif
constexpr int kParGroups = MHPC_PAR_GROUPS;
constexpr int kParD0[4] = {2, kParGroups == 4 ? 5 : 9, 9, 14};
constexpr int kParD1[4] = {kParGroups == 1 ? 18 : kParGroups == 4 ? 5 : 7, kParGroups == 4 ? 7 : 18, 14, 18};

// rec: the knot's piece of column block 0 (column c at rec + c * NK * 9, mhpc_solver.h par_col)
template <int SF, int G>
__device__ __forceinline__ void partials_knot(const real* nk, real* rec, int NK) {
  constexpr int d0 = kParD0[G], d1 = kParD1[G];
  real x[14], u[4];
#pragma unroll
  for (int i = 0; i < 14; ++i) x[i] = nk[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = nk[14 + i];
  WbKnot K;
  wb_knot_primal<SF>(x, u, K);
#pragma unroll 1
  for (int dir = d0; dir < (d1 < 7 ? d1 : 7); ++dir) {
    real o[9];
    wb_knot_partial_q<SF>(x, K, dir, o);
#pragma unroll
    for (int i = 0; i < 9; ++i) rec[(size_t)dir * NK * 9 + i] = o[i];
  }
#pragma unroll 1
  for (int dir = d0 > 9 ? d0 : 9; dir < (d1 < 14 ? d1 : 14); ++dir) {
    real o[9];
    wb_knot_partial_qd<SF>(x, K, dir, o);
#pragma unroll
    for (int i = 0; i < 9; ++i) rec[(size_t)dir * NK * 9 + i] = o[i];
  }
#pragma unroll 1
  for (int dir = d0 > 14 ? d0 : 14; dir < d1; ++dir) {
    real o[9];
    wb_knot_partial_u<SF>(K, dir, o);
#pragma unroll
    for (int i = 0; i < 9; ++i) rec[(size_t)dir * NK * 9 + i] = o[i];
  }
}

// MHPC_PAR_MINB: blocks per CU the register allocator must allow for the partials (1: no cap;
// round 6: 2 in the fp32 build, 258 -> 256 VGPRs, two waves per SIMD, measured identical)
#ifndef MHPC_PAR_MINB
#define MHPC_PAR_MINB 1
#endif
// MHPC_PAR_BLOCK: threads per block of the direction-group launches.  128 (two waves) rather
// than 256: at one wave per SIMD (the configuration group's 340 VGPRs) a block needs that many
// SIMDs of one CU free at once, so smaller blocks fill the SIMDs the other group and the SRB
// half of the sweep leave -- partials 1.10 -> 0.74 ms per step at batch 1024 (+1.9 % solves/s),
// +0.3 % at 4096; 64 measured the same within noise (round 6, one group: again)
#ifndef MHPC_PAR_BLOCK
#define MHPC_PAR_BLOCK 128
#endif
template <int G>
__global__ __launch_bounds__(MHPC_PAR_BLOCK, MHPC_PAR_MINB) void k_partials(SolveParams sp, DevBufs d) {
  // blocks by layout group, lanes = (problem of the group, WB knot)
  long t0 = 0;
  const int g = block_group_items(sp, sp.gpk, 0, blockIdx.x, MHPC_PAR_BLOCK, &t0);
  if (g < 0) return;
  const Layout& L = layout_of(d, g);
  const long t = t0 + threadIdx.x;
  const int i0 = (int)(t / L.par_knots);
  if (i0 >= sp.go[g + 1] - sp.go[g]) return;
  const int it = (int)(t - (long)i0 * L.par_knots);
  const int b = prob_at(sp, d, sp.go[g] + i0);
  const ProbState* st = &d.st[b];
  if (!(st->active && st->ddp_active)) return;
  int p = 0;
  while (it >= L.par_knot_off[p + 1]) ++p;
  const int k = it - L.par_knot_off[p];
  const int ko = L.ko[p], mode = L.mode[p];
  const real* nk = traj_ptr(sp, d, b, st->nom_slot, ko + k);
  real* rec = d.par + par_col(sp.NK, b, 0, ko + k);
  if (mode == 1) partials_knot<kBack, G>(nk, rec, sp.NK);
  else if (mode == 3) partials_knot<kFront, G>(nk, rec, sp.NK);
  else partials_knot<-1, G>(nk, rec, sp.NK);
  if (G == 0) {
    // running-cost derivatives of controls and contact forces at the nominal knot
    // (CostBase.cpp:19-34 + ReB barrier, SinglePhase.cpp:219-249 CALC_PARTIALS_ONLY)
    real c[14];
    wb_cost_uy_derivs(sp, mode, L.dt[p], nk + 14, nk + 18, st->reb_active != 0, st->delta[p],
                      st->eps_tq[p], st->eps_grf[p], c);
#pragma unroll
    for (int i = 0; i < 14; ++i) d.par[par_jac(sp.NK, b, ko + k) + i] = c[i];
  }
}

__global__ __launch_bounds__(256) void k_partials_impact(SolveParams sp, DevBufs d) {
  long t0 = 0;
  const int g = block_group_items(sp, sp.gpi, 0, blockIdx.x, 256, &t0);
  if (g < 0) return;
  const Layout& L = layout_of(d, g);
  const long t = t0 + threadIdx.x;
  const int i0 = (int)(t / L.par_imp);
  if (i0 >= sp.go[g + 1] - sp.go[g]) return;
  const int it = (int)(t - (long)i0 * L.par_imp);
  const int b = prob_at(sp, d, sp.go[g] + i0);
  const ProbState* st = &d.st[b];
  if (!(st->active && st->ddp_active)) return;
  int p = 0;
  while (it >= L.par_imp_off[p + 1]) ++p;
  const int dir = it - L.par_imp_off[p];
  const int mode = L.mode[p];
  const real* nk = traj_ptr(sp, d, b, st->nom_slot, L.ko[p] + L.N[p] - 1);
  Dual x[14], xp[14], lam[2];
#pragma unroll
  for (int i = 0; i < 14; ++i) x[i] = Dual(nk[i], i == dir ? real(1.0) : real(0.0));
  wb_impact<Dual>(x, mode == 2 ? kFront : kBack, xp, lam);
  real* out = d.px + ((size_t)b * MAXP + p) * 196 + dir * 14;
#pragma unroll
  for (int i = 0; i < 14; ++i) out[i] = xp[i].d;
}

// ============================================================================================
// AL / ReB update (MultiPhaseDDP.cpp:273-284, SinglePhase.cpp:334-354)
// ============================================================================================
__global__ void k_al_end(SolveParams sp, DevBufs d, int last) {
  const GrpBlk gb = block_group(sp, blockIdx.x, 64);
  if (gb.g < 0 || gb.p0 + (int)threadIdx.x >= gb.p1) return;
  const Layout& L = layout_of(d, gb.g);
  const int b = prob_at(sp, d, gb.p0 + threadIdx.x);
  ProbState* st = &d.st[b];
  if (st->active) {
    real up = st->cap_pen;  // _option.update_penalty = captured value, 0 if satisfied
    if (st->viol < real(0.03)) up = 0;
    st->opt_pen = up;
    for (int p = 0; p < L.P; ++p) {
      const bool wb = p < L.n_wb;
      if (ntc_of(L.mode[p], wb)) st->lambda[p] += st->sigma[p] * st->h[p];
      st->sigma[p] *= up;
      if (st->reb_active && wb) {
        st->delta[p] *= sp.update_relax;
        const real dmin = sp.cw.delta_min[L.mode[p] - 1];
        if (st->delta[p] < dmin) st->delta[p] = dmin;
        st->eps_tq[p] *= sp.update_ReB;
        st->eps_grf[p] *= sp.update_ReB;
      }
    }
    if (st->viol < sp.AL_thresh) st->active = 0;
  }
  if (last && st->status == MHPC_SOLVE_OK && !isfinite(st->J)) st->status = MHPC_SOLVE_NONFINITE;
}

// ============================================================================================
// initialization: references, state, PD warm start (MHPCLocomotion.cpp:47-53,200-215)
// ============================================================================================
// warm = 0 (mhpc_update_problem): references and per-problem state only -- the reference's
// update_problem() regenerates the references and re-initialises the AL / ReB parameters of
// every phase but keeps the (rotated) nominal trajectories and gains as the warm start.
// References (ReferenceGen.h:94-109) and the per-problem solver state of one problem;
// warm = 1 also resets the option fields a solve rewrites (see ProbState).
__device__ void k_init_state(const SolveParams& sp, const DevBufs& d, const Layout& L, int b,
                             int warm) {
  const real* x0 = d.x0 + (size_t)b * 14;
  real* pos = d.refpos + (size_t)b * sp.NK;
  for (int p = 0; p < L.P; ++p) {
    const int ko = L.ko[p];
    pos[ko] = p == 0 ? x0[0] : pos[L.ko[p - 1] + L.N[p - 1] - 1];
    for (int k = 1; k < L.N[p]; ++k) pos[ko + k] = pos[ko + k - 1] + sp.vel * L.dt[p];
  }
  ProbState* st = &d.st[b];
  st->J = 0; st->viol = 0; st->dV_exp = 0; st->reg = 0; st->cost_prev = 0;
  for (int p = 0; p < MAXP; ++p) {
    st->V[p] = 0; st->dV[p] = 0; st->h[p] = 0; st->lambda[p] = 0;
    const bool wb = p < L.n_wb && p < L.P;
    // AL_REB_PARAMETER of the phase's mode (MHPCConstraints.cpp:43-88, mhpc_set_constraint_params)
    const int m = p < L.P ? L.mode[p] - 1 : 0;
    st->sigma[p] = (wb && ntc_of(L.mode[p], true)) ? sp.cw.sigma0[m] : real(0.0);
    st->delta[p] = sp.cw.delta0[m];
    st->eps_tq[p] = sp.cw.eps_tq0[m];
    st->eps_grf[p] = sp.cw.eps_grf0[m];
  }
  st->status = MHPC_SOLVE_OK;
  // ReB flag as the options set it (what a sweep right after initialization() sees); the
  // first forward_sweep(0) applies the per-AL-iteration rule (MultiPhaseDDP.cpp:178-183)
  st->active = 1; st->ddp_active = 0; st->reb_active = sp.ReB_active ? 1 : 0; st->al_partials = 0;
  st->nom_slot = 0; st->al_iter = 0; st->ddp_iter = 0; st->bws_iter = 0; st->ntrace = 0;
  for (int i = 0; i < TRACE; ++i) st->trace[i] = -1;
  for (int i = 0; i < NCNT; ++i) st->cnt[i] = 0;
  st->par_slot = 0;
  st->par_al = 0;
  st->ls_nt = 0;
  st->ls_nom = 0;
  st->reroll_j = -1;
  st->reroll_nom = 0;
  st->reroll_eps = real(0.0);
  for (int p = 0; p < MAXP; ++p) {
    st->par_sigma[p] = 0; st->par_lambda[p] = 0; st->ls_sigma[p] = 0; st->ls_lambda[p] = 0;
  }
  if (!warm) return;
  st->opt_reb = sp.ReB_active ? 1 : 0;
  st->opt_pen = sp.update_penalty;
  st->cap_reb = st->opt_reb;
  st->cap_pen = st->opt_pen;
}

// A lane pair per problem (even lane: front leg, odd: back leg of the pair dynamics,
// mhpc_model_pair.h): the warm-start rollout is one serial chain per problem, so halving its
// per-knot latency is what counts; both lanes carry the same state and controls (the pair
// model returns xdot and y on both, bit for bit the single-lane model's), the even lane
// writes the references and the per-problem state, each lane half of every knot record.
// memory_reset (MHPCLocomotion.cpp:265-288), launched on the second stream beside k_init and
// hidden behind its serial warm-start chains: K, du and G of every knot, and u and y of
// every phase's last knot in every trajectory slot (no rollout writes them, quirk B11; a slot
// becoming the nominal carries them into the exports).  Everything else of traj is written
// before it is read (slot 0 by k_init, the candidate slots by the line search), so initialize
// does not clear the whole array (2.8 GB at batch 4096).  k_init reads none of these arrays
// and writes other elements of the tail records.
__device__ void init_reset_arrays(const SolveParams& sp, const DevBufs& d, long t, long nt) {
  const long nk = (long)sp.B * sp.NK;
  for (long i = t; i < nk * 56; i += nt) d.K[i] = real(0.0);
  for (long i = t; i < nk * 4; i += nt) d.du[i] = real(0.0);
  for (long i = t; i < nk * 14; i += nt) d.G[i] = real(0.0);
  const long n = (long)sp.B * sp.nslot * sp.pmax;
  for (long i = t; i < n; i += nt) {
    const int p = (int)(i % sp.pmax);
    const long bs = i / sp.pmax;
    const int slot = (int)(bs % sp.nslot), b = (int)(bs / sp.nslot);
    const Layout& L = d.lay[d.lid[b]];  // the problem's layout (per lane; hidden beside k_init)
    if (p >= L.P) continue;
    const int nx = p < L.n_wb ? 14 : 6;
    real* r = traj_ptr(sp, d, b, slot, L.ko[p] + L.N[p] - 1);
    for (int e = nx; e < KS; ++e) r[e] = real(0.0);
  }
}

__global__ __launch_bounds__(256) void k_reset_arrays(SolveParams sp, DevBufs d) {
  init_reset_arrays(sp, d, (long)blockIdx.x * 256 + threadIdx.x, (long)gridDim.x * 256);
}

__global__ __launch_bounds__(64) void k_init(SolveParams sp, DevBufs d, int warm) {
  // blocks by layout group, 32 problems a block
  const GrpBlk gb = block_group(sp, blockIdx.x, 32);
  const int i0 = threadIdx.x >> 1;
  const bool back = (threadIdx.x & 1) != 0;
  if (gb.g < 0 || gb.p0 + i0 >= gb.p1) return;  // both lanes of a pair
  const Layout& L = layout_of(d, gb.g);
  const int b = prob_at(sp, d, gb.p0 + i0);
  const real* x0 = d.x0 + (size_t)b * 14;
  if (!back) k_init_state(sp, d, L, b, warm);
  if (!warm) return;
  // warm start of the WB phases into slot 0 (bounding_PDcontrol, boundingPDControl.cpp:3-46)
  real x[14];
  for (int i = 0; i < 14; ++i) x[i] = x0[i];
  const real qnom[4] = {PI / 4, -PI * 7 / 12, PI / 4, -PI * 7 / 12};
  const real Kp[4] = {5 * real(8.0), 5 * real(1.0), 5 * real(12.0), 5 * real(10.0)};
  SinCosK scK = kSinCosK;  // VGPR copies (see k_rollout)
#if MHPC_RO_VCONST && !defined(MHPC_FP32)
#pragma unroll
  for (int i = 0; i < 15; ++i) asm volatile("" : "+v"(scK.c[i]));
#endif
  for (int p = 0; p < L.n_wb; ++p) {
    const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    const real dt = L.dt[p];
    for (int k = 0; k < N - 1; ++k) {
      // the state-only part of the dynamics first: the stance controller reuses its geometry
      WbPairPrep P;
      wb_pair_prep(x, back, P, scK);
      real u[4];
#ifdef MHPC_FP32
      // (fp32: the reference-ordered evaluation below; its C5 accuracy is chaotic in the warm
      // start's last bits -- the pair-geometry form moved the X 95th percentile of
      // tests/test_gpu_fp32.py from 7.9e-3 to 1.2e-2, past the 1e-2 target)
      if (mode == 1 || mode == 3) {
        real J[14], Jd[14], v[2];
        if (mode == 1) { wb_foot_jacobian_f<kBack>(x, J, Jd); wb_leg_ext<kBack>(x, v); }
        else { wb_foot_jacobian_f<kFront>(x, J, Jd); wb_leg_ext<kFront>(x, v); }
        const real sq = v[0] * v[0] + v[1] * v[1], nrm = sqrt(sq);
        const real n0 = v[0] / nrm, n1 = v[1] / nrm;
        const real F0 = -n0 * real(2200.0) * (nrm - real(0.2462)), F1 = -n1 * real(2200.0) * (nrm - real(0.2462));
        const real gain = mode == 1 ? 3 : real(2.2);
        for (int i = 0; i < 4; ++i) u[i] = (J[3 + i] * F0 + J[7 + 3 + i] * F1) * gain;
      }
#else
      if (mode == 1 || mode == 3) {
        // the stance foot's Jacobian (wb_foot_jacobian_f: its leg's hip / knee columns; the
        // other leg's are exact zeros) and hip-to-foot vector (wb_leg_ext) from the stance
        // lane's own-leg geometry -- the same expressions on the same sines / cosines
        const bool mine = (mode == 1) == back;
        real jx[5], jz[5], jdx, jdz;
        pair_point_jac(P.L, P.sg, P.sth, P.cth, kThighLen, kShankLen, jx, jz, &jdx, &jdz);
        const real ve0 = -kThighLen * P.L.s1 - kShankLen * P.L.s2;
        const real ve1 = -kThighLen * P.L.c1 - kShankLen * P.L.c2;
        const real v[2] = {mode == 1 ? pair_from<1>(ve0) : pair_from<0>(ve0),
                           mode == 1 ? pair_from<1>(ve1) : pair_from<0>(ve1)};
        const real sq = v[0] * v[0] + v[1] * v[1], nrm = sqrt(sq);
        const real n0 = v[0] / nrm, n1 = v[1] / nrm;
        const real F0 = -n0 * real(2200.0) * (nrm - real(0.2462)), F1 = -n1 * real(2200.0) * (nrm - real(0.2462));
        const real gain = mode == 1 ? 3 : real(2.2);
        real uo[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const real jxa = mine ? jx[3 + a] : real(0.0), jza = mine ? jz[3 + a] : real(0.0);
          uo[a] = (jxa * F0 + jza * F1) * gain;
        }
        u[0] = pair_from<0>(uo[0]); u[1] = pair_from<0>(uo[1]);
        u[2] = pair_from<1>(uo[0]); u[3] = pair_from<1>(uo[1]);
      }
#endif
      else {
        for (int i = 0; i < 4; ++i) u[i] = Kp[i] * (qnom[i] - x[3 + i]) - x[10 + i];
      }
      const real u2[2] = {back ? u[2] : u[0], back ? u[3] : u[1]};
      real xd[14], y[4];
      wb_pair_finish(x, u2, mode, back, P, xd, y);
      // record x (14) u (4) y (4): even lane entries 0..10, odd lane 11..21
      real rec[22];
      for (int i = 0; i < 14; ++i) rec[i] = x[i];
      for (int i = 0; i < 4; ++i) { rec[14 + i] = u[i]; rec[18 + i] = y[i]; }
      real* o = traj_ptr(sp, d, b, 0, ko + k) + (back ? 11 : 0);
#pragma unroll
      for (int i = 0; i < 11; ++i) o[i] = back ? rec[11 + i] : rec[i];
      for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
    }
    real* oe = traj_ptr(sp, d, b, 0, ko + N - 1);
    if (!back) for (int i = 0; i < 14; ++i) oe[i] = x[i];
    // phase transition exactly as the forward sweep does it (MultiPhaseDDP.cpp:351-379)
    if (p + 1 < L.P) {
      if (mode == 2 || mode == 4) {
        real xp[14], lam[2];
        wb_impact<real>(x, mode == 2 ? kFront : kBack, xp, lam);
        for (int i = 0; i < 14; ++i) x[i] = xp[i];
      }
      if (p + 1 >= L.n_wb) {
        const real t0 = x[0], t1 = x[1], t2 = x[2], t7 = x[7], t8 = x[8], t9 = x[9];
        x[0] = t0; x[1] = t1; x[2] = t2; x[3] = t7; x[4] = t8; x[5] = t9;
      }
    }
  }
  // SRB phases: the reference's first forward_sweep(0) rolls them out with the initial
  // (zero) controls and zero gains -- u = (0 + 0*0) + sum 0*(x - 0) = +0 exactly -- so the
  // nominal is completed here and forward_sweep(0) reduces to a cost evaluation (k_cost).
  // Both lanes run the (cheap) SRB chain; each writes half of every record.
  if (L.n_wb == 0)
    for (int i = 0; i < 6; ++i) x[i] = x0[i];
  for (int p = L.n_wb; p < L.P; ++p) {
    const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    const real dt = L.dt[p];
    real f[4], s[2];
    plan_foothold(x, dt * N, mode, f);
    srb_contact(mode, s);
    const real u[4] = {real(0.0), real(0.0), real(0.0), real(0.0)};
    for (int k = 0; k < N - 1; ++k) {
      real xd[6];
      srb_dynamics(x, u, f, s, xd);
      real rec[14];
      for (int i = 0; i < 6; ++i) rec[i] = x[i];
      for (int i = 0; i < 4; ++i) { rec[6 + i] = u[i]; rec[10 + i] = real(0.0); }
      real* o = traj_ptr(sp, d, b, 0, ko + k) + (back ? 7 : 0);
#pragma unroll
      for (int i = 0; i < 7; ++i) o[i] = back ? rec[7 + i] : rec[i];
      for (int i = 0; i < 6; ++i) x[i] = x[i] + xd[i] * dt;
    }
    real* oe = traj_ptr(sp, d, b, 0, ko + N - 1);
    if (!back) for (int i = 0; i < 6; ++i) oe[i] = x[i];
  }
}

// ============================================================================================
// k_cost: forward_sweep(0) at the top of an AL iteration (MultiPhaseDDP.cpp:172-190).
// With eps = 0 the rollout reproduces the nominal trajectory bit for bit (u = u_nom + 0 +
// K * 0 and the same dynamics code on the same state), so only the costs change (new ReB
// flag, sigma / lambda).  One wave per problem: the running cost of every knot in
// parallel, then per phase the sum in knot order (the rollout's association), terminal
// cost, AL term and touchdown constraint.
// ============================================================================================
__global__ __launch_bounds__(64) void k_cost(SolveParams sp, DevBufs d, int al_iter) {
  MHPC_NO_FMA_F32
  const GrpBlk gb = block_group(sp, blockIdx.x, 1);  // one problem a block
  if (gb.g < 0) return;
  const Layout& L = layout_of(d, gb.g);
  const int b = prob_at(sp, d, gb.p0);
  ProbState* st = &d.st[b];
  if (!st->active) return;
  const int lane = threadIdx.x;
  __shared__ real sc[MHPC_MAX_KNOTS];
  __shared__ acc sV[MAXP];
  __shared__ real sH[MAXP];
  const bool reb_off = (st->viol > real(0.05)) || al_iter == 1;
  // solve() captures _option.ReB_active at its start, restores it every AL iteration
  const int cap_reb = al_iter == 1 ? st->opt_reb : st->cap_reb;
  const bool reb = cap_reb && !reb_off;
  const int nom = st->nom_slot;
  const real* refpos = d.refpos + (size_t)b * sp.NK;
  for (int kk = lane; kk < L.NK; kk += 64) {
    int p = 0;
    while (p + 1 < L.P && kk >= L.ko[p + 1]) ++p;
    const int k = kk - L.ko[p], mode = L.mode[p];
    real c = real(0.0);
    if (k < L.N[p] - 1) {
      const real* r = traj_ptr(sp, d, b, nom, kk);
      if (p < L.n_wb)
        c = wb_running_cost(sp, mode, L.dt[p], refpos[kk], r, r + 14, r + 18, reb, st->delta[p],
                            st->eps_tq[p], st->eps_grf[p]);
      else
        c = fb_running_cost(sp, mode, L.dt[p], refpos[kk], r, r + 6);
    }
    sc[kk] = c;
  }
  __syncthreads();
  if (lane < L.P) {
    MHPC_NO_FMA_COST
    const int p = lane, mode = L.mode[p], N = L.N[p], ko = L.ko[p];
    acc V = 0;
    real h = 0;
    for (int k = 0; k < N - 1; ++k) V += sc[ko + k];
    const real* x = traj_ptr(sp, d, b, nom, ko + N - 1);
    if (p < L.n_wb) {
      real rx[14];
      wb_term_ref(sp, mode, refpos[ko + N - 1], rx);
      acc Phi = 0;
      for (int i = 0; i < 14; ++i) { const real e = x[i] - rx[i]; Phi += e * sp.cw.wQf[mode - 1][i] * e; }
      Phi = Phi * acc(0.5);
      if (ntc_of(mode, true)) {
        h = mode == 2 ? wb_touchdown_value<kFront>(x) : wb_touchdown_value<kBack>(x);
        if (sp.AL_active) {
          const acc s = st->sigma[p], lam = st->lambda[p];
          const acc sh2 = s * h / 2;
          Phi += 50 * (sh2 * sh2 + lam * h);
        }
      }
      V += Phi;
    } else {
      real rx[6];
      fb_term_ref(sp, refpos[ko + N - 1], rx);
      acc Phi = 0;
      for (int i = 0; i < 6; ++i) { const real e = x[i] - rx[i]; Phi += e * sp.cw.fQf[mode - 1][i] * e; }
      V += Phi * acc(0.5);
    }
    sV[p] = V;
    sH[p] = h;
  }
  __syncthreads();
  if (lane == 0) {
    acc J = 0, viol2 = 0;
    for (int p = 0; p < L.P; ++p) {
      J += sV[p];
      viol2 += acc(sH[p]) * sH[p];
      st->V[p] = sV[p];
      st->h[p] = sH[p];
    }
    if (al_iter == 1) { st->cap_reb = st->opt_reb; st->cap_pen = st->opt_pen; }
    st->reb_active = reb ? 1 : 0;
    st->opt_reb = st->reb_active;
    st->J = J;
    st->viol = sqrt(viol2);
    st->par_slot = nom;  // forward_sweep(0) evaluated the partials (with AL, B1) here
    st->par_al = sp.AL_active ? 1 : 0;
    st->ls_nt = 0;
    for (int p = 0; p < L.P; ++p) { st->par_sigma[p] = st->sigma[p]; st->par_lambda[p] = st->lambda[p]; }
    st->al_iter = al_iter;
    st->reg = 0;
    st->ddp_active = 1;
    st->al_partials = 1;
    st->cnt[C_FWD]++;
    st->cnt[C_PAR_RUN]++;
  }
}

// Copy each problem's nominal trajectory (slot nom_slot) to a dense staging buffer.
__global__ void k_export(SolveParams sp, DevBufs d) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)sp.NK * KS;
  const int b = (int)(t / per);
  if (b >= sp.B) return;
  const long r = t - (long)b * per;
  const int nom = d.st[b].nom_slot;
  d.out[(size_t)b * per + r] = d.traj[(((size_t)b * sp.nslot + nom) * sp.NK) * KS + r];
}

// ---- kernel-level parity hooks (batched CasADi replacements) -----------------------------
__global__ void k_eval_wb_dyn(int n, int mode, const real* x, const real* u, real* xd,
                              real* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  wb_dynamics<real>(x + (size_t)i * 14, u + (size_t)i * 4, mode, xd + (size_t)i * 14, y + (size_t)i * 4);
}

// The line search's lane-pair dynamics (mhpc_model_pair.h): lane 2i + leg of point i, both
// lanes' xdot / y written ([n][2][14], [n][2][4]) so a test can check that each equals the
// single-lane model.  Lanes past 2n hold whole idle pairs (the DPP swaps stay inside pairs).
__global__ void k_eval_wb_dyn_pair(int n, int mode, const real* x, const real* u, real* xd,
                                   real* y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 1;
  const bool back = t & 1;
  if (i >= n) return;
  const real* xi = x + (size_t)i * 14;
  const real u2[2] = {u[(size_t)i * 4 + (back ? 2 : 0)], u[(size_t)i * 4 + (back ? 3 : 1)]};
  real f[14], yy[4];
  wb_dynamics_pair(xi, u2, mode, back, f, yy);
  for (int r = 0; r < 14; ++r) xd[(size_t)t * 14 + r] = f[r];
  for (int r = 0; r < 4; ++r) y[(size_t)t * 4 + r] = yy[r];
}

// Touchdown constraint (WB_FL1/FL2_terminal_constr) as the kernels evaluate it: h both from
// the derivative routine (backward sweep) and from the value-only one (line search), hx, hxx;
// and the foot Jacobian (Jacob_F / Jacob_B) of the PD warm start.
__global__ void k_eval_wb_aux(int n, int foot, const real* x, real* h, real* hx, real* hxx,
                              real* J, real* Jd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const real* xi = x + (size_t)i * 14;
  wb_touchdown(xi, foot, h + (size_t)i * 2, hx + (size_t)i * 14, hxx + (size_t)i * 196);
  h[(size_t)i * 2 + 1] = foot == kFront ? wb_touchdown_value<kFront>(xi) : wb_touchdown_value<kBack>(xi);
  wb_foot_jacobian(xi, foot, J + (size_t)i * 14, Jd + (size_t)i * 14);
}

__global__ void k_eval_wb_par(int n, int mode, const real* x, const real* u, real* Ac,
                              real* Bc, real* C, real* D) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * 18) return;
  const int i = t / 18, dir = t % 18;
  // the partials kernel's method (implicit differentiation at the point's solution)
  real a[14], c[4];
  wb_partial_column(x + (size_t)i * 14, u + (size_t)i * 4, mode, dir, a, c);
  if (dir < 14) {
    for (int r = 0; r < 14; ++r) Ac[(size_t)i * 196 + r * 14 + dir] = a[r];
    for (int r = 0; r < 4; ++r) C[(size_t)i * 56 + r * 14 + dir] = c[r];
  } else {
    for (int r = 0; r < 14; ++r) Bc[(size_t)i * 56 + r * 4 + dir - 14] = a[r];
    for (int r = 0; r < 4; ++r) D[(size_t)i * 16 + r * 4 + dir - 14] = c[r];
  }
}

__global__ void k_eval_wb_impact(int n, int foot, const real* x, real* xp, real* Px) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * 14) return;
  const int i = t / 14, dir = t % 14;
  Dual xx[14], yy[14], lam[2];
  for (int a = 0; a < 14; ++a) xx[a] = Dual(x[(size_t)i * 14 + a], a == dir ? real(1.0) : real(0.0));
  wb_impact<Dual>(xx, foot, yy, lam);
  for (int r = 0; r < 14; ++r) Px[(size_t)i * 196 + r * 14 + dir] = yy[r].d;
  if (dir == 0)
    for (int r = 0; r < 14; ++r) xp[(size_t)i * 14 + r] = yy[r].v;
}

__global__ void k_eval_srb(int n, const real* x, const real* u, const real* p,
                           const real* s, real* xd, real* Ac, real* Bc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  srb_dynamics(x + (size_t)i * 6, u + (size_t)i * 4, p + (size_t)i * 4, s + (size_t)i * 2, xd + (size_t)i * 6);
  srb_jacobians(x + (size_t)i * 6, u + (size_t)i * 4, p + (size_t)i * 4, s + (size_t)i * 2, Ac + (size_t)i * 36, Bc + (size_t)i * 24);
}

// Sum the per-problem counters of each layout group (int64 atomics into NCNT slots per group).
// One block of 256 threads, strided over the batch, tree-reduced in LDS: NCNT atomics per
// block instead of per problem (the per-problem atomics on NCNT words serialised, ~35 us).
__global__ __launch_bounds__(256) void k_reduce_counters(SolveParams sp, DevBufs d,
                                                         unsigned long long* out) {
  __shared__ unsigned long long part[NCNT][256];
  const int t = threadIdx.x;
  unsigned long long acc[NCNT];
#pragma unroll
  for (int i = 0; i < NCNT; ++i) acc[i] = 0;
  const int g = blockIdx.y;  // layout group: its problems' totals go to out[g]
  for (int pos = sp.go[g] + blockIdx.x * 256 + t; pos < sp.go[g + 1]; pos += gridDim.x * 256) {
    const int b = prob_at(sp, d, pos);
#pragma unroll
    for (int i = 0; i < NCNT; ++i) acc[i] += (unsigned long long)d.st[b].cnt[i];
  }
#pragma unroll
  for (int i = 0; i < NCNT; ++i) part[i][t] = acc[i];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
#pragma unroll
      for (int i = 0; i < NCNT; ++i) part[i][t] += part[i][t + w];
    __syncthreads();
  }
  if (t < NCNT) atomicAdd(&out[g * NCNT + t], part[t][0]);
}

// ---- launchers (called by mhpc_runtime.cpp) ---------------------------------------------
// Blocks of a launch over the layout groups with `per` problems a block (block_group)
static unsigned grid_of(const SolveParams& sp, int per) {
  long n = 0;
  for (int g = 0; g < sp.ngrp; ++g) n += (sp.go[g + 1] - sp.go[g] + per - 1) / per;
  return (unsigned)n;
}
// ... and with items[g] (or n_items) work items per problem, nt a block (block_group_items)
static unsigned grid_items(const SolveParams& sp, const int* items, int n_items, int nt) {
  long n = 0;
  for (int g = 0; g < sp.ngrp; ++g)
    n += ((long)(sp.go[g + 1] - sp.go[g]) * (items ? items[g] : n_items) + nt - 1) / nt;
  return (unsigned)n;
}
// Problems of a launch (a sub-batch's share of the batch)
int launch_problems(const SolveParams& sp) { return sp.go[sp.ngrp] - sp.go[0]; }
hipError_t launch_reduce_counters(const SolveParams& sp, const DevBufs& d,
                                  unsigned long long* out, hipStream_t s) {
  const int nb = std::min((sp.B + 255) / 256, 64);
  hipLaunchKernelGGL(k_reduce_counters, dim3(nb, sp.ngrp), dim3(256), 0, s, sp, d, out);
  return hipGetLastError();
}
hipError_t launch_reset(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  hipLaunchKernelGGL(k_init, dim3(grid_of(sp, 32)), dim3(64), 0, s, sp, d, 0);
  return hipGetLastError();
}
hipError_t launch_reset_arrays(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  // ~64 elements per lane, at most 2 blocks per CU
  const long e = (long)sp.B * sp.NK * 74 + (long)sp.B * sp.nslot * sp.pmax;
  const long nb = std::min((e + 256 * 64 - 1) / (256 * 64), 2L * sp.ncu);
  hipLaunchKernelGGL(k_reset_arrays, dim3((unsigned)nb), dim3(256), 0, s, sp, d);
  return hipGetLastError();
}
hipError_t launch_init(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  hipLaunchKernelGGL(k_init, dim3(grid_of(sp, 32)), dim3(64), 0, s, sp, d, 1);
  return hipGetLastError();
}
hipError_t launch_cost(const SolveParams& sp, const DevBufs& d, int al_iter, hipStream_t s) {
  hipLaunchKernelGGL(k_cost, dim3(grid_of(sp, 1)), dim3(64), 0, s, sp, d, al_iter);
  return hipGetLastError();
}

// The line search's launch shape for a batch (the variant launch_rollout takes)
struct RoShape {
  bool pair, pipe, st;
  int nblk, nblk2;
};
static RoShape ro_shape(const SolveParams& sp) {
  RoShape r;
  const int ppw = 64 / sp.n_cand;
  r.nblk = (int)grid_of(sp, ppw);
  const int ncu = sp.ncu;
#ifdef MHPC_RO_PIPE
  r.pipe = MHPC_RO_PIPE;
#else
  r.pipe = r.nblk <= 2 * ncu;  // measured crossover: beyond it the second
                               // wave per block only competes for issue slots
#endif
  // staged: ST_PPW problems per wave at most, and every phase within the reference stage
  const bool fits = sp.stage_fits != 0;
  r.st = ppw <= ST_PPW && fits;
  // lane pairs (two lanes per candidate) while the chip has SIMDs to spare for them
  const int ppw2 = std::min(32 / sp.n_cand, RO_PAIR_PPB);
  r.nblk2 = ppw2 > 0 ? (int)grid_of(sp, ppw2) : 0;
#ifdef MHPC_RO_PAIR_MAX_BLK
  const int pair_max = MHPC_RO_PAIR_MAX_BLK;
#else
  const int pair_max = 2 * ncu;
#endif
  r.pair = r.pipe && r.st && ppw2 > 0 && r.nblk2 <= pair_max;
  if (sp.var_ro) {  // forced (mhpc_set_kernel_variant checked that it applies)
    const int v = sp.var_ro;
    r.pair = v == MHPC_VARIANT_RO_PAIR;
    r.pipe = r.pair || v == MHPC_VARIANT_RO_PIPE_STAGED || v == MHPC_VARIANT_RO_PIPE;
    r.st = r.pair || v == MHPC_VARIANT_RO_PIPE_STAGED || v == MHPC_VARIANT_RO_FUSED_STAGED;
    if (!fits) r.pair = r.st = false;  // a phase longer than the stage: the unstaged form
  }
  return r;
}

// Trials that store their running records by default, for the shape the batch takes: the
// two-wave shapes (up to ~2k problems: the line search is a latency chain and a re-roll
// launch is another one) store the first RO_STORE_FIRST; the one-wave shape (the chip full,
// record stores a large part of the launch) the first two when the batch has one layout --
// interleaved A/B round 5: C3 at 4096 344.4k / 345.1k -> 348.3k / 350.5k solves/s (3 stored:
// +0.6 %), C5 at 4096 110.6k -> 118.4k, C3 at 1024 188.0k -> 172.6k with 2.  A mixed batch
// keeps RO_STORE_FIRST (134.2k -> 127.5k with 2): its re-roll launch, needed when any problem
// accepts an unstored trial, lasts as long as its longest layout's chain.
int ro_store_auto(const SolveParams& sp) {
  const RoShape r = ro_shape(sp);
  return (r.pipe || sp.ngrp > 1) ? RO_STORE_FIRST : 2;
}

hipError_t launch_rollout(const SolveParams& sp, const DevBufs& d, int al_iter, int ddp_iter,
                          int max_ddp, int full, hipStream_t s) {
  if (full) {
    hipLaunchKernelGGL((k_rollout<false, false, false>), dim3(grid_of(sp, 64)), dim3(64), 0, s,
                       sp, d, al_iter, 0, 0, 1);
    return hipGetLastError();
  }
  const RoShape r = ro_shape(sp);
  const bool pair = r.pair, pipe = r.pipe, st = r.st, fits = sp.stage_fits != 0;
  const int nblk = r.nblk, nblk2 = r.nblk2;
  if (pair)
    hipLaunchKernelGGL((k_rollout<true, true, true>), dim3(nblk2), dim3(128), 0, s, sp, d, al_iter,
                       ddp_iter, max_ddp, 0);
  else if (pipe && st)
    hipLaunchKernelGGL((k_rollout<true, true, false>), dim3(nblk), dim3(128), 0, s, sp, d, al_iter,
                       ddp_iter, max_ddp, 0);
  else if (pipe)
    hipLaunchKernelGGL((k_rollout<true, false, false>), dim3(nblk), dim3(128), 0, s, sp, d,
                       al_iter, ddp_iter, max_ddp, 0);
  else if (st)
    hipLaunchKernelGGL((k_rollout<false, true, false>), dim3(nblk), dim3(64), 0, s, sp, d,
                       al_iter, ddp_iter, max_ddp, 0);
  else
    hipLaunchKernelGGL((k_rollout<false, false, false>), dim3(nblk), dim3(64), 0, s, sp, d,
                       al_iter, ddp_iter, max_ddp, 0);
  // the accepted trials whose records were not stored (RO_STORE_FIRST), rolled out again:
  // lane = problem, ST_PPW problems a block so that their operands go through the LDS stage
  // (a global round trip per knot otherwise: ~2x the latency); a block without one returns
  // at once
  if (sp.ro_store < sp.n_cand - 1) {
    if (fits)
      hipLaunchKernelGGL((k_rollout<false, true, false>), dim3(grid_of(sp, ST_PPW)), dim3(64),
                         0, s, sp, d, al_iter, 0, 0, 2);
    else
      hipLaunchKernelGGL((k_rollout<false, false, false>), dim3(grid_of(sp, 64)), dim3(64), 0, s,
                         sp, d, al_iter, 0, 0, 2);
  }
  return hipGetLastError();
}
hipError_t launch_eps_rollout(const SolveParams& sp, const DevBufs& d, int n_eps,
                              const real* eps, real* J, real* viol, hipStream_t s) {
  hipLaunchKernelGGL(k_eps_rollout, dim3(grid_items(sp, nullptr, n_eps, 64)), dim3(64), 0, s, sp, d,
                     n_eps, eps, J, viol);
  return hipGetLastError();
}
hipError_t launch_cost_grad(const SolveParams& sp, const DevBufs& d, int g, int p, int N, int b0,
                            int nb, real* lx, real* phix, hipStream_t s) {
  const long n = (long)nb * N;
  hipLaunchKernelGGL(k_cost_grad, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, sp, d, g, p,
                     b0, nb, lx, phix);
  return hipGetLastError();
}
// With a second stream s3 the impact Jacobians (px: they read only the nominal) run there
// beside the knot partials; with two direction groups (MHPC_PAR_GROUPS = 2, disjoint columns
// of the records) the velocity / control group (G = 1, 252 VGPRs, two waves per SIMD) runs on
// s3 too, beside the configuration group (340 VGPRs, one wave per SIMD), and the impact
// Jacobians follow it; s joins s3 before returning.
hipError_t launch_partials(const SolveParams& sp, const DevBufs& d, hipStream_t s, hipStream_t s3,
                           hipEvent_t fork, hipEvent_t join) {
  const unsigned tk = grid_items(sp, sp.gpk, 0, MHPC_PAR_BLOCK), ti = grid_items(sp, sp.gpi, 0, 256);
  const bool two = s3 && fork && join && kParGroups <= 2 && tk > 0;
  if (two) {
    hipError_t e = hipEventRecord(fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s3, fork, 0);
    if (e != hipSuccess) return e;
  }
#ifdef MHPC_PAR_IMPACT_FIRST  // experiment: the impact Jacobians ahead of the second group
  if (ti > 0)
    hipLaunchKernelGGL(k_partials_impact, dim3(ti), dim3(256), 0, two ? s3 : s, sp, d);
#endif
  if (tk > 0) {
    constexpr int nt = MHPC_PAR_BLOCK;
    const dim3 grid(tk);
    if constexpr (kParGroups > 1) hipLaunchKernelGGL(k_partials<1>, grid, dim3(nt), 0, two ? s3 : s, sp, d);
    hipLaunchKernelGGL(k_partials<0>, grid, dim3(nt), 0, s, sp, d);
    if constexpr (kParGroups == 4) {
      hipLaunchKernelGGL(k_partials<2>, grid, dim3(nt), 0, s, sp, d);
      hipLaunchKernelGGL(k_partials<3>, grid, dim3(nt), 0, s, sp, d);
    }
  }
#ifndef MHPC_PAR_IMPACT_FIRST
  if (ti > 0)
    hipLaunchKernelGGL(k_partials_impact, dim3(ti), dim3(256), 0, two ? s3 : s,
                       sp, d);
#endif
  if (two) {
    hipError_t e = hipEventRecord(join, s3);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, join, 0);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}
hipError_t launch_al_end(const SolveParams& sp, const DevBufs& d, int last, hipStream_t s) {
  hipLaunchKernelGGL(k_al_end, dim3(grid_of(sp, 64)), dim3(64), 0, s, sp, d, last);
  return hipGetLastError();
}
hipError_t launch_export(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  const long total = (long)sp.B * sp.NK * KS;
  hipLaunchKernelGGL(k_export, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sp, d);
  return hipGetLastError();
}
hipError_t launch_eval_wb_dyn(int n, int mode, const real* x, const real* u, real* xd,
                              real* y, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_dyn, dim3((n + 63) / 64), dim3(64), 0, s, n, mode, x, u, xd, y);
  return hipGetLastError();
}
hipError_t launch_eval_wb_dyn_pair(int n, int mode, const real* x, const real* u, real* xd,
                                   real* y, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_dyn_pair, dim3((2 * n + 63) / 64), dim3(64), 0, s, n, mode, x, u, xd,
                     y);
  return hipGetLastError();
}
hipError_t launch_eval_wb_aux(int n, int foot, const real* x, real* h, real* hx, real* hxx,
                              real* J, real* Jd, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_aux, dim3((n + 63) / 64), dim3(64), 0, s, n, foot, x, h, hx, hxx, J,
                     Jd);
  return hipGetLastError();
}
hipError_t launch_eval_wb_par(int n, int mode, const real* x, const real* u, real* Ac,
                              real* Bc, real* C, real* D, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_par, dim3((n * 18 + 63) / 64), dim3(64), 0, s, n, mode, x, u, Ac,
                     Bc, C, D);
  return hipGetLastError();
}
hipError_t launch_eval_wb_impact(int n, int foot, const real* x, real* xp, real* Px,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_impact, dim3((n * 14 + 63) / 64), dim3(64), 0, s, n, foot, x, xp, Px);
  return hipGetLastError();
}
hipError_t launch_eval_srb(int n, const real* x, const real* u, const real* p,
                           const real* c, real* xd, real* Ac, real* Bc, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_srb, dim3((n + 63) / 64), dim3(64), 0, s, n, x, u, p, c, xd, Ac, Bc);
  return hipGetLastError();
}

}  // namespace MHPC_NS

#ifdef MHPC_RO_TIMING
extern "C" int mhpc_dbg_ro_cycles(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(MHPC_NS::g_ro_cyc), sizeof(unsigned long long) * 11) !=
      hipSuccess)
    return 1;
  if (reset) {
    unsigned long long z[11] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(MHPC_NS::g_ro_cyc), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
