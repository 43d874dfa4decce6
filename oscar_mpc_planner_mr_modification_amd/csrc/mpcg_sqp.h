// mpcg_sqp.h — the batched SQP-RTI solve kernel (one wavefront per solve).
//
// Reference: one `Solver::solve()` of the OpenMP fan-out in
// GuidanceConstraints::optimize (guidance_constraints.cpp:304-421) =
// `sqp_iters` acados SQP-RTI iterations (acados_solver_interface.cpp:86-119).
//
// Lane layout (PARTS lanes per shooting stage, lane = k * PARTS + part):
//   part 0 of stage k  cost / ERK4 / MIRROR / stage algebra of stage k
//   every part p       the inequality rows of stage k it owns: both bound rows
//                      of the variables p, p + PARTS, ... and the h rows
//                      p, p + PARTS, ...  All parts run the same code on
//                      runtime row indices, so a row loop costs
//                      ceil(7 / PARTS) * 2 + ceil(nh / PARTS) iterations
//                      (12 for C2) whatever the part.
// Every inequality row keeps its interior-point state (slack t, multiplier l,
// 1/t, residual, predictor product) in REGISTERS of its owner lane for the
// whole QP; LDS holds only the stage blocks (~37 KB per solve for N=20 ->
// 4 solves per CU, one wavefront per SIMD).
//   element lanes      lane e < nz (nz + 1) / 2 owns entry (i >= j) of the nz x nz block in the
//                      Riccati factorisation; the next stage's block is
//                      prefetched while the current one is reduced
//   chains             the two 5-vector recursions of each Newton solve run as
//                      affine maps p_k = h_k + G_k p_{k+1}, dx_{k+1} = G_k' dx_k + e_k
//                      carried in SGPRs through v_readlane.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mpcg.h"
#include "mpcg_bicycle.h"
#include "mpcg_device.h"

namespace mpcg {

enum { AC_SUCCESS = 0, AC_NAN = 1, AC_MAXITER = 2, AC_MINSTEP = 3, AC_QP_FAILURE = 4 };

__host__ __device__ constexpr int imax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int sym(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }
// column-major packed lower triangle of an n x n block, a >= c
__host__ __device__ constexpr int cpk(int n, int a, int c) { return c * n - c * (c - 1) / 2 + (a - c); }

// LDS cycles of one ds_read_b64 in which lane l = k * parts + p reads the double at
// s * k + off * p (a per-stage array, stage stride s doubles, part offset off): each 32-lane
// half is one group, dword d sits on bank d mod 64, every extra distinct dword on a busy
// bank costs a cycle (MI355X_MICROARCH.md §LDS).  Conflict-free = 2.
__host__ __device__ constexpr int lds_b64_cycles(int s, int off, int parts) {
    int total = 0;
    for (int half = 0; half < 2; ++half) {
        int dw[64] = {};
        int n = 0;
        for (int l = 32 * half; l < 32 * half + 32; ++l) {
            const int a = 2 * (s * (l / parts) + off * (l % parts));
            for (int h = 0; h < 2; ++h) {
                bool seen = false;
                for (int i = 0; i < n; ++i) seen = seen || dw[i] == a + h;
                if (!seen) dw[n++] = a + h;
            }
        }
        int worst = 0;
        for (int b = 0; b < 64; ++b) {
            int c = 0;
            for (int i = 0; i < n; ++i) c += (dw[i] % 64) == b;
            worst = c > worst ? c : worst;
        }
        total += worst;
    }
    return total;
}
// the stage stride in [base, base + maxpad] (steps of step) with the fewest such cycles
__host__ __device__ constexpr int lds_stride(int base, int off, int parts, int step, int maxpad) {
    int best = base, bc = lds_b64_cycles(base, off, parts);
    for (int s = base + step; s <= base + maxpad; s += step) {
        const int c = lds_b64_cycles(s, off, parts);
        if (c < bc) { bc = c; best = s; }
    }
    return best;
}

// N: horizon, NL / NE / NS: topology halfspaces, obstacle ellipsoids,
// scenario (or, C3, decomp) halfspaces per stage, NX_: 5 (unicycle) or 6
// (unicycle + slack state, or the bicycle), MODEL_: 0 contouring unicycle,
// 1 curvature-aware bicycle (C3: nu 3 with the slack input, mpcg_bicycle.h)
template <int N_, int NL_, int NE_, int NS_ = 0, int NX_ = 5, int MODEL_ = 0>
struct Cfg {
    static constexpr int N = N_, NL = NL_, NE = NE_, NS = NS_, MODEL = MODEL_;
    static constexpr int NU = MODEL_ == 1 ? 3 : 2;
    static constexpr int NX = NX_, NZ = NU + NX_;
    static_assert(MODEL_ == 1 ? NX == 6 : (NX == 5 || NX == 6), "unicycle (+ slack state) or bicycle");
    // position and heading in z = [u x]; the slack variable (a state of the
    // SH-MPC unicycle, an input of the bicycle)
    static constexpr int IX = NU, IY = NU + 1, IPSI = NU + 2;
    static constexpr bool HAS_SLACK = MODEL_ == 1 || NX > 5;
    static constexpr int ZSL = MODEL_ == 1 ? 2 : NU + 5;
    // Cholesky factor of Muu per stage: off-diagonal entries, then reciprocal diagonal
    // (nu 2: l00, l10, 1/l00, 1/l11, the layout of the unicycle's hand-unrolled code)
    static constexpr int NLO = NU * (NU - 1) / 2, NLC = NU == 2 ? 4 : NLO + NU;
    __host__ __device__ static constexpr int lo_idx(int i, int j) { return i * (i - 1) / 2 + j; }  // i > j
    static constexpr int NH = NL + NE + NS;
    static constexpr int NTRI = NZ * (NZ + 1) / 2;  // packed stage block
    static constexpr int NPT = NX * (NX + 1) / 2;   // packed cost-to-go
#ifndef MPCG_P_PAD
#define MPCG_P_PAD 1
#endif
    // cost-to-go rows padded to an even count of doubles: every stage's broadcast read is
    // 16-B aligned (ds_read_b128 with immediate offsets instead of ds_read2_b64 on every
    // other stage): C2 12.49 -> 12.26 ms, C5 20.51 -> 19.93.  Not on the long horizons
    // (C4 measured 53.84 -> 54.19) nor on the compact C3 storage (at its occupancy line)
    static constexpr int NPTP = (MPCG_P_PAD && MODEL_ != 1 && (64 / (N_ + 1)) >= 3) ? NPT + (NPT & 1) : NPT;
    // h rows touch (x, y, psi) and, with the slack model, the slack state:
    // the barrier block of the h rows is NB x NB on those variables
    static constexpr int NB = (HAS_SLACK && NS > 0) ? 4 : 3;
    static constexpr int NBT = NB * (NB + 1) / 2;
    static constexpr int NDH = NZ + NBT + 1;         // dH: diag | block | zero slot
    // the bicycle instances run two parts per stage (C3's N = 30 allows no more; the
    // register-starved bicycle keeps its row state small on the short test shapes too).
    // MPCG_PARTS_BIKE=3 builds three parts where they fit (A/B and parity runs only)
#ifndef MPCG_PARTS_BIKE
#define MPCG_PARTS_BIKE 2
#endif
    static constexpr int PARTS_MAX = (64 / (N + 1)) >= 3 ? 3 : 2;
    static constexpr int PARTS = MODEL_ == 1 ? (MPCG_PARTS_BIKE < PARTS_MAX ? MPCG_PARTS_BIKE : PARTS_MAX) : PARTS_MAX;
    static_assert((N + 1) * PARTS <= 64, "horizon too long for one wavefront");
    static_assert(NTRI <= 64, "stage block larger than a wavefront");
    // work-queue launch (sqp_kernel): the N <= 20 three-part unicycle instances (C1, C2, C5).  On the
    // long horizons the loop around the solve moves the register allocation into scratch (C4 132 ->
    // 840 B/lane, 44.3 -> 71.3 ms; JS / JD 0 -> 456 / 528 B/lane, C3 552 -> 720), so they keep one
    // workgroup per problem (MPCG_QUEUE_ALL / MPCG_NO_QUEUE: A/B)
#if defined(MPCG_NO_QUEUE)
    static constexpr bool QUEUE = false;
#elif defined(MPCG_QUEUE_ALL)
    static constexpr bool QUEUE = true;
#else
    static constexpr bool QUEUE = MODEL_ == 0 && PARTS_MAX == 3;
#endif
    // rows of a lane: box slots j (variable part + PARTS j, lower and upper
    // side: slots 2j, 2j + 1), then h slots r (h row part + PARTS r)
    static constexpr int BVS = (NZ + PARTS - 1) / PARTS;
    static constexpr int HS = (NH + PARTS - 1) / PARTS;
    static constexpr int SLOTS = 2 * BVS + HS;
    // 1/t of every row kept in registers when the row state is small (up to 13 slots on the three-part
    // instances: C1, C2); C5 (14 slots), C3 (16) and C4 (20) recompute it, which keeps them out of
    // scratch.  Round 5: 14 -> 13, C5 stops storing it (with the HPIPM profile's cold start and
    // refinement test its stored 1/t pushed the residual and step passes into scratch, 232 -> 80
    // B/lane; profiles/r05c_ab_st14_C5.jsonl).  MPCG_STORE_IT_MAX=0 recomputes it everywhere.
    // Two-part instances (JS, JD) recompute it: a round-2 build that stored 1/t there computed wrong
    // trajectories and faulted once, and that fault's cause was never named (its build no longer
    // exists).  Round 5 built the stored form again on the shipped sources, ran full-size parity on JS
    // and JD without a fault (profiles/r05f_variant_storeit.jsonl) and lifted the gate for a 1.4 % JS
    // gain (52.45 -> 51.73 ms, profiles/r05f_ab_storeit.jsonl); one clean run shows the fault did not
    // recur, not that its cause is gone, so round 6 restores the gate.  -DMPCG_STORE_IT_ANY
    // (or MPCG_STORE_IT_MAX2 > 0) builds the stored form on two-part instances for A/B runs only.
#ifndef MPCG_STORE_IT_MAX
#define MPCG_STORE_IT_MAX 13
#endif
#ifndef MPCG_STORE_IT_MAX2
#ifdef MPCG_STORE_IT_ANY
#define MPCG_STORE_IT_MAX2 12
#else
#define MPCG_STORE_IT_MAX2 0
#endif
#endif
    static constexpr bool STORE_IT = SLOTS <= (PARTS == 3 ? MPCG_STORE_IT_MAX : MPCG_STORE_IT_MAX2);
    // box bounds selected per use instead of held in registers (LaneBounds; MPCG_BOUNDS_SEL=1, A/B
    // only): C2 went into scratch with it (0 -> 68 B/lane), C3 unchanged, and C4 (148 -> 132 B/lane
    // of scratch) measured 50.75 vs 50.72 ms in two alternating repetitions (profiles/r03k_ab.jsonl)
#ifndef MPCG_BOUNDS_SEL
#define MPCG_BOUNDS_SEL 0
#endif
    static constexpr bool BOUNDS_SEL = MPCG_BOUNDS_SEL > 0;
    static constexpr int NBOX = 2 * NU + 2 * NX;  // box rows of a stage in 1..N-1 (input + state bounds)
    // Linear rows (topology and scenario halfspaces) read their coefficients from the
    // parameter block instead of LDS, and their gaps are recomputed from the iterate:
    // only the ellipsoid rows keep gradients / gaps in LDS.  Used where it lowers the
    // LDS footprint below an occupancy step (C5: 51.6 -> 36.6 KB, 3 -> 4 solves per CU).
#ifdef MPCG_LIN_PARAMS_ALL
    static constexpr bool LIN_PARAMS = true;  // occupancy experiments: the compact row storage everywhere
#else
    static constexpr bool LIN_PARAMS = NS > 0 || N >= 30;
#endif
    // gradient components kept per LDS row: with LIN_PARAMS the psi component is
    // rebuilt from (x, y) components and the stage's disc-offset derivatives
    static constexpr int DGC = LIN_PARAMS ? 2 : 3;
    static constexpr int NHS = LIN_PARAMS ? (NE > 0 ? NE : 1) : NH;  // rows with LDS storage
    // Keep parameter loads inside the SQP / QP loops (no hoisting into long-lived
    // registers): removes most scratch spills of the long-horizon and slack-model
    // instances (C4 188 -> 20 B/lane, C5 420 -> 140); C1/C2 fit without it and run
    // 1 % faster with the hoisted loads.
    static constexpr bool RELOAD_PARAMS = NS > 0 || N >= 30;
    static constexpr int M_TOTAL = 2 * NU + (N - 1) * (NBOX + NH);
    // block index of z variable v (-1: not touched by h rows)
    __host__ __device__ static constexpr int blk(int v) {
        return (v >= IX && v <= IPSI) ? v - IX : ((NB == 4 && v == ZSL) ? 3 : -1);
    }
    // z variable of block index b
    __host__ __device__ static constexpr int bvar(int b) { return b < 3 ? IX + b : ZSL; }
    // C3 storage (LDS under the 3-solves-per-CU line): the bicycle's [B A] keeps the rows of
    // x+, y+, psi+, s+ without the slack column (v+ = v + dt a, delta+ = delta + dt w are
    // known), its Hessian block drops the slack row / column but the diagonal, and the new
    // dynamics multipliers and the dynamics residuals live in registers / are recomputed
    static constexpr bool COMPACT = MODEL_ == 1;
    // the unicycle's rows psi+ = psi + dt w, v+ = v + dt a, s+ = s + dt v + dt^2/2 a (and slack+ =
    // slack) of [B A] are the same constants at every stage (RK4 integrates them exactly,
    // erk_srow): on the long horizons with few obstacles only the x+ and y+ rows are stored,
    // which (with the LEAN storage) brings N 30 with 4 or 5 obstacles under the four-solves-
    // per-CU line (JS 47.2 -> 39.9 KB, 365.8k -> 459.6k solves/s).  C4 (12 obstacles) stays above
    // the line either way and keeps its blocks in the global workspace (GFH), where the constant
    // rows shrink the per-solve block 15.3 -> 10.3 KB: 52.85 -> 51.26 ms, 304.5k -> 314.0k solves/s
    // (profiles/r02v_ab_*_C4.json; at three solves per CU, before GFH, it was 2.6 % slower).  On
    // N 20 the constant rows changed the register allocation into scratch (C2 0 -> 128 B/lane).
    // (MPCG_FCONST_N=20, A/B: the N 20 instances with the constant rows and their hoisting went into
    // scratch and ran slower -- C2 11.97 -> 13.34 ms, C5 19.46 -> 25.71, C1 10.43 -> 11.21;
    // profiles/r03q_ab.jsonl)
#ifndef MPCG_FCONST_N
#define MPCG_FCONST_N 30
#endif
    static constexpr bool FCONST = MODEL_ == 0 && N_ >= MPCG_FCONST_N;
    static constexpr int NFR = COMPACT ? 4 : (FCONST ? 2 : NX), NFC = COMPACT ? NZ - 1 : NZ;
    static constexpr int NHP = COMPACT ? (NZ - 1) * NZ / 2 + 1 : NTRI;
    // the vector chains split over the parts of a stage (rows of the backward map, columns of
    // the forward one); the register-starved bicycle instance keeps one owner per stage
#ifndef MPCG_C3_SPLIT
#define MPCG_C3_SPLIT 0
#endif
#ifndef MPCG_C3_FACFLAT
#define MPCG_C3_FACFLAT 0
#endif
    static constexpr bool CHAIN_SPLIT = !COMPACT || MPCG_C3_SPLIT;
    // the split chains as two-stage composed maps (half the sequential steps; see the
    // vector passes in sqp_kernel).  Measured against the one-step chains: JS 43.45 ->
    // 42.20 ms; C2 12.74 -> 13.09, C4 53.34 -> 53.78, C5 19.49 -> 20.07 (the compositions
    // and the extra live state cost more than the halved chain there), so only the long
    // horizons with the constant-row storage use them.  MPCG_PAIR_ALL / MPCG_NO_PAIR: A/B.
#if defined(MPCG_NO_PAIR)
    static constexpr bool PAIR_WANTED = false;
#elif defined(MPCG_PAIR_ALL)
    static constexpr bool PAIR_WANTED = true;
#else
    static constexpr bool PAIR_WANTED = FCONST && NE_ <= 8;
#endif
    static constexpr bool PAIR_CHAINS = PAIR_WANTED && CHAIN_SPLIT && (N_ + 1) / 2 * NX_ * NX_ <= (N_ + 1) * NDH &&
                                        (N_ + 1) / 2 * NX_ <= 128;
    // branch-free Riccati step (every lane, prefetch after the pivot reads, pivot failures
    // voted from a register)
    static constexpr bool FAC_FLAT = !COMPACT || MPCG_C3_FACFLAT;
#ifndef MPCG_REC_P2
#define MPCG_REC_P2 0
#endif
    // branch-free chain records (three parts per stage: C2 13.40 -> 12.92 ms, C5 23.45 -> 22.75;
    // the two-part long horizon C4 spills with it, 56.4 -> 76.2 ms)
#ifdef MPCG_REC_SELECT
    static constexpr bool REC_FLAT = CHAIN_SPLIT && PARTS == 3;
#else
    static constexpr bool REC_FLAT = CHAIN_SPLIT && (PARTS == 3 || MPCG_REC_P2);
#endif
    // the capsule's QP memory (mpcg_io.qp_in / qp_out, opaque): per slot and lane the row's
    // slack then multiplier ([2 s + {0, 1}][64 lanes]), then the QP step [N+1][NZ] and the
    // dynamics multipliers [N][NX]
    static constexpr int QPM_ROWS = 2 * SLOTS * 64;
    static constexpr int QPM = QPM_ROWS + (N + 1) * NZ + N * NX;
    // slack coefficient of h row hh (scenario rows with the slack model)
    __host__ __device__ static constexpr double slack_coef(int hh) { return (NB == 4 && hh >= NL + NE) ? -1.0 : 0.0; }
};

// LEAN storage: the dynamics residuals are recomputed where used and the new dynamics multipliers
// stay in the owner lane's registers (always for the compact C3 storage; elsewhere only where it
// brings the footprint under the four-solves-per-CU line, see lds_lean)
//
// GFH: the stage blocks H and [B A] live in a per-solve global workspace (L2-resident: the
// solves resident on one XCD hold 128 x ~16 KB) instead of LDS -- for the instances above
// the four-solves-per-CU line even with the LEAN storage (C3, C4): at one wave per SIMD a
// CU with three solves leaves a SIMD idle.  They are written once per linearisation and
// read by the Riccati step (prefetched a stage ahead) and the vector passes.
//
// PAD: the row-owner arrays (h-row gradients and gaps, read by every lane at its own stage
// and rows) and the cost-to-go rows (read by every lane at its own stage in the vector
// passes) get the stage strides with the fewest LDS bank conflicts (lds_stride; the
// cost-to-go rows stay 16-B aligned for the Riccati step's broadcast reads), where the
// padded footprint stays under the four-solves-per-CU line (lds_pad).  PAD 2 also pads the
// unpadded odd cost-to-go rows of the long horizons to an even conflict-free stride (16-B
// aligned broadcast reads; N 30: 15 -> 18 doubles) where that still fits
template <class C, bool LEAN = C::COMPACT, bool GFH = false, int PAD = 0>
struct Lds {
    static constexpr int N = C::N, NX = C::NX, NZ = C::NZ;
    // (an even gradient row keeps its 16-B alignment: its (x, y) pair is one ds_read_b128; JS with
    // the odd stride 9 measured 41.65 -> 42.03 ms)
    static constexpr int DGS =
        PAD ? lds_stride(C::NHS * C::DGC, C::DGC, C::PARTS, C::DGC % 2 == 0 ? 2 : 1, 3) : C::NHS * C::DGC;
    static constexpr int HDS = PAD ? lds_stride(C::NHS, 1, C::PARTS, 1, 3) : C::NHS;
    static constexpr int PS = PAD == 0   ? C::NPTP
                              : PAD == 2 ? lds_stride(C::NPT + (C::NPT & 1), 0, C::PARTS, 2, 4)
                                         : lds_stride(C::NPTP, 0, C::PARTS, C::NPTP == C::NPT ? 1 : 2, 4);
    double z[N + 1][NZ];      // NLP iterate [u x]
    double H[GFH ? 1 : N + 1][C::NHP];  // MIRROR-regularised Lagrangian Hessian, packed lower triangle (C::COMPACT)
    double g[N + 1][NZ];
    double F[GFH ? 1 : N][C::NFR][C::NFC];  // [B A] (C::COMPACT: rows x+ y+ psi+ s+, no slack column)
    // GFH: the Riccati step's copy of the next stage's blocks (one coalesced global load per
    // lane per stage instead of a gather per entry)
    double Fst[GFH && !C::COMPACT ? C::NFR : 1][C::NFC];
    double Hst[GFH && !C::COMPACT ? C::NHP : 1];
    double b[N][NX];          // shooting defects
    double dH[N + 1][C::NDH]; // barrier terms: diag(nz) + h-row block (column-major packed), last = 0
    double q[N + 1][NZ];      // Newton gradient
    double dz[N + 1][NZ];     // QP iterate
    double ddz[N + 1][NZ];    // QP step
    double pi_nlp[N][NX];
    double piq[N][NX];
    double pin[LEAN ? 1 : N][NX];
    double rdyn[LEAN ? 1 : N][NX];
    alignas(16) double P[N + 1][PS];  // Riccati cost-to-go, packed (row padded, C::NPTP / PS)
    double Lc[N][C::NLC];     // chol(Muu): off-diagonal l_ij (i > j), then 1/l_ii (nu 2: l00 l10 1/l00 1/l11)
    double Y[N][C::NU][NX];   // L^-1 Mux
    double bx[N + 1][NZ];     // per-variable box-row sums, written by the variable's owner lane;
                              // dead from the Newton gradient to the next residuals: holds the
                              // backward vector chain p_k [N][NX] meanwhile
    double Dg[N][DGS];        // signed h-row gradients on (x, y[, psi]) per row ([NHS][DGC]); the slack one is C::slack_coef
    double hd[N][HDS];        // h-row bound gaps (uh - h or h - lh)
    double disc[C::LIN_PARAMS ? N : 1][4];  // LIN_PARAMS: off cos psi, off sin psi, d/dpsi of both
    double Msc[128];          // factorisation scratch: the stage block (lanes < nz(nz+1)/2) and
                              // dummy targets (64 + lane) of the branch-free stores
    double xinit[NX];
    int flag;                 // failed pivot (C::COMPACT; the others vote in registers)
};

// four solves per CU need at most a quarter of the CU's 160 KiB of LDS per workgroup
// (MPCG_LDS_SOLVES_PER_CU, occupancy experiments only: another LDS line -- 8 for two waves per SIMD
// -- and the smallest storage that gets under it)
#ifdef MPCG_LDS_SOLVES_PER_CU
constexpr size_t LDS_QUARTER = 160 * 1024 / MPCG_LDS_SOLVES_PER_CU;
constexpr bool LDS_SMALLEST = true;
#else
constexpr size_t LDS_QUARTER = 160 * 1024 / 4;
constexpr bool LDS_SMALLEST = false;
#endif
template <class C>
__host__ __device__ constexpr bool lds_lean() {
    if (LDS_SMALLEST) return C::COMPACT || sizeof(Lds<C, false>) > LDS_QUARTER;
    return C::COMPACT || (sizeof(Lds<C, false>) > LDS_QUARTER && sizeof(Lds<C, true>) <= LDS_QUARTER);
}
template <class C>
__host__ __device__ constexpr bool lds_gfh() {
#ifdef MPCG_NO_GFH
    return false;
#else
    if (LDS_SMALLEST) return sizeof(Lds<C, lds_lean<C>(), false>) > LDS_QUARTER;
    return sizeof(Lds<C, lds_lean<C>(), false>) > LDS_QUARTER && sizeof(Lds<C, lds_lean<C>(), true>) <= LDS_QUARTER;
#endif
}
// conflict-minimal strides where they fit under the line (MPCG_NO_STRIDE_PAD: A/B)
template <class C>
__host__ __device__ constexpr int lds_pad() {
#if defined(MPCG_NO_STRIDE_PAD)
    return 0;
#else
#if defined(MPCG_NO_P_ALIGN)
    constexpr bool P_ALIGN = false;
#else
    constexpr bool P_ALIGN = !C::COMPACT;  // C3 with 21 -> 22: 21.14 -> 21.40 ms (profiles/r03n_ab.jsonl)
#endif
    return P_ALIGN && sizeof(Lds<C, lds_lean<C>(), lds_gfh<C>(), 2>) <= LDS_QUARTER ? 2
           : sizeof(Lds<C, lds_lean<C>(), lds_gfh<C>(), 1>) <= LDS_QUARTER         ? 1
                                                                                   : 0;
#endif
}
template <class C>
using LdsOf = Lds<C, lds_lean<C>(), lds_gfh<C>(), lds_pad<C>()>;
// doubles of one solve's global workspace (GFH: [B A] blocks, then the Hessian blocks)
template <class C>
__host__ __device__ constexpr size_t gfh_doubles() {
    return lds_gfh<C>() ? (size_t)C::N * C::NFR * C::NFC + (size_t)(C::N + 1) * C::NHP : 0;
}
// doubles of one solve's iterative-refinement scratch (qp_itref_corr_max, the rare path: the
// unrefined direction's step [N+1][NZ] and dynamics multipliers [N][NX], and -- LEAN -- the iterate's
// QP step [N+1][NZ] while S.dz holds the trial point)
template <class C>
__host__ __device__ constexpr size_t itref_doubles() {
    return 2 * (size_t)(C::N + 1) * C::NZ + (size_t)C::N * C::NX;
}
// The split launch (MPCG_SPLIT): the lean SQP-RTI as one linearisation
// kernel and one interior-point kernel per RTI iteration instead of the fused loop, each compiled for
// its phase alone.  Bit 0: split every lean instance; bit 1: the interior-point launches take the work
// queue; bit 2: the linearisation launches do.  (A/B build only.)
#ifndef MPCG_SPLIT
#define MPCG_SPLIT 0
#endif
enum { MODE_FUSED = 0, MODE_LIN = 1, MODE_QP = 2 };
template <class C>
__host__ __device__ constexpr bool split_on() {
    return (MPCG_SPLIT & 1) != 0;
}
// the block one split launch hands the next for a solve (global, after the refinement scratch): the
// iterate (z, pi), the linearisation (g, b, the h rows' gradients, gaps and offsets; [B A] and H unless
// GFH keeps them in the workspace already), the rows' NLP multipliers lane-major, and the counters
template <class C>
struct Carry {
    using L = LdsOf<C>;
    static constexpr size_t Z = 0, PI = Z + sizeof(L::z) / 8, G = PI + sizeof(L::pi_nlp) / 8,
                            B = G + sizeof(L::g) / 8, DG = B + sizeof(L::b) / 8, HD = DG + sizeof(L::Dg) / 8,
                            DISC = HD + sizeof(L::hd) / 8, H = DISC + sizeof(L::disc) / 8,
                            F = H + (lds_gfh<C>() ? 0 : sizeof(L::H) / 8),
                            NLAM = F + (lds_gfh<C>() ? 0 : sizeof(L::F) / 8), META = NLAM + 64 * (size_t)C::HS,
                            SIZE = META + 8;
    // META: res_eq, done, acados_status, qp_status, sqp_iter, qp_total, n_maxit
};
// one solve's global workspace: the GFH blocks, then the refinement scratch (then the split's carry)
template <class C>
__host__ __device__ constexpr size_t ws_doubles() {
    return gfh_doubles<C>() + itref_doubles<C>() + (split_on<C>() ? Carry<C>::SIZE : 0);
}

// Diagnostic per-phase cycle stamps (separate build with -DMPCG_STAMPS; the
// production build compiles them out).  Read shares, not absolute times.
#ifdef MPCG_STAMPS
#define MPCG_NSTAMP 24
#define STAMP_DECL unsigned long long st_acc_[MPCG_NSTAMP] = {}, st_t0_ = 0, st_l_ = 0;
#define STAMP_BEGIN() do { __syncthreads(); st_t0_ = __builtin_amdgcn_s_memtime(); st_l_ = st_t0_; } while (0)
#define STAMP_END(i) do { __syncthreads(); st_acc_[i] += __builtin_amdgcn_s_memtime() - st_t0_; } while (0)
// sub-phase lap inside a phase (the wave runs divergent branches one after the other)
#define STAMP_LAP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc_[i] += t_ - st_l_; st_l_ = t_; } while (0)
#define STAMP_STORE(ptr, sol) \
    do { if ((ptr) && threadIdx.x == 0) for (int i_ = 0; i_ < MPCG_NSTAMP; ++i_) (ptr)[(size_t)(sol) * MPCG_NSTAMP + i_] = st_acc_[i_]; } while (0)
#elif defined(MPCG_MARKERS)
// assembly markers of the phases (ISA inspection builds only)
#define STAMP_DECL
#define STAMP_BEGIN() asm volatile("; @@begin")
#define STAMP_END(i) asm volatile("; @@end " #i)
#define STAMP_LAP(i) asm volatile("; @@lap " #i)
#define STAMP_STORE(ptr, sol) do {} while (0)
#else
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(i) do {} while (0)
#define STAMP_LAP(i) do {} while (0)
#define STAMP_STORE(ptr, sol) do {} while (0)
#endif

// Unrolling of the stage loops of the interior point: the Riccati recursion (MPCG_UNROLL_FAC) and the split
// vector chains (MPCG_UNROLL_CHAIN).  Default: fully unrolled (every stage's addresses, lane masks and
// readlane lanes literal).  MPCG_FAC_UNROLL / MPCG_CHAIN_UNROLL = n: unrolled by n (1: a rolled loop with
// run-time stage offsets), for A/B runs of the instruction footprint.
#define MPCG_PRAGMA_(x) _Pragma(#x)
#ifdef MPCG_FAC_UNROLL
#define MPCG_UNROLL_FAC MPCG_PRAGMA_(unroll MPCG_FAC_UNROLL)
#else
#define MPCG_UNROLL_FAC MPCG_PRAGMA_(unroll)
#endif
#ifdef MPCG_CHAIN_UNROLL
#define MPCG_UNROLL_CHAIN MPCG_PRAGMA_(unroll MPCG_CHAIN_UNROLL)
#else
#define MPCG_UNROLL_CHAIN MPCG_PRAGMA_(unroll)
#endif

// One wavefront per workgroup (blockDim 64): the lanes exchange data through LDS,
// and a wave's LDS instructions execute in issue order, so an exchange needs a
// compiler barrier only, not an s_waitcnt on the producing stores before the
// consuming loads issue (-DMPCG_LDS_WAIT restores __syncthreads for A/B runs).
__device__ __forceinline__ void wave_sync() {
#ifdef MPCG_LDS_WAIT
    __syncthreads();
#else
    __asm__ volatile("" ::: "memory");
#endif
}

#ifndef MPCG_REC_SELECT
typedef __attribute__((address_space(3))) double lds_double;
// lanes in MASK get `on`, the others `off` (a literal lane mask: no per-step compare and no
// precomputed per-step addresses kept in registers)
__device__ __forceinline__ unsigned sel_lanes(unsigned long long mask, unsigned off, unsigned on) {
    unsigned r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(off), "v"(on), "s"(mask));
    return r;
}
__device__ __forceinline__ unsigned lds_addr(double* p) { return (unsigned)(size_t)(lds_double*)p; }
__device__ __forceinline__ void lds_store(unsigned a, double v) { *(lds_double*)(size_t)a = v; }
#endif
__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
// DPP move of both halves of a double (lanes outside row_mask keep `v`)
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), CTRL, ROW_MASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), CTRL, ROW_MASK, 0xF, false);
    return __hiloint2double(hi, lo);
}
// value of lane + p (p = 1, 2: the other parts of a stage) for part 0's fold: DPP
// whole-wave shifts (wave_shl:1) instead of ds_bpermute (-DMPCG_FOLD_BPERMUTE restores it)
__device__ __forceinline__ double lane_down(double v, int p) {
#ifdef MPCG_FOLD_BPERMUTE
    return __shfl_down(v, p);
#else
    double w = dpp_d<0x130>(v);
    if (p == 2) w = dpp_d<0x130>(w);
    return w;
#endif
}
__device__ __forceinline__ double wave_max(double v) {
#ifdef MPCG_MAX_BPERMUTE
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
#else
    // max is exact in any order: a DPP tree (quads, half rows, rows, then row 15 /
    // row 31 broadcasts) instead of six ds_bpermute levels, lane 63 broadcast
    v = fmax(v, dpp_d<0xB1>(v));        // quad_perm [1,0,3,2]
    v = fmax(v, dpp_d<0x4E>(v));        // quad_perm [2,3,0,1]
    v = fmax(v, dpp_d<0x141>(v));       // row_half_mirror
    v = fmax(v, dpp_d<0x140>(v));       // row_mirror
    v = fmax(v, dpp_d<0x142, 0xA>(v));  // row_bcast15 -> rows 1, 3
    v = fmax(v, dpp_d<0x143, 0xC>(v));  // row_bcast31 -> rows 2, 3
    return readlane_d(v, 63);
#endif
}
__device__ __forceinline__ double wave_sum(double v) {
    // the same DPP tree as wave_max: every lane gets lane 63's sum, so the result is
    // bit-identical across lanes and deterministic (one fixed association order)
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    v += dpp_d<0x142, 0xA>(v);
    v += dpp_d<0x143, 0xC>(v);
    return readlane_d(v, 63);
}


// One step of a split vector chain: h + G . v.  MPCG_CHAIN_TREE: two partial sums (the first
// half of the terms from h, the second from 0) joined by one add, so the step's dependent chain is
// ceil(n/2) + 1 operations deep instead of n (the chains are latency-bound at one wave per SIMD)
#ifndef MPCG_CHAIN_TREE
#define MPCG_CHAIN_TREE 0
#endif
template <int n>
__device__ __forceinline__ double chain_dot(double h, const double* G, const double* v) {
    if constexpr (MPCG_CHAIN_TREE) {
        constexpr int m = (n + 1) / 2;
        double a = h, b = G[m] * v[m];
#pragma unroll
        for (int j = 0; j < m; ++j) a += G[j] * v[j];
#pragma unroll
        for (int j = m + 1; j < n; ++j) b += G[j] * v[j];
        return a + b;
    } else {
        double a = h;
#pragma unroll
        for (int j = 0; j < n; ++j) a += G[j] * v[j];
        return a;
    }
}

// barrier contribution at (i, j), i >= j: diagonal part dh[0..nz) plus the
// h-row block dh[nz..nz + NBT)
template <class C>
__device__ __forceinline__ double dh_at(const double* dh, int i, int j) {
    double v = (i == j) ? dh[i] : 0.0;
    const int a = C::blk(i), c = C::blk(j);
    if (a >= 0 && c >= 0) v += dh[C::NZ + (a >= c ? cpk(C::NB, a, c) : cpk(C::NB, c, a))];
    return v;
}

// Register state of the inequality rows a lane owns (slot s).
template <class C>
struct Rows {
    double t[C::SLOTS], l[C::SLOTS], it_[C::STORE_IT ? C::SLOTS : 1], rin[C::SLOTS], pr[C::SLOTS];
    __device__ __forceinline__ double it(int s) const {
        if constexpr (C::STORE_IT) return it_[s];
        else return frcp(t[s]);
    }
    __device__ __forceinline__ void set_it(int s, double v) {
        if constexpr (C::STORE_IT) it_[s] = v;
    }
    double nlam[C::HS];  // NLP multiplier of the h row (Hessian weight of the next linearisation)
};

// The rows of the lane (stage k, part p): box slot j <-> variable v(j) = p + PARTS j,
// h slot r <-> h row hh(r) = p + PARTS r.
// Cfg::BOUNDS_SEL: the box bounds of a lane's variables are selected from the uniform problem
// arguments by the lane's part at each use (two v_cndmask per bound) instead of living in
// 2 BVS VGPR pairs for the whole solve
template <class C, bool SEL = C::BOUNDS_SEL>
struct LaneBounds {
    int k, part;
    double lo[C::BVS], hi[C::BVS];
    __device__ __forceinline__ double lo_at(int j) const { return lo[j]; }
    __device__ __forceinline__ double hi_at(int j) const { return hi[j]; }
};
template <class C>
struct LaneBounds<C, true> {
    int k, part;
    const mpcg_problem* prb;
    __device__ __forceinline__ static double bnd(const mpcg_problem& p, int v, bool upper) {
        if (v >= C::NZ) return 0.0;
        return v < C::NU ? (upper ? p.ubu[v] : p.lbu[v]) : (upper ? p.ubx[v - C::NU] : p.lbx[v - C::NU]);
    }
    __device__ __forceinline__ double sel(int j, bool upper) const {
        double b = bnd(*prb, C::PARTS * j, upper);
#pragma unroll
        for (int q = 1; q < C::PARTS; ++q) b = part == q ? bnd(*prb, q + C::PARTS * j, upper) : b;
        return b;
    }
    __device__ __forceinline__ double lo_at(int j) const { return sel(j, false); }
    __device__ __forceinline__ double hi_at(int j) const { return sel(j, true); }
};
template <class C>
struct LaneRows : LaneBounds<C> {
    using LaneBounds<C>::k;
    using LaneBounds<C>::part;
    __device__ __forceinline__ int var(int j) const { return part + C::PARTS * j; }
    __device__ __forceinline__ int hrow(int r) const { return part + C::PARTS * r; }
    // input bounds on every stage < N, state bounds on 1..N-1
    __device__ __forceinline__ bool box_on(int j) const {
        const int v = var(j);
        return v < C::NZ && (k == 0 ? v < C::NU : k < C::N);
    }
    __device__ __forceinline__ bool h_on(int r) const { return k >= 1 && k < C::N && hrow(r) < C::NH; }
};

// h values, signed gradients, bound gaps and the multiplier-weighted Hessian
// (xx xy xp yy yp pp on x, y, psi) of the h rows of a lane at stage k.
template <class C>
__device__ __forceinline__ void h_rows(const mpcg_problem& pr, const double* __restrict__ pk, const double z[C::NZ],
                                       const LaneRows<C>& LR, const double* nlam, double hb6[6],
                                       double (*Dg)[C::DGC], double* hd, double* disc) {
    const double x = z[C::IX], y = z[C::IY], psi = z[C::IPSI];
    const double rdisc = C::NE > 0 ? pk[pr.i_disc_r] : 0.0, off = pk[pr.i_disc_off];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double dxp = -off * sp, dyp = off * cp, dxpp = -off * cp, dypp = -off * sp;
    if constexpr (C::LIN_PARAMS) {
        if (LR.part == 0) { disc[0] = off * cp; disc[1] = off * sp; disc[2] = dxp; disc[3] = dyp; }
    }
#pragma unroll
    for (int r = 0; r < C::HS; ++r) {
        if (!LR.h_on(r)) continue;
        const int hh = LR.hrow(r);
        if (hh < C::NL) {
            // topology halfspace a1 x + a2 y - b <= 0 (guidance_constraints.py:355-370)
            if constexpr (!C::LIN_PARAMS) {  // else read from the parameters where used
                const double* c = pk + pr.i_lin0 + 3 * hh;
                hd[hh] = 0.0 - (c[0] * x + c[1] * y - c[2]);
                Dg[hh][0] = c[0];
                Dg[hh][1] = c[1];
                Dg[hh][2] = 0.0;
            }
        } else if (hh >= C::NL + C::NE) {
            // scenario halfspace a1 xd + a2 yd - (b + slack) <= 0 at the disc
            // position (scenario_constraints.py:64-94)
            const double* c = pk + pr.i_scen0 + 3 * (hh - C::NL - C::NE);
            if constexpr (!C::LIN_PARAMS) {
                const double sl = C::HAS_SLACK ? z[C::ZSL] : 0.0;
                hd[hh] = 0.0 - (c[0] * (x + off * cp) + c[1] * (y + off * sp) - (c[2] + sl));
                Dg[hh][0] = c[0];
                Dg[hh][1] = c[1];
                Dg[hh][2] = c[0] * dxp + c[1] * dyp;
            }
            const double wgt = nlam[r];  // upper-bound row: Hessian weight +lambda
            hb6[5] += wgt * (c[0] * dxpp + c[1] * dypp);
        } else {
            // obstacle ellipsoid d' R'DR d >= 1 (ellipsoid_constraints.py:435-489)
            const double* o = pk + pr.i_ell0 + 7 * (hh - C::NL);
            const double chi = sqrt(o[5]);
            const double ra = o[3] * chi + rdisc + o[6];
            const double rb = o[4] * chi + rdisc + o[6];
            const double D0 = frcp(ra * ra), D1 = frcp(rb * rb);
            double so, co;
            sincos(o[2], &so, &co);
            const double M00 = co * co * D0 + so * so * D1;
            const double M01 = -co * so * D0 + so * co * D1;
            const double M11 = so * so * D0 + co * co * D1;
            const double ddx = x + off * cp - o[0], ddy = y + off * sp - o[1];
            const double Mdx = M00 * ddx + M01 * ddy, Mdy = M01 * ddx + M11 * ddy;
            const int he = C::LIN_PARAMS ? hh - C::NL : hh;
            hd[he] = (ddx * Mdx + ddy * Mdy) - 1.0;
            Dg[he][0] = -2.0 * Mdx;
            Dg[he][1] = -2.0 * Mdy;
            if constexpr (!C::LIN_PARAMS) Dg[he][2] = -2.0 * (Mdx * dxp + Mdy * dyp);
            const double wgt = -nlam[r];  // lower-bound row: Hessian weight -lambda
            if (wgt != 0.0) {
                const double hxp = 2.0 * (M00 * dxp + M01 * dyp);
                const double hyp = 2.0 * (M01 * dxp + M11 * dyp);
                const double hpp = 2.0 * (dxp * (M00 * dxp + M01 * dyp) + dyp * (M01 * dxp + M11 * dyp)) +
                                   2.0 * (Mdx * dxpp + Mdy * dypp);
                hb6[0] += wgt * 2.0 * M00; hb6[1] += wgt * 2.0 * M01; hb6[2] += wgt * hxp;
                hb6[3] += wgt * 2.0 * M11; hb6[4] += wgt * hyp; hb6[5] += wgt * hpp;
            }
        }
    }
}

// The FULL variant is needed for a full SQP call (its termination test reads the NLP
// residuals) and for a first QP that starts warm; the SQP-RTI default (every QP the first
// of its acados call, cold) runs the lean one.
__host__ __device__ inline bool needs_full(const mpcg_problem& pr) {
    return pr.nlp_solver == MPCG_NLP_SQP || (pr.qp_warm_start == 2 && pr.qp_warm_first);
}

// The interior point's profile (mpcg_problem_set_qp_profile) as a template parameter of
// the kernel: the lean kernels are compiled once per profile with its structural switches (the primal box
// move, the conditional corrector, the corrector's refinement, sigma's clip, the exit order, the divergence
// test, the pivot rule) as constants, so neither profile carries the other's code or its live state.  PROF_RUNTIME reads
// them from mpcg_problem (the FULL variant, and a lean call with a combination of switches that is neither
// profile).  The continuous constants (mu0, thr0, t_min, mu_max) stay run-time arguments.
enum { PROF_RUNTIME = 0, PROF_HPIPM = 1, PROF_ROBUST = 2 };
__host__ __device__ inline int qp_profile_kind(const mpcg_problem& pr) {
    if (pr.qp_init_move == 1 && pr.qp_cond_pred_corr == 1 && pr.qp_itref_corr_max == 2 && pr.qp_sigma_clip == 0 &&
        pr.qp_maxit_first == 1 && !(pr.qp_mu_max > 0.0) && pr.qp_pivot_zero == 1)
        return PROF_HPIPM;
    if (pr.qp_init_move == 0 && pr.qp_cond_pred_corr == 0 && pr.qp_itref_corr_max == 0 && pr.qp_sigma_clip == 1 &&
        pr.qp_maxit_first == 0 && pr.qp_mu_max > 0.0 && pr.qp_pivot_zero == 0)
        return PROF_ROBUST;
    return PROF_RUNTIME;
}

// FULL: the variant with the capsule's QP memory (mpcg_io.qp_in / qp_out), the HPIPM warm
// start (pr.qp_warm_start == 2) and the NLP residuals of every linearisation
// (mpcg_io.stats; the drop-in's AcadosInfo).  The lean variant (FULL = false: cold
// start, no QP memory, no residuals) is the batched path: there the rows' interior-point
// state is rewritten at every QP start and dead across the linearisation, which keeps
// the register allocation of the hot loops (the warm start and the residual pass hold
// the previous QP's row state across the linearisation).
// MPCG_WAVES_PER_EU (register-budget experiments only): the allocator's target waves per SIMD
#ifdef MPCG_WAVES_PER_EU
#define MPCG_KERNEL_ATTR __launch_bounds__(MPCG_WG_LANES) __attribute__((amdgpu_waves_per_eu(MPCG_WAVES_PER_EU, MPCG_WAVES_PER_EU)))
#else
#define MPCG_KERNEL_ATTR __launch_bounds__(64, 1)
#endif
// one solve `sol` on the calling wavefront (the body of sqp_kernel)
template <class C, bool FULL, int PROF, int MODE>
__device__ __forceinline__ void sqp_solve(mpcg_problem pr, int batch, mpcg_io io,
                                          unsigned long long* __restrict__ stamps, double* __restrict__ gws,
                                          const int sol, const int split_it) {
#include "mpcg_sqp_body.inc"
}

// The batched solve.  queue == NULL or an instance without C::QUEUE: workgroup b solves problem b
// (a grid of `batch` workgroups).  Otherwise a grid of at most the resident workgroups (launch_instance: MPCG_QUEUE) takes the
// problems from the head of a work queue, queue[0], one at a time until it runs past `batch`:
// the hardware deals workgroups to the XCDs round robin and starts a new one only when a slot
// frees, so with a grid of one workgroup per solve each XCD works through a fixed eighth of the
// batch and every solve pays a workgroup launch; here a wave that finishes early takes the next
// solve of the whole batch (the tail).  Every wave leaves the loop on its first
// ticket >= batch.  launch_instance zeroes the queue words on the launch stream before every
// launch, so no launch depends on how the previous one on the same workspace ended.
// MODE (the split launch, split_on): MODE_LIN linearises RTI iteration split_it, MODE_QP solves its QP and
// steps; the fused kernel (MODE_FUSED) runs the whole loop
template <class C, int MODE>
__host__ __device__ constexpr bool kernel_queue() {
    return MODE == MODE_FUSED ? C::QUEUE : MODE == MODE_QP ? (MPCG_SPLIT & 2) != 0 : (MPCG_SPLIT & 4) != 0;
}
template <class C, bool FULL = false, int PROF = PROF_RUNTIME, int MODE = MODE_FUSED>
__global__ MPCG_KERNEL_ATTR void sqp_kernel(mpcg_problem pr, int batch, mpcg_io io,
                                                    unsigned long long* __restrict__ stamps,
                                                    double* __restrict__ gws, unsigned* __restrict__ queue,
                                                    int split_it) {
    static_assert(!(FULL && MODE != MODE_FUSED), "the full variant is not split");
    if constexpr (!kernel_queue<C, MODE>()) {
        (void)queue;
        const int sol = blockIdx.x;
#include "mpcg_sqp_body.inc"
    } else {
        if (blockDim.x != 64) {
            // the lane exchanges assume one wavefront per workgroup (wave_sync): any other launch
            // shape reports an invalid exit code instead of racing
            if (threadIdx.x == 0)
                for (int sol = blockIdx.x; sol < batch; sol += gridDim.x) io.exit_code[sol] = -1;
            return;
        }
        const bool q = queue != nullptr;
        // (a ticket past INT_MAX -- a queue left non-zero by an aborted launch -- ends the loop too)
        auto next = [&]() -> int {
            unsigned t = 0;
            if (threadIdx.x == 0) t = atomicAdd(&queue[0], 1u);
            t = __builtin_amdgcn_readfirstlane(t);
            return t < (unsigned)batch ? (int)t : batch;
        };
        for (int sol = q ? next() : (int)blockIdx.x; sol < batch; sol = q ? next() : batch) {
            sqp_solve<C, FULL, PROF, MODE>(pr, batch, io, stamps, gws, sol, split_it);
            wave_sync();
        }
    }
}

}  // namespace mpcg
