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
    // 1/t of every row kept in registers when the row state is small (up to 14 slots) on the
    // three-part instances (C1, C2, C5); the instances with more row slots per lane (C4 20, C3 16)
    // recompute it, which keeps them out of scratch.  The two-part instances (JS, JD) recompute it
    // too: the round-2 build that stored 1/t on a two-part instance computed wrong trajectories
    // and faulted once, and its cause was never named, so the gate stays until it
    // is.  Measured with the gate lifted (-DMPCG_STORE_IT_ANY; scripts/ab_bench.py,
    // profiles/r03d_ab_*): JS 42.11 -> 41.39 ms, JD unchanged; full-size parity passed that way
    // (profiles/r03c_variant_storeit.jsonl).  C5 stored: 20.89 -> 20.68 ms.  Without it C5 is
    // scratch-free (28 B/lane with it) but slower, 20.69 -> 20.91 (profiles/r03k_ab.jsonl,
    // MPCG_STORE_IT_MAX=12).  MPCG_STORE_IT_MAX=0 recomputes it everywhere.
#ifndef MPCG_STORE_IT_MAX
#define MPCG_STORE_IT_MAX 14
#endif
#ifdef MPCG_STORE_IT_ANY
    static constexpr bool STORE_IT_PARTS_OK = true;
#else
    static constexpr bool STORE_IT_PARTS_OK = PARTS == 3;
#endif
    static constexpr bool STORE_IT = SLOTS <= MPCG_STORE_IT_MAX && STORE_IT_PARTS_OK;
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

// Diagnostic per-phase cycle stamps (separate build with -DMPCG_STAMPS; the
// production build compiles them out).  Read shares, not absolute times.
#ifdef MPCG_STAMPS
#define MPCG_NSTAMP 20
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
template <class C, bool FULL>
__device__ __forceinline__ void sqp_solve(mpcg_problem pr, int batch, mpcg_io io,
                                          unsigned long long* __restrict__ stamps, double* __restrict__ gws,
                                          const int sol) {
    constexpr int N = C::N, PARTS = C::PARTS, NX = C::NX, NZ = C::NZ, NB = C::NB, NBT = C::NBT;
    constexpr int NU = C::NU;   // (shadows the unicycle's mpcg::NU)
    constexpr int ZS = C::ZSL;  // slack variable (NB == 4)
    constexpr int X0 = C::IX, X1 = C::IY, X2 = C::IPSI;
    constexpr bool LEAN = lds_lean<C>();
    constexpr bool GFH = lds_gfh<C>();
    // the predictor's barrier pass fused into the residual pass: its barrier terms come from the row
    // state the residual pass has just computed, with the same operations, and one box-sum exchange,
    // loop and fold fewer per interior-point iteration (wasted only on the iteration that exits).
    // Measured (profiles/r03q_ab.jsonl, two alternating repetitions): C2 12.32 -> 11.97 ms, C1 10.61
    // -> 10.43, C4 47.48 -> 45.38, C5 20.60 -> 19.46, JS 38.32 -> 37.17; C3 20.30 -> 19.81
    // (profiles/r03s_ab.jsonl).  (MPCG_FUSE_BAR=0: A/B)
#ifndef MPCG_FUSE_BAR
#define MPCG_FUSE_BAR 1
#endif
    constexpr bool FUSE_BAR = MPCG_FUSE_BAR > 0;
    // RES_SPLIT: the stage algebra of the residual and barrier passes (H dz, the stationarity rows,
    // the Newton gradient, the dynamics rows) split over the parts of a stage -- part p owns the
    // rows of its box variables p, p + PARTS, ... (and dynamics rows p, p + PARTS, ...), whose box
    // sums it holds in registers -- instead of one stage lane doing all of them while the other
    // parts wait.  Same operations per row.  Measured (profiles/r03r_ab.jsonl, two alternating
    // repetitions): C2 11.99 -> 11.68 ms, C1 10.42 -> 10.15, C5 unchanged; on the two-part long
    // horizons it moves the allocation into scratch (C4 45.29 -> 46.76, JD 40.45 -> 40.70, JS
    // 37.25 -> 37.13), so three-part instances only; and not on the slack model, where it was neutral
    // in time but moved the allocation into scratch (C5 52 -> 188 B/lane, 264 -> 782 MB of HBM traffic
    // per launch, profiles/r03u_c5_pmc.json).  (MPCG_RES_SPLIT=0: off, 2: every instance)
#ifndef MPCG_RES_SPLIT
#define MPCG_RES_SPLIT 1
#endif
    constexpr bool RES_SPLIT = MPCG_RES_SPLIT > 0 && FUSE_BAR && !C::COMPACT && PARTS > 1 && 2 * NB <= NZ &&
                               ((PARTS == 3 && NX == 5) || MPCG_RES_SPLIT > 1);
    constexpr int DRS = (NX + PARTS - 1) / PARTS;  // dynamics rows per part
    // MIRROR's eigenvector rows split over the parts of a stage (MPCG_MSPLIT=1, A/B only): bit-identical
    // outputs (scripts/bitcmp.py on C2, C5, C4, JS: profiles/r03t_bitcmp.log) but slower everywhere --
    // the stage matrix and row exchanges and the longer-lived state push the linearisation into
    // scratch: C2 11.65 -> 12.46 ms, C1 10.16 -> 10.45, C4 45.41 -> 50.57, C5 19.47 -> 21.53, JS
    // 37.24 -> 39.63, JD 40.56 -> 43.38 (profiles/r03t_ab.jsonl)
#ifndef MPCG_MSPLIT
#define MPCG_MSPLIT 0
#endif
    constexpr bool MSPLIT = MPCG_MSPLIT > 0 && C::MODEL == 0;
    // the feedback's new dynamics multipliers split over the parts too (MPCG_PIN_SPLIT=1, A/B only:
    // measured slower, C2 11.69 -> 11.78 ms, C1 10.16 -> 10.22, C5 unchanged; profiles/r03s_ab.jsonl)
#ifndef MPCG_PIN_SPLIT
#define MPCG_PIN_SPLIT 0
#endif
    constexpr bool PIN_SPLIT = MPCG_PIN_SPLIT > 0 && RES_SPLIT && !LEAN && C::CHAIN_SPLIT;
    __shared__ LdsOf<C> S;
#ifdef MPCG_LDS_PAD
    // occupancy experiment only: pad the LDS footprint
    __shared__ char lds_pad[MPCG_LDS_PAD];
    if (threadIdx.x == 1000) lds_pad[blockIdx.x % MPCG_LDS_PAD] = 0;
#endif
    if (sol >= batch) return;
    // the lane exchanges assume one wavefront per workgroup (wave_sync): any other launch
    // shape reports an invalid exit code instead of racing
    if (blockDim.x != 64) {
        if (threadIdx.x == 0) io.exit_code[sol] = -1;
        return;
    }
    // (laundered per solve: with the work queue this body is a loop, and nothing lane-dependent
    // may be hoisted out of it to stay live across solves)
    int lane_ = threadIdx.x;
    if constexpr (C::QUEUE) __asm__ volatile("" : "+v"(lane_));
    const int lane = lane_;
    const int k = lane / PARTS;          // my stage
    const int part = lane - k * PARTS;   // my part
    const bool stage_lane = (part == 0) && (k <= N);
    const int ks = k <= N ? k : N;       // clamped stage (always a valid LDS index)
    const int kc = k < N ? k : N - 1;    // clamped stage < N
    const int npar = pr.npar;
    constexpr int LAMS = NX + C::NH;  // multiplier block per stage (include/mpcg.h, mpcg_io)
#ifdef MPCG_DIAG_PARAMS_OF
    // diagnostic build only (scripts/param_locality.py): solve sol reads the parameter block of
    // solve sol % MPCG_DIAG_PARAMS_OF (a batch of identical copies: the cost of the parameter reads'
    // misses)
    const double* pbase = io.params + (size_t)(sol % MPCG_DIAG_PARAMS_OF) * N * npar;
#else
    const double* pbase = io.params + (size_t)sol * N * npar;
#endif
    const double* pk = pbase + (size_t)kc * npar;
    (void)stamps;
    // the stage blocks [B A] (Fb) and H (Hb): LDS, or this solve's global workspace (GFH)
    double* const gF = GFH ? gws + (size_t)sol * gfh_doubles<C>() : nullptr;
    double* const gH = GFH ? gF + (size_t)N * C::NFR * C::NFC : nullptr;
    auto Fb = [&](int kq) -> double (*)[C::NFC] {
        if constexpr (GFH) return (double (*)[C::NFC])(gF + (size_t)kq * C::NFR * C::NFC);
        else return S.F[kq];
    };
    auto Hb = [&](int kq) -> double* {
        if constexpr (GFH) return gH + (size_t)kq * C::NHP;
        else return S.H[kq];
    };
    STAMP_DECL

    // NLP multipliers carried over from the previous solve of this planner
    // (zero for a fresh or reset acados capsule)
    const double* lam_in = io.lam_in ? io.lam_in + (size_t)sol * N * LAMS : nullptr;
    constexpr int BVS = C::BVS, HS = C::HS, HB = 2 * C::BVS;  // HB: first h slot
    LaneRows<C> LR;
    LR.k = k;
    LR.part = part;
    if constexpr (C::BOUNDS_SEL) {
        LR.prb = &pr;
    } else {
#pragma unroll
        for (int j = 0; j < BVS; ++j) {
            const int v = LR.var(j);
            double lo = 0.0, hi = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; ++i)
                if (v == i) { lo = i < NU ? pr.lbu[i] : pr.lbx[i - NU]; hi = i < NU ? pr.ubu[i] : pr.ubx[i - NU]; }
            LR.lo[j] = lo;
            LR.hi[j] = hi;
        }
    }
    // gradient (x, y, psi) and gap of h row hh of this lane's stage
    auto rowg = [&](int hh, double& a, double& b, double& c) {
        if constexpr (C::LIN_PARAMS) {
            if (hh < C::NL || hh >= C::NL + C::NE) {
                const double* p = hh < C::NL ? pk + pr.i_lin0 + 3 * hh : pk + pr.i_scen0 + 3 * (hh - C::NL - C::NE);
                a = p[0];
                b = p[1];
                c = hh < C::NL ? 0.0 : p[0] * S.disc[k][2] + p[1] * S.disc[k][3];
                return;
            }
            const int he = hh - C::NL;
            a = S.Dg[k][he * C::DGC + 0];
            b = S.Dg[k][he * C::DGC + 1];
            c = a * S.disc[k][2] + b * S.disc[k][3];
        } else {
            a = S.Dg[k][hh * C::DGC + 0]; b = S.Dg[k][hh * C::DGC + 1]; c = S.Dg[k][hh * C::DGC + 2];
        }
    };
    auto rowgap = [&](int hh) -> double {
        if constexpr (C::LIN_PARAMS) {
            const double x = S.z[k][X0], y = S.z[k][X1];
            if (hh < C::NL) {
                const double* p = pk + pr.i_lin0 + 3 * hh;
                return 0.0 - (p[0] * x + p[1] * y - p[2]);
            }
            if (hh >= C::NL + C::NE) {
                const double* p = pk + pr.i_scen0 + 3 * (hh - C::NL - C::NE);
                const double sl = C::HAS_SLACK ? S.z[k][ZS] : 0.0;
                return 0.0 - (p[0] * (x + S.disc[k][0]) + p[1] * (y + S.disc[k][1]) - (p[2] + sl));
            }
            return S.hd[k][hh - C::NL];
        } else {
            return S.hd[k][hh];
        }
    };
    // [B A] and Hessian entries of stage kq (the compact C3 storage rebuilds the known ones)
    // the s+ row's coefficients of a and v (uniform, bit-identical to erk_unicycle's)
    double srow_a = 0.0, srow_v = 0.0;
    if constexpr (C::FCONST) erk_srow(pr, srow_a, srow_v);
    auto FatB = [&](const double (*Fk)[C::NFC], int m, int j) -> double {
        if constexpr (C::FCONST) {
            // rows psi+, v+, s+ (, slack+) are constants (z = [a w x y psi v s (slack)])
            if (m == 2) return j == 1 ? pr.dt : (j == 4 ? 1.0 : 0.0);
            if (m == 3) return j == 0 ? pr.dt : (j == 5 ? 1.0 : 0.0);
            if (m == 4) return j == 0 ? srow_a : (j == 5 ? srow_v : (j == 6 ? 1.0 : 0.0));
            if (m >= 5) return j == NU + m ? 1.0 : 0.0;
            return Fk[m][j];
        } else if constexpr (C::COMPACT) {
            if (m == 3) return j == bike::ZV ? 1.0 : (j == bike::ZA ? pr.dt : 0.0);
            if (m == 4) return j == bike::ZDELTA ? 1.0 : (j == bike::ZW ? pr.dt : 0.0);
            if (j == ZS) return 0.0;
            return Fk[m < 3 ? m : 3][j < ZS ? j : j - 1];
        } else {
            return Fk[m][j];
        }
    };
    auto HatB = [&](const double* Hk, int i, int j) -> double {
        if constexpr (C::COMPACT) {
            if (i == ZS || j == ZS) return (i == j) ? Hk[C::NHP - 1] : 0.0;
            return Hk[sym(i < ZS ? i : i - 1, j < ZS ? j : j - 1)];
        } else {
            return Hk[sym(i, j)];
        }
    };
    auto Fat = [&](int kq, int m, int j) -> double { return FatB(Fb(kq), m, j); };
    auto Hat = [&](int kq, int i, int j) -> double { return HatB(Hb(kq), i, j); };
    // dynamics residual b + F dz - dz+ of stage kq at the current QP iterate (same operation order
    // as the residual phase, which stores it unless C::COMPACT)
    auto rdyn_at = [&](int kq, int i) -> double {
        double a = S.b[kq][i] - S.dz[kq + 1][NU + i];
#pragma unroll
        for (int j = 0; j < NZ; ++j) a += Fat(kq, i, j) * S.dz[kq][j];
        return a;
    };
    Rows<C> R;
#pragma unroll
    for (int r = 0; r < HS; ++r) R.nlam[r] = (lam_in && LR.h_on(r)) ? lam_in[(size_t)k * LAMS + NX + LR.hrow(r)] : 0.0;

    // ---- load warm start (loadWarmstart, acados_solver_interface.cpp:274-284)
    const double* w = io.warm + (size_t)sol * (N + 1) * NZ;
    for (int e = lane; e < (N + 1) * NZ; e += 64) (&S.z[0][0])[e] = w[e];
    if (lane < NX) S.xinit[lane] = io.xinit[(size_t)sol * NX + lane];
    for (int e = lane; e < N * NX; e += 64)
        (&S.pi_nlp[0][0])[e] = lam_in ? lam_in[(size_t)(e / NX) * LAMS + e % NX] : 0.0;
    for (int e = lane; e <= N; e += 64) S.dH[e][C::NDH - 1] = 0.0;
    // the capsule's QP memory, if any: the previous QP's solution, whose row multipliers are
    // also the NLP's (FIXED_STEP) -- read by the NLP residuals -- and, with the HPIPM warm
    // start (qp_solver_warm_start 2), the initial point of the first QP; the later QPs
    // start from their predecessor's solution
    const bool qp_warm = FULL && pr.qp_warm_start == 2;
    // solver_type SQP: one acados SQP call (acados_solver_interface.cpp:27-29), terminated by the
    // NLP residuals (FULL only)
    const bool sqp_mode = FULL && pr.nlp_solver == MPCG_NLP_SQP;
    bool have_qp = false;
    if (FULL && io.qp_in && !isnan(io.qp_in[(size_t)sol * C::QPM])) {
        const double* q = io.qp_in + (size_t)sol * C::QPM;
#pragma unroll
        for (int sl = 0; sl < C::SLOTS; ++sl) {
            R.t[sl] = q[(2 * sl) * 64 + lane];
            R.l[sl] = q[(2 * sl + 1) * 64 + lane];
        }
        for (int e = lane; e < (N + 1) * NZ; e += 64) (&S.dz[0][0])[e] = q[C::QPM_ROWS + e];
        for (int e = lane; e < N * NX; e += 64) (&S.piq[0][0])[e] = q[C::QPM_ROWS + (N + 1) * NZ + e];
        have_qp = true;
    }
    wave_sync();
    if (lane < NU) S.z[N][lane] = 0.0;
    wave_sync();

    // the interior point's divergence test and t / lambda floor, read once
    const double mu_max = pr.qp_mu_max, tmin = pr.qp_t_min;
    int acados_status = AC_SUCCESS, qp_status = AC_SUCCESS, sqp_iter = 0, qp_total = 0, n_maxit = 0;
    double res_eq = 0.0;
    double nlp_stat = 0.0, nlp_ineq = 0.0, nlp_comp = 0.0;  // NLP residuals of the last linearisation
    bool nlp_nonfinite = false;

    for (int it = 0; sqp_mode || it < pr.sqp_iters; ++it) {
        // parameter loads are re-issued where they are used rather than hoisted out of
        // the SQP / QP loops into registers that stay live (and spill) across them
        if constexpr (C::RELOAD_PARAMS) asm volatile("" : "+v"(pk));
        // =============== preparation: linearise every stage ===============
        STAMP_BEGIN();
        {
            double zk[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) zk[i] = S.z[ks][i];
            double hb6[6] = {0, 0, 0, 0, 0, 0};
            if (k >= 1 && k < N) h_rows<C>(pr, pk, zk, LR, R.nlam, hb6, (double (*)[C::DGC])S.Dg[k], S.hd[k], S.disc[C::LIN_PARAMS ? k : 0]);
            STAMP_LAP(10);
            // fold the h-row Hessian terms of parts 1.. into part 0 (fixed order)
            {
                double acc[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) acc[i] = hb6[i];
#pragma unroll
                for (int p = 1; p < PARTS; ++p)
#pragma unroll
                    for (int i = 0; i < 6; ++i) acc[i] += lane_down(hb6[i], p);
#pragma unroll
                for (int i = 0; i < 6; ++i) hb6[i] = acc[i];
            }
            double resl = 0.0;
            // MSPLIT: the MIRROR sweeps run on all parts of a stage, each accumulating its rows of the
            // eigenvectors (mirror_rows); the stage matrix goes out from part 0 and the other parts'
            // rows come back through MX, a per-stage exchange area over the Riccati arrays P, Lc, Y
            // and the box sums (all dead during the linearisation)
            constexpr int MNA = NZ == 8 ? NZ - 1 : NZ;  // the slack model's decoupled slack diagonal aside
            constexpr int MRV = (MNA + PARTS - 1) / PARTS;
            constexpr int MXS = imax(MNA * (MNA + 1) / 2, (MNA - (MNA + PARTS - 1) / PARTS) * MNA) + 1;
            double* const MX = &S.P[0][0];
            static_assert(!MSPLIT || offsetof(LdsOf<C>, Dg) - offsetof(LdsOf<C>, P) >= sizeof(double) * N * MXS,
                          "MIRROR exchange area (P, Lc, Y, bx)");
            double H[NZ][NZ];
            if (stage_lane && k < N) {
                double g[NZ], xn[NX], pi[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) pi[i] = S.pi_nlp[k][i];
                if constexpr (C::MODEL == 1) {
                    // the bicycle: the discrete map first (F and its Hessian straight to the stage's
                    // LDS blocks, H[k] rewritten below), then the cost, so that the map's jets and the
                    // 9x9 cost block are not live together
                    double* const Hd = Hb(k);
                    bike::discrete(pr, pk, zk, pi, xn, Fb(k), Hd);
                    STAMP_LAP(12);
                    bike::stage_cost(pr, pk, k, zk, g, H, true);
                    STAMP_LAP(11);
#pragma unroll
                    for (int i = 0; i < NZ; ++i)
#pragma unroll
                        for (int j = 0; j < NZ; ++j)
                            if (i != ZS && j != ZS) H[i][j] += Hd[sym(i < ZS ? i : i - 1, j < ZS ? j : j - 1)];
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        const double bi = xn[i] - S.z[k + 1][NU + i];
                        S.b[k][i] = bi;
                        resl = fmax(resl, fabs(bi));
                    }
                } else {
                    double F[NX][NZ];
                    stage_cost<NX>(pr, pk, zk, g, H, true);
                    STAMP_LAP(11);
                    erk_unicycle<NX>(pr, zk, pi, xn, F, H);
                    STAMP_LAP(12);
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        const double bi = xn[i] - S.z[k + 1][NU + i];
                        S.b[k][i] = bi;
                        resl = fmax(resl, fabs(bi));
                        if (i < C::NFR) {
#pragma unroll
                            for (int j = 0; j < NZ; ++j) Fb(k)[i][j] = F[i][j];
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < NZ; ++i) S.g[k][i] = g[i];
                H[X0][X0] += hb6[0]; H[X0][X1] += hb6[1]; H[X1][X0] += hb6[1];
                H[X0][X2] += hb6[2]; H[X2][X0] += hb6[2];
                H[X1][X1] += hb6[3]; H[X1][X2] += hb6[4]; H[X2][X1] += hb6[4];
                H[X2][X2] += hb6[5];
                STAMP_LAP(13);
                if constexpr (MSPLIT) {
                    // mirror()'s symmetrisation, then the upper triangle (and the slack diagonal's
                    // square, which enters the sweeps' convergence test) to the stage's exchange slot
#pragma unroll
                    for (int i = 0; i < MNA; ++i)
#pragma unroll
                        for (int j = i + 1; j < MNA; ++j) H[i][j] = 0.5 * (H[i][j] + H[j][i]);
#pragma unroll
                    for (int i = 0; i < MNA; ++i)
#pragma unroll
                        for (int j = i; j < MNA; ++j) MX[k * MXS + sym(j, i)] = H[i][j];
                    MX[k * MXS + MXS - 1] = NZ == 8 ? H[NZ - 1][NZ - 1] * H[NZ - 1][NZ - 1] : 0.0;
                } else if constexpr (C::MODEL == 0 && NZ == 8) {
                    // the slack row/column of the slack model is exactly zero off the
                    // diagonal (quadratic slack cost, linear in every h row, no dynamics
                    // coupling): MIRROR of the 8x8 block = MIRROR of the leading 7x7 block
                    // plus the mirrored slack diagonal, with the same sweep count
                    const double hs = H[NZ - 1][NZ - 1];
                    mirror<NZ, NZ - 1>(H, pr.reg_eps, hs * hs);
                    H[NZ - 1][NZ - 1] = (hs >= -pr.reg_eps && hs <= pr.reg_eps) ? pr.reg_eps : fabs(hs);
                } else if constexpr (C::MODEL == 1) {
                    // the bicycle's slack input is decoupled the same way (quadratic cost, linear
                    // in the decomp rows, no dynamics): with the slack moved last, MIRROR of the
                    // leading 8x8 block (the 9x9 sweep's rotation order restricted to the other
                    // variables) plus the mirrored slack diagonal
                    double Hp[NZ][NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i)
#pragma unroll
                        for (int j = 0; j < NZ; ++j) {
                            const int pi2 = i == NZ - 1 ? ZS : (i < ZS ? i : i + 1);
                            const int pj2 = j == NZ - 1 ? ZS : (j < ZS ? j : j + 1);
                            Hp[i][j] = H[pi2][pj2];
                        }
                    const double hs = Hp[NZ - 1][NZ - 1];
                    mirror<NZ, NZ - 1>(Hp, pr.reg_eps, hs * hs);
                    Hp[NZ - 1][NZ - 1] = (hs >= -pr.reg_eps && hs <= pr.reg_eps) ? pr.reg_eps : fabs(hs);
#pragma unroll
                    for (int i = 0; i < NZ; ++i)
#pragma unroll
                        for (int j = 0; j < NZ; ++j) {
                            const int pi2 = i == NZ - 1 ? ZS : (i < ZS ? i : i + 1);
                            const int pj2 = j == NZ - 1 ? ZS : (j < ZS ? j : j + 1);
                            H[pi2][pj2] = Hp[i][j];
                        }
                } else {
                    mirror<NZ>(H, pr.reg_eps);
                }
                STAMP_LAP(14);
                if constexpr (MSPLIT) {
                } else if constexpr (C::COMPACT) {
#pragma unroll
                    for (int i = 0; i < NZ; ++i)
#pragma unroll
                        for (int j = 0; j <= i; ++j)
                            if (i != ZS && j != ZS) Hb(k)[sym(i < ZS ? i : i - 1, j < ZS ? j : j - 1)] = H[i][j];
                    Hb(k)[C::NHP - 1] = H[ZS][ZS];
                } else {
#pragma unroll
                    for (int i = 0; i < NZ; ++i)
#pragma unroll
                        for (int j = 0; j <= i; ++j) Hb(k)[sym(i, j)] = H[i][j];
                }
            } else if (stage_lane && k == N) {
#pragma unroll
                for (int i = 0; i < NZ; ++i) S.g[N][i] = 0.0;
#pragma unroll
                for (int e = 0; e < C::NHP; ++e) Hb(N)[e] = 0.0;
#pragma unroll
                for (int i = NU; i < NZ; ++i) {
                    if constexpr (C::COMPACT) Hb(N)[sym(i - 1, i - 1)] = pr.reg_eps;
                    else Hb(N)[sym(i, i)] = pr.reg_eps;
                }
            }
            if constexpr (MSPLIT) {
                wave_sync();
                if (k < N) {
                    double dx2 = 0.0;
                    if (part != 0) {
#pragma unroll
                        for (int i = 0; i < MNA; ++i)
#pragma unroll
                            for (int j = i; j < MNA; ++j) H[i][j] = MX[k * MXS + sym(j, i)];
                    }
                    dx2 = MX[k * MXS + MXS - 1];
                    double Vr[MRV][MNA];
                    mirror_rows<NZ, MNA, PARTS>(H, Vr, part, dx2);
                    wave_sync();  // every part has read the stage matrix
                    if (part != 0) {
#pragma unroll
                        for (int t = 0; t < MRV; ++t) {
                            const int r = part + PARTS * t;
                            if (r >= MNA) continue;
                            const int sl = r - 1 - (r - 1) / PARTS;  // rank among the rows of parts 1..
#pragma unroll
                            for (int j = 0; j < MNA; ++j) MX[k * MXS + sl * MNA + j] = Vr[t][j];
                        }
                    }
                    wave_sync();
                    if (part == 0) {
                        double V[MNA][MNA];
#pragma unroll
                        for (int r = 0; r < MNA; ++r) {
                            if (r % PARTS == 0) {
#pragma unroll
                                for (int j = 0; j < MNA; ++j) V[r][j] = Vr[r / PARTS][j];
                            } else {
                                const int sl = r - 1 - (r - 1) / PARTS;
#pragma unroll
                                for (int j = 0; j < MNA; ++j) V[r][j] = MX[k * MXS + sl * MNA + j];
                            }
                        }
                        mirror_rebuild<NZ, MNA>(H, V, pr.reg_eps);
                        if constexpr (NZ == 8) {
                            const double hs = H[NZ - 1][NZ - 1];
                            H[NZ - 1][NZ - 1] = (hs >= -pr.reg_eps && hs <= pr.reg_eps) ? pr.reg_eps : fabs(hs);
                        }
#pragma unroll
                        for (int i = 0; i < NZ; ++i)
#pragma unroll
                            for (int j = 0; j <= i; ++j) Hb(k)[sym(i, j)] = H[i][j];
                    }
                }
            }
            res_eq = wave_max(resl);
            if (lane < NX) S.dz[0][NU + lane] = S.xinit[lane] - S.z[0][NU + lane];
        }
        // GFH: the stage lanes' global stores of the blocks complete before any lane reads them
        if constexpr (GFH) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        wave_sync();
        STAMP_END(0);

        // =============== feedback: QP by Riccati interior point ===============
        STAMP_BEGIN();
        if (FULL && (io.stats || sqp_mode)) {
            // NLP residuals at the linearisation point (acados ocp_nlp_res_compute) with the
            // multipliers the NLP holds: pi_nlp and, per row, the previous QP's multiplier
            // (FIXED_STEP: lam = lam_qp) or, before any QP, the carried h-row ones (box 0)
            double rh[NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) rh[i] = 0.0;
            double vin = 0.0, vcp = 0.0, vst = 0.0;
            // non-finite guard: 0 x every residual operand is NaN iff the operand is not finite (the
            // fmax reductions below drop NaN, so a NaN iterate could otherwise pass the SQP test)
            double chk = 0.0;
#pragma unroll
            for (int j = 0; j < BVS; ++j) {
                double lb = 0.0;
                if (LR.box_on(j)) {
                    const double zv = S.z[k][LR.var(j)];
                    const double gl = zv - LR.lo_at(j), gh = LR.hi_at(j) - zv;
                    const double ll = have_qp ? R.l[2 * j] : 0.0, lh = have_qp ? R.l[2 * j + 1] : 0.0;
                    chk += 0.0 * (zv + ll + lh);
                    vin = fmax(vin, -gl);
                    vin = fmax(vin, -gh);
                    vcp = fmax(vcp, fabs(ll * gl));
                    vcp = fmax(vcp, fabs(lh * gh));
                    lb = lh - ll;
                }
                if (k <= N && LR.var(j) < NZ) S.bx[k][LR.var(j)] = lb;
            }
#pragma unroll
            for (int r = 0; r < HS; ++r) {
                if (!LR.h_on(r)) continue;
                const int hh = LR.hrow(r);
                double a, bq, c;
                rowg(hh, a, bq, c);
                const double gap = rowgap(hh);
                const double lam = have_qp ? R.l[HB + r] : R.nlam[r];
                rh[0] += a * lam; rh[1] += bq * lam; rh[2] += c * lam;
                if constexpr (NB == 4) rh[3] += C::slack_coef(hh) * lam;
                vin = fmax(vin, -gap);
                vcp = fmax(vcp, fabs(lam * gap));
                chk += 0.0 * (gap + lam);
            }
            double acc[NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) acc[i] = rh[i];
#pragma unroll
            for (int p = 1; p < PARTS; ++p)
#pragma unroll
                for (int i = 0; i < NB; ++i) acc[i] += lane_down(rh[i], p);
            wave_sync();  // the owner lanes' box sums S.bx
            if (stage_lane) {
                double r[NZ];
#pragma unroll
                for (int i = 0; i < NZ; ++i) r[i] = S.g[k][i] + S.bx[k][i];
#pragma unroll
                for (int i = 0; i < NB; ++i) r[C::bvar(i)] += acc[i];
                if (k < N) {
#pragma unroll
                    for (int m = 0; m < NX; ++m) {
                        const double pm = S.pi_nlp[k][m];
#pragma unroll
                        for (int i = 0; i < NZ; ++i) r[i] += Fat(k, m, i) * pm;
                    }
                }
                if (k > 0) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) r[NU + i] -= S.pi_nlp[k - 1][i];
                }
#pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    const bool free_var = (k == N) ? (i >= NU) : ((k == 0) ? (i < NU) : true);
                    if (free_var) vst = fmax(vst, fabs(r[i]));
                    chk += 0.0 * r[i];
                }
                if (k < N) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) chk += 0.0 * S.b[k][i];  // res_eq's operands
                }
            }
            nlp_stat = wave_max(vst);
            nlp_ineq = wave_max(vin);
            nlp_comp = wave_max(vcp);
            nlp_nonfinite = !(wave_sum(chk) == 0.0);
            wave_sync();
        }
        if (sqp_mode) {
            // a non-finite NLP residual ends the call with the NaN status (an iterate gone non-finite
            // after an applied max-iter QP step would otherwise run every remaining iteration)
            if (nlp_nonfinite) {
                acados_status = AC_NAN;
                break;
            }
            // acados SQP: converged at this linearisation point, or out of iterations (its
            // residuals and res_eq are the final iterate's either way)
            if (nlp_stat < pr.nlp_tol && res_eq < pr.nlp_tol && nlp_ineq < pr.nlp_tol && nlp_comp < pr.nlp_tol) {
                acados_status = AC_SUCCESS;
                break;
            }
            if (it >= pr.nlp_max_iter) {
                acados_status = AC_MAXITER;
                break;
            }
        }
        // HPIPM warm start for every QP of an acados call after its first (SQP: it > 0), and for
        // the first with warm_start_first_qp; SQP-RTI calls consist of one QP each
        const bool warm_now = qp_warm && have_qp && ((sqp_mode && it > 0) || pr.qp_warm_first);
        if (warm_now) {
            // HPIPM warm_start 2 (d_ocp_qp_ipm init_var): the previous QP's solution is the
            // initial point -- step and dynamics multipliers stay in LDS, the rows' slacks and
            // multipliers in registers -- with slacks and multipliers clipped below at thr0
            const double thr = pr.qp_ws_thr;
#pragma unroll
            for (int sl = 0; sl < C::SLOTS; ++sl) {
                if (R.t[sl] < thr) R.t[sl] = thr;
                if (R.l[sl] < thr) R.l[sl] = thr;
                R.pr[sl] = 0.0;
            }
        } else {
        // cold start: t = max(gap, thr0), l = mu0 / t
        {
            auto cold = [&](int s, double gap) {
                const double t0 = gap > pr.qp_thr0 ? gap : pr.qp_thr0;
                R.t[s] = t0;
                R.l[s] = pr.qp_mu0 / t0;
                R.pr[s] = 0.0;
            };
            // every slot is (re)written, inactive ones with placeholders that are never
            // read: the row state is then dead between two QPs and the linearisation
            // does not have to keep it in registers
#pragma unroll
            for (int j = 0; j < BVS; ++j) {
                const bool on = LR.box_on(j);
                const double zv = S.z[ks][on ? LR.var(j) : 0];
                cold(2 * j, on ? zv - LR.lo_at(j) : 1.0);
                cold(2 * j + 1, on ? LR.hi_at(j) - zv : 1.0);
            }
#pragma unroll
            for (int r = 0; r < HS; ++r) {
                const bool on = LR.h_on(r);
                cold(HB + r, on ? rowgap(on ? LR.hrow(r) : 0) : 1.0);
            }
        }
        if (stage_lane) {
#pragma unroll
            for (int i = 0; i < NZ; ++i)
                if (!(k == 0 && i >= NU)) S.dz[k][i] = 0.0;
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.piq[k][i] = 0.0;
            }
        }
        }
        have_qp = true;
        wave_sync();
        STAMP_END(1);
        int qstat = AC_MAXITER, qit = 0;
        double pinr[LEAN ? NX : 1];  // LEAN: the new dynamics multipliers of the own stage
        double Hdz[RES_SPLIT ? BVS : NZ];  // H_k dz_k of the current iterate: part 0 (RES_SPLIT: the lane's variables)
        for (;; ++qit) {
            if constexpr (C::RELOAD_PARAMS) asm volatile("" : "+v"(pk));
            // ---- residuals
            STAMP_BEGIN();
            double rs = 0.0, re = 0.0, ri = 0.0, comp = 0.0;
            {
                double zk[NZ], dzk[NZ];
#pragma unroll
                for (int i = 0; i < NZ; ++i) { dzk[i] = S.dz[ks][i]; zk[i] = S.z[ks][i]; }
                double rh[NB], qh[NB], dbh[NBT], rbj[BVS], qbj[BVS];
#pragma unroll
                for (int i = 0; i < NB; ++i) rh[i] = qh[i] = 0.0;
#pragma unroll
                for (int i = 0; i < NBT; ++i) dbh[i] = 0.0;
                // FUSE_BAR: the predictor's barrier terms (rc = l t, the same operations as the
                // barrier pass) from the row state just computed
                auto bar0 = [&](int s, double& coef, double& wgt) {
                    const double l = R.l[s], t = R.t[s], itt = R.it(s);
                    const double rc = l * t;
                    coef = l + (l * R.rin[s] - rc) * itt;
                    wgt = l * itt;
                };
                auto row_res = [&](int s, double ddot, double gap) {
                    const double l = R.l[s], t = R.t[s];
                    const double rin = ddot + t - gap;
                    R.rin[s] = rin;
                    R.set_it(s, frcp(t));
                    ri = fmax(ri, fabs(rin));
                    comp += l * t;
                };
#pragma unroll
                for (int j = 0; j < BVS; ++j) {
                    double& rb = rbj[j];
                    double& qb = qbj[j];
                    double dd = 0.0;
                    rb = qb = 0.0;
                    if (LR.box_on(j)) {
                        const int v = LR.var(j);
                        const double zv = S.z[k][v], dzv = S.dz[k][v];
                        rb = R.l[2 * j + 1] - R.l[2 * j];
                        row_res(2 * j, -dzv, zv - LR.lo_at(j));
                        row_res(2 * j + 1, dzv, LR.hi_at(j) - zv);
                        if constexpr (FUSE_BAR) {
                            double c0, w0, c1, w1;
                            bar0(2 * j, c0, w0);
                            bar0(2 * j + 1, c1, w1);
                            qb = c1 - c0;
                            dd = w0 + w1;
                        }
                    } else {
                        R.rin[2 * j] = R.rin[2 * j + 1] = 0.0;
                        R.set_it(2 * j, 1.0);
                        R.set_it(2 * j + 1, 1.0);
                    }
                    if (k <= N && LR.var(j) < NZ) {
                        if constexpr (!RES_SPLIT) S.bx[k][LR.var(j)] = rb;
                        if constexpr (FUSE_BAR) {
                            if constexpr (!RES_SPLIT) S.q[k][LR.var(j)] = qb;  // dead since the last vector pass
                            S.dH[k][LR.var(j)] = dd;
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < HS; ++r) {
                    if (!LR.h_on(r)) {
                        R.rin[HB + r] = 0.0;
                        R.set_it(HB + r, 1.0);
                        continue;
                    }
                    const int hh = LR.hrow(r);
                    double a, bq, c;
                    rowg(hh, a, bq, c);
                    const double l = R.l[HB + r];
                    rh[0] += a * l; rh[1] += bq * l; rh[2] += c * l;
                    double dd = a * dzk[X0] + bq * dzk[X1] + c * dzk[X2];
                    if constexpr (NB == 4) {
                        const double sc = C::slack_coef(hh);
                        rh[3] += sc * l;
                        dd += sc * dzk[ZS];
                    }
                    row_res(HB + r, dd, rowgap(hh));
                    if constexpr (FUSE_BAR) {
                        double coef, wgt;
                        bar0(HB + r, coef, wgt);
                        double dg[NB];
                        dg[0] = a; dg[1] = bq; dg[2] = c;
                        if constexpr (NB == 4) dg[3] = C::slack_coef(hh);
#pragma unroll
                        for (int i = 0; i < NB; ++i) qh[i] += dg[i] * coef;
#pragma unroll
                        for (int cc = 0; cc < NB; ++cc)
#pragma unroll
                            for (int aa = cc; aa < NB; ++aa) dbh[cpk(NB, aa, cc)] += dg[aa] * wgt * dg[cc];
                    }
                }
                double acc[NB], aq[NB], ab[NBT];
#pragma unroll
                for (int i = 0; i < NB; ++i) { acc[i] = rh[i]; aq[i] = qh[i]; }
#pragma unroll
                for (int i = 0; i < NBT; ++i) ab[i] = dbh[i];
#pragma unroll
                for (int p = 1; p < PARTS; ++p) {
#pragma unroll
                    for (int i = 0; i < NB; ++i) acc[i] += lane_down(rh[i], p);
                    if constexpr (FUSE_BAR) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) aq[i] += lane_down(qh[i], p);
#pragma unroll
                        for (int i = 0; i < NBT; ++i) ab[i] += lane_down(dbh[i], p);
                    }
                }
                if constexpr (RES_SPLIT) {
                    // part 0's stage sums of the h rows to the owners of the block variables
                    if (stage_lane) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) { S.bx[k][i] = acc[i]; S.bx[k][NB + i] = aq[i]; }
#pragma unroll
                        for (int i = 0; i < NBT; ++i) S.dH[k][NZ + i] = ab[i];
                    }
                    wave_sync();
                    if (k <= N) {
                        double pq[NX];
#pragma unroll
                        for (int m = 0; m < NX; ++m) pq[m] = k < N ? S.piq[k][m] : 0.0;
#pragma unroll
                        for (int j = 0; j < BVS; ++j) {
                            const int v = LR.var(j);
                            if (v >= NZ) continue;
                            double a = 0.0;
#pragma unroll
                            for (int jj = 0; jj < NZ; ++jj) a += Hat(k, v, jj) * dzk[jj];
                            Hdz[j] = a;
                            const int bi = C::blk(v);
                            double rbox = rbj[j];
                            if (bi >= 0) rbox += S.bx[k][bi];
                            double rr = a + S.g[k][v] + rbox;
                            {
                                // the predictor's Newton gradient (barrier pass)
                                double qv = a + S.g[k][v] + qbj[j];
                                if (bi >= 0) qv += S.bx[k][NB + bi];
                                S.q[k][v] = qv;
                            }
                            if (k < N) {
#pragma unroll
                                for (int m = 0; m < NX; ++m) rr += Fat(k, m, v) * pq[m];
                            }
                            if (k > 0 && v >= NU) rr -= S.piq[k - 1][v - NU];
                            const bool free_var = (k == N) ? (v >= NU) : ((k == 0) ? (v < NU) : true);
                            if (free_var) rs = fmax(rs, fabs(rr));
                        }
                        if (k < N) {
#pragma unroll
                            for (int jd = 0; jd < DRS; ++jd) {
                                const int i = part + PARTS * jd;
                                if (i >= NX) continue;
                                double a = S.b[k][i] - S.dz[k + 1][NU + i];
#pragma unroll
                                for (int jj = 0; jj < NZ; ++jj) a += Fat(k, i, jj) * dzk[jj];
                                if constexpr (!LEAN) S.rdyn[k][i] = a;
                                re = fmax(re, fabs(a));
                            }
                        }
                    }
                } else {
                wave_sync();  // the owner lanes' box sums S.bx
                if (stage_lane) {
                    double rbox[NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) rbox[i] = S.bx[k][i];
#pragma unroll
                    for (int i = 0; i < NB; ++i) rbox[C::bvar(i)] += acc[i];
                    double r[NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) {
                        double a = 0.0;
#pragma unroll
                        for (int j = 0; j < NZ; ++j) a += Hat(k, i, j) * dzk[j];
                        if constexpr (!RES_SPLIT) Hdz[i] = a;
                        r[i] = a + S.g[k][i] + rbox[i];
                    }
                    if constexpr (FUSE_BAR) {
                        // the predictor's Newton gradient and h-row barrier block (barrier pass)
#pragma unroll
                        for (int i = 0; i < NZ; ++i) S.q[k][i] = Hdz[RES_SPLIT ? 0 : i] + S.g[k][i] + S.q[k][i];
#pragma unroll
                        for (int i = 0; i < NB; ++i) S.q[k][C::bvar(i)] += aq[i];
#pragma unroll
                        for (int i = 0; i < NBT; ++i) S.dH[k][NZ + i] = ab[i];
                    }
                    if (k < N) {
#pragma unroll
                        for (int m = 0; m < NX; ++m) {
                            const double pm = S.piq[k][m];
#pragma unroll
                            for (int i = 0; i < NZ; ++i) r[i] += Fat(k, m, i) * pm;
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = S.b[k][i] - S.dz[k + 1][NU + i];
#pragma unroll
                            for (int j = 0; j < NZ; ++j) a += Fat(k, i, j) * dzk[j];
                            if constexpr (!LEAN) S.rdyn[k][i] = a;
                            re = fmax(re, fabs(a));
                        }
                    }
                    if (k > 0) {
#pragma unroll
                        for (int i = 0; i < NX; ++i) r[NU + i] -= S.piq[k - 1][i];
                    }
#pragma unroll
                    for (int i = 0; i < NZ; ++i) {
                        const bool free_var = (k == N) ? (i >= NU) : ((k == 0) ? (i < NU) : true);
                        if (free_var) rs = fmax(rs, fabs(r[i]));
                    }
                }
                }
            }
#ifdef MPCG_TRACE
            rs = wave_max(rs);
            re = wave_max(re);
            ri = wave_max(ri);
#else
            // the exit tests compare all three residuals with the same bounds: one reduction of
            // their lane maximum (fmax drops NaN exactly as the per-lane accumulation above does)
            rs = wave_max(fmax(fmax(rs, re), ri));
            re = ri = rs;
#endif
            comp = wave_sum(comp);
            const double mu = comp / C::M_TOTAL;
#ifdef MPCG_TRACE
            // diagnostic build only (scripts/trace_solve.py): the oracle's ORC_DEBUG line of solve
            // MPCG_TRACE (-1: every solve, prefixed with its index)
            if ((MPCG_TRACE < 0 || sol == MPCG_TRACE) && lane == 0)
                printf("[%d]  ipm it %d rs %.3e re %.3e ri %.3e mu %.3e\n", sol, qit, rs, re, ri, mu);
#endif
            if (!(rs < 1e30) || !(re < 1e30) || !(ri < 1e30) || !(mu < mu_max)) { qstat = AC_NAN; break; }
            if (rs < pr.qp_tol && re < pr.qp_tol && ri < pr.qp_tol && mu < pr.qp_tol) { qstat = AC_SUCCESS; break; }
            if (qit >= pr.qp_iter_max) { qstat = AC_MAXITER; break; }
            wave_sync();
            STAMP_END(2);

            double alpha = 1.0, sigma_mu = 0.0;
            for (int phase = 0; phase < 2; ++phase) {
                // ---- barrier terms + Newton gradient (FUSE_BAR: the predictor's came with the residuals)
                STAMP_BEGIN();
                if (!FUSE_BAR || phase == 1) {
                    double qh[NB], dbh[NBT];
#pragma unroll
                    for (int i = 0; i < NB; ++i) qh[i] = 0.0;
#pragma unroll
                    for (int i = 0; i < NBT; ++i) dbh[i] = 0.0;
                    // coef = l + (l rin - rc) / t, wgt = l / t of slot s
                    auto bar = [&](int s, double& coef, double& wgt) {
                        const double l = R.l[s], t = R.t[s], itt = R.it(s);
                        const double rc = (phase == 0) ? l * t : l * t + R.pr[s] - sigma_mu;
                        coef = l + (l * R.rin[s] - rc) * itt;
                        wgt = l * itt;
                    };
                    double qbj[BVS];
#pragma unroll
                    for (int j = 0; j < BVS; ++j) {
                        double qb = 0.0, dd = 0.0;
                        if (LR.box_on(j)) {
                            double c0, w0, c1, w1;
                            bar(2 * j, c0, w0);
                            bar(2 * j + 1, c1, w1);
                            qb = c1 - c0;
                            dd = w0 + w1;
                        }
                        qbj[j] = qb;
                        if (k <= N && LR.var(j) < NZ) {
                            if constexpr (!RES_SPLIT) S.bx[k][LR.var(j)] = qb;
                            if (phase == 0) S.dH[k][LR.var(j)] = dd;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < HS; ++r) {
                        if (!LR.h_on(r)) continue;
                        const int hh = LR.hrow(r);
                        double coef, wgt;
                        bar(HB + r, coef, wgt);
                        double dg[NB];
                        rowg(hh, dg[0], dg[1], dg[2]);
                        if constexpr (NB == 4) dg[3] = C::slack_coef(hh);
#pragma unroll
                        for (int i = 0; i < NB; ++i) qh[i] += dg[i] * coef;
                        if (phase == 0) {
#pragma unroll
                            for (int c = 0; c < NB; ++c)
#pragma unroll
                                for (int a = c; a < NB; ++a) dbh[cpk(NB, a, c)] += dg[a] * wgt * dg[c];
                        }
                    }
                    double aq[NB], ab[NBT];
#pragma unroll
                    for (int i = 0; i < NB; ++i) aq[i] = qh[i];
#pragma unroll
                    for (int i = 0; i < NBT; ++i) ab[i] = dbh[i];
#pragma unroll
                    for (int p = 1; p < PARTS; ++p) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) aq[i] += lane_down(qh[i], p);
                        if (phase == 0) {
#pragma unroll
                            for (int i = 0; i < NBT; ++i) ab[i] += lane_down(dbh[i], p);
                        }
                    }
                    if constexpr (RES_SPLIT) {
                        // part 0's h-row sums to the owners of the block variables, then every
                        // owner its variables' entries of the Newton gradient
                        if (stage_lane) {
#pragma unroll
                            for (int i = 0; i < NB; ++i) S.bx[k][i] = aq[i];
                        }
                        wave_sync();
                        if (k <= N) {
#pragma unroll
                            for (int j = 0; j < BVS; ++j) {
                                const int v = LR.var(j);
                                if (v >= NZ) continue;
                                const int bi = C::blk(v);
                                double qv = Hdz[j] + S.g[k][v] + qbj[j];
                                if (bi >= 0) qv += S.bx[k][bi];
                                S.q[k][v] = qv;
                            }
                        }
                    } else {
                    wave_sync();  // the owner lanes' box sums S.bx
                    if (stage_lane) {
#pragma unroll
                        for (int i = 0; i < NZ; ++i) S.q[k][i] = Hdz[RES_SPLIT ? 0 : i] + S.g[k][i] + S.bx[k][i];
#pragma unroll
                        for (int i = 0; i < NB; ++i) S.q[k][C::bvar(i)] += aq[i];
                        if (phase == 0) {
#pragma unroll
                            for (int i = 0; i < NBT; ++i) S.dH[k][NZ + i] = ab[i];
                        }
                    }
                    }
                    wave_sync();
                }
                STAMP_END(3);
                // ---- Riccati factorisation (predictor only; the corrector reuses it)
                STAMP_BEGIN();
                if (phase == 0) {
                    constexpr int NT = C::NTRI, NP = C::NPT, DZ = C::NDH - 1;
                    constexpr bool FAC_FLAT = C::FAC_FLAT;
                    // FAC_PAIR: two lanes per block entry (lanes 2e, 2e + 1 of entry e), each forming the
                    // cost-to-go product P F[:, ej] on half of the rows (0-2 / 3-4) and its part of
                    // F[:, ei]' (P F[:, ej]); a DPP add joins the halves.  18 fp64 FMAs per lane and step
                    // instead of 30 (the nz 7 unicycle: 28 entries, 56 lanes)
#ifndef MPCG_FAC_PAIR
#define MPCG_FAC_PAIR 0
#endif
                    constexpr bool PAIR_EL = MPCG_FAC_PAIR && FAC_FLAT && NU == 2 && NX == 5 && !C::COMPACT &&
                                             !C::FCONST && !GFH && 2 * NT <= 64;
                    constexpr int RH = PAIR_EL ? 3 : NX;  // cost-to-go rows per lane
                    const int el = PAIR_EL ? (lane >> 1) : lane;  // the lane's block entry
                    const int half = PAIR_EL ? (lane & 1) : 0;
                    // the lane's rows of P F (half 1: rows 3, 4 and a dummy row 4 with a zero weight)
                    auto prow = [&](int t) -> int { return PAIR_EL ? (half == 0 ? t : (t < 2 ? 3 + t : 4)) : t; };
                    auto prow_on = [&](int t) -> bool { return !PAIR_EL || half == 0 || t < 2; };
                    // element lane -> (ei, ej), ei >= ej, of the nz x nz block
                    int ei = 0;
                    while ((ei + 1) * (ei + 2) / 2 <= el && ei < NZ - 1) ++ei;
                    const int ej = el < NT ? el - ei * (ei + 1) / 2 : 0;
                    // barrier entries of (ei, ej); DZ is the always-zero slot
                    const int dhd = (ei == ej) ? ei : DZ;
                    int dhb = DZ;
                    {
                        const int a = C::blk(ei), c = C::blk(ej);
                        if (a >= 0 && c >= 0) dhb = NZ + (a >= c ? cpk(NB, a, c) : cpk(NB, c, a));
                    }
                    // P lanes: (pi_, pj_) of the nx x nx block
                    int pi_ = 0;
                    while ((pi_ + 1) * (pi_ + 2) / 2 <= lane && pi_ < NX - 1) ++pi_;
                    const int pj_ = lane < NP ? lane - pi_ * (pi_ + 1) / 2 : 0;
                    if (lane < NP) S.P[N][lane] = Hat(N, NU + pi_, NU + pj_) + dh_at<C>(S.dH[N], NU + pi_, NU + pj_);
                    // failed pivots accumulate in a register and are voted once after the
                    // recursion (a store under a branch inside the stage loop kept the
                    // scheduler from hoisting the next LDS reads over it).  The register-starved
                    // bicycle instance keeps the LDS flag: there the hoisted reads spill.
                    bool fbad = false;
                    if (!FAC_FLAT && lane == 0) S.flag = 0;
                    wave_sync();
                    // prefetch of stage N-1's block
                    const int le = el < NT ? el : 0;
                    double fi[NX], fj[NX], hv;
#pragma unroll
                    for (int m = 0; m < NX; ++m) fj[m] = Fat(N - 1, m, ej);
#pragma unroll
                    for (int t = 0; t < RH; ++t) fi[t] = prow_on(t) ? Fat(N - 1, prow(t), ei) : 0.0;
                    // rows of [B A] that vary over the stages: with the constant rows (FCONST) only x+ and
                    // y+; the others stay in fi / fj from the fill above (their per-stage re-evaluation
                    // on the lane's runtime column compiled to branches inside the recursion)
                    constexpr int NFV = C::FCONST ? C::NFR : NX;
                    // (the compact bicycle storage: its v+ and delta+ rows are the known constants)
                    auto varies = [](int m) { return !C::COMPACT || (m != 3 && m != 4); };
                    // packed Hessian entry of the element lane (the compact storage: slack row / column 0
                    // but the diagonal)
                    auto Hel = [&](int kq) -> double {
                        if constexpr (C::COMPACT) return Hat(kq, ei, ej);
                        else return Hb(kq)[le];
                    };
                    // GFH: stage kn's blocks come from the staging copy (written this step from the
                    // coalesced loads issued one step earlier)
                    auto HelS = [&]() -> double {
                        if constexpr (C::COMPACT) return HatB(S.Hst, ei, ej);
                        else return S.Hst[le];
                    };
                    // measured: C4 53.40 -> 52.82 ms with the staging copy, C3 21.01 -> 21.67 (its
                    // compact blocks are rebuilt entry by entry and the copy adds live state): C4 only
#ifdef MPCG_NO_STAGE
                    constexpr bool STG = false;  // A/B: the Riccati step reads the global blocks directly
#else
                    constexpr bool STG = GFH && !C::COMPACT;
#endif
                    constexpr int NFB = C::NFR * C::NFC;
                    static_assert(!GFH || (NFB <= 64 && C::NHP <= 64), "one staged entry per lane");
                    double gsf = 0.0, gsh = 0.0;  // the staged entries of the next block in flight
                    auto stage_load = [&](int kq) {
                        if constexpr (STG) {
                            gsf = lane < NFB ? gF[(size_t)kq * NFB + lane] : 0.0;
                            gsh = lane < C::NHP ? gH[(size_t)kq * C::NHP + lane] : 0.0;
                        }
                    };
                    if (N >= 2) stage_load(N - 2);
                    hv = Hel(N - 1) + S.dH[N - 1][dhd] + S.dH[N - 1][dhb];
#pragma unroll
                    for (int kk = N - 1; kk >= 0; --kk) {
                        double Pm[NP];
                        if constexpr (PAIR_EL) {
                            // the lane's rows of the cost-to-go (two distinct addresses per read)
#pragma unroll
                            for (int t = 0; t < RH; ++t)
#pragma unroll
                                for (int l = 0; l < NX; ++l) Pm[t * NX + l] = S.P[kk + 1][sym(prow(t), l)];
                        } else {
#pragma unroll
                            for (int e = 0; e < NP; ++e) Pm[e] = S.P[kk + 1][e];
                        }
                        // prefetch of the next (lower) stage's block; it lands while this one is
                        // reduced.  FAC_FLAT: every lane runs one branch-free block, the five row
                        // products advance together, and the prefetch is issued after the pivot
                        // block's reads (off the recursion's critical path, and not in front of
                        // the LDS traffic the next step waits for)
                        const int kn = kk > 0 ? kk - 1 : 0;
                        if constexpr (STG) {
                            // stage kn's blocks into the staging copy, then the loads of kn - 1
                            if (lane < NFB) (&S.Fst[0][0])[lane] = gsf;
                            if (lane < C::NHP) S.Hst[lane] = gsh;
                            wave_sync();
                            if (kk >= 2) stage_load(kk - 2);
                        }
                        double fi2[NX], fj2[NX], hv2;
                        auto prefetch = [&]() {
                            if constexpr (STG) {
#pragma unroll
                                for (int m = 0; m < NFV; ++m)
                                    if (varies(m)) { fi2[m] = FatB(S.Fst, m, ei); fj2[m] = FatB(S.Fst, m, ej); }
                                hv2 = HelS() + S.dH[kn][dhd] + S.dH[kn][dhb];
                            } else if constexpr (PAIR_EL) {
#pragma unroll
                                for (int m = 0; m < NX; ++m) fj2[m] = Fat(kn, m, ej);
#pragma unroll
                                for (int t = 0; t < RH; ++t) fi2[t] = prow_on(t) ? Fat(kn, prow(t), ei) : 0.0;
                                hv2 = Hel(kn) + S.dH[kn][dhd] + S.dH[kn][dhb];
                            } else {
#pragma unroll
                                for (int m = 0; m < NFV; ++m)
                                    if (varies(m)) { fi2[m] = Fat(kn, m, ei); fj2[m] = Fat(kn, m, ej); }
                                hv2 = Hel(kn) + S.dH[kn][dhd] + S.dH[kn][dhb];
                            }
                        };
                        if constexpr (!FAC_FLAT) prefetch();
                        double v = hv;
                        if constexpr (PAIR_EL) {
                            // the lane's rows t of P F[:, ej], then its part of F[:, ei]' (P F[:, ej]) (half 1
                            // starts from 0), the halves joined on the even lane (DPP row_shl:1)
                            double tm[RH];
#pragma unroll
                            for (int t = 0; t < RH; ++t) tm[t] = 0.0;
#pragma unroll
                            for (int l = 0; l < NX; ++l)
#pragma unroll
                                for (int t = 0; t < RH; ++t) tm[t] += Pm[t * NX + l] * fj[l];
                            v = half == 0 ? hv : 0.0;
#pragma unroll
                            for (int t = 0; t < RH; ++t) v += fi[t] * tm[t];
                            v += dpp_d<0x101>(v);
                            S.Msc[(el < NT && half == 0) ? el : 64 + lane] = v;
                        } else if constexpr (FAC_FLAT) {
                            double tm[NX];
#pragma unroll
                            for (int m = 0; m < NX; ++m) tm[m] = 0.0;
#pragma unroll
                            for (int l = 0; l < NX; ++l)
#pragma unroll
                                for (int m = 0; m < NX; ++m) tm[m] += Pm[sym(m, l)] * fj[l];
#pragma unroll
                            for (int m = 0; m < NX; ++m) v += fi[m] * tm[m];
                            S.Msc[lane < NT ? lane : 64 + lane] = v;
                        } else {
#pragma unroll
                            for (int m = 0; m < NX; ++m) {
                                double tm = 0.0;
#pragma unroll
                                for (int l = 0; l < NX; ++l) tm += Pm[sym(m, l)] * fj[l];
                                v += fi[m] * tm;
                            }
                            if (lane < NT) S.Msc[lane] = v;
                        }
                        STAMP_LAP(16);
                        wave_sync();
                        STAMP_LAP(17);
                        if constexpr (NU == 2) {
                          if (FAC_FLAT || lane < NP) {
                            // the pivot block (element lanes 0, 1, 2) straight from their registers:
                            // the recursion's critical path skips one LDS round trip
                            constexpr int LS_ = PAIR_EL ? 2 : 1;  // lane stride of the block entries
                            const double m00 = FAC_FLAT ? readlane_d(v, 0) : S.Msc[0];
                            const double m10 = FAC_FLAT ? readlane_d(v, LS_) : S.Msc[1];
                            const double m11 = FAC_FLAT ? readlane_d(v, 2 * LS_) : S.Msc[2];
                            const double mi0 = S.Msc[sym(NU + pi_, 0)], mi1 = S.Msc[sym(NU + pi_, 1)];
                            const double mj0 = S.Msc[sym(NU + pj_, 0)], mj1 = S.Msc[sym(NU + pj_, 1)];
                            const double mij = S.Msc[sym(NU + pi_, NU + pj_)];
                            if constexpr (FAC_FLAT) {
                                __builtin_amdgcn_sched_barrier(0);
                                prefetch();
                                __builtin_amdgcn_sched_barrier(0);
                            }
                            // 2x2 Cholesky through reciprocal square roots
                            // 1/l11 = sqrt(m00 / det) = l00 / sqrt(det): both reciprocal square
                            // roots start from the block entries and run side by side
                            const double il00 = frsq(m00);
                            const double det = fma(m00, m11, -(m10 * m10));
                            const double ild = frsq(det);
                            const double l00 = m00 * il00;
                            const double l10 = m10 * il00;
                            const double il11 = l00 * ild;
                            fbad = fbad | !(m00 > 0.0) | !(det > 0.0);
                            const double y0i = mi0 * il00;
                            const double y1i = (mi1 - l10 * y0i) * il11;
                            const double y0j = mj0 * il00;
                            const double y1j = (mj1 - l10 * y0j) * il11;
                            *(lane < NP ? &S.P[kk][lane] : &S.Msc[64 + lane]) = mij - y0i * y0j - y1i * y1j;
                            if (pj_ == 0 && lane < NP) { S.Y[kk][0][pi_] = y0i; S.Y[kk][1][pi_] = y1i; }
                            if (lane == 0) { S.Lc[kk][0] = l00; S.Lc[kk][1] = l10; S.Lc[kk][2] = il00; S.Lc[kk][3] = il11; }
                          }
                        } else if (FAC_FLAT || lane < NP) {
                            // Cholesky of Muu through reciprocal square roots
                            double Lm[NU][NU], il[NU];
                            bool bad = false;
                            double Mu[C::NTRI > 0 ? NU * (NU + 1) / 2 : 1], Mi[NU], Mj[NU], mij = 0.0;
                            if constexpr (FAC_FLAT) {
#pragma unroll
                                for (int e = 0; e < NU * (NU + 1) / 2; ++e) Mu[e] = S.Msc[e];
#pragma unroll
                                for (int u = 0; u < NU; ++u) { Mi[u] = S.Msc[sym(NU + pi_, u)]; Mj[u] = S.Msc[sym(NU + pj_, u)]; }
                                mij = S.Msc[sym(NU + pi_, NU + pj_)];
                                __builtin_amdgcn_sched_barrier(0);
                                prefetch();
                                __builtin_amdgcn_sched_barrier(0);
                            }
                            auto msc = [&](int i, int j) -> double {  // entry of the pivot block
                                if constexpr (FAC_FLAT) return Mu[sym(i, j)];
                                else return S.Msc[sym(i, j)];
                            };
#pragma unroll
                            for (int j = 0; j < NU; ++j) {
                                double d = msc(j, j);
#pragma unroll
                                for (int m = 0; m < j; ++m) d -= Lm[j][m] * Lm[j][m];
                                il[j] = frsq(d);
                                Lm[j][j] = d * il[j];
                                bad = bad || !(d > 0.0);
#pragma unroll
                                for (int i = j + 1; i < NU; ++i) {
                                    double acc = msc(i, j);
#pragma unroll
                                    for (int m = 0; m < j; ++m) acc -= Lm[i][m] * Lm[j][m];
                                    Lm[i][j] = acc * il[j];
                                }
                            }
                            if constexpr (FAC_FLAT) {
                                fbad = fbad | bad;
                            } else {
                                if (bad) S.flag = 1;
                            }
                            double yi[NU], yj[NU];
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                double ai = FAC_FLAT ? Mi[u] : S.Msc[sym(NU + pi_, u)];
                                double aj = FAC_FLAT ? Mj[u] : S.Msc[sym(NU + pj_, u)];
#pragma unroll
                                for (int m = 0; m < u; ++m) { ai -= Lm[u][m] * yi[m]; aj -= Lm[u][m] * yj[m]; }
                                yi[u] = ai * il[u];
                                yj[u] = aj * il[u];
                            }
                            double pv = FAC_FLAT ? mij : S.Msc[sym(NU + pi_, NU + pj_)];
#pragma unroll
                            for (int u = 0; u < NU; ++u) pv -= yi[u] * yj[u];
                            *(lane < NP ? &S.P[kk][lane] : &S.Msc[64 + lane]) = pv;
                            if (pj_ == 0 && lane < NP) {
#pragma unroll
                                for (int u = 0; u < NU; ++u) S.Y[kk][u][pi_] = yi[u];
                            }
                            if (lane == 0) {
#pragma unroll
                                for (int i = 1; i < NU; ++i)
#pragma unroll
                                    for (int j = 0; j < i; ++j) S.Lc[kk][C::lo_idx(i, j)] = Lm[i][j];
#pragma unroll
                                for (int u = 0; u < NU; ++u) S.Lc[kk][C::NLO + u] = il[u];
                            }
                        }
#pragma unroll
                        for (int m = 0; m < NFV; ++m)
                            if (varies(m)) { fi[m] = fi2[m]; fj[m] = fj2[m]; }
                        hv = hv2;
                        STAMP_LAP(18);
                        wave_sync();
                        STAMP_LAP(19);
                    }
                    if (FAC_FLAT ? __any(fbad) : S.flag != 0) {
#ifdef MPCG_TRACE
                        if ((MPCG_TRACE < 0 || sol == MPCG_TRACE) && lane == 0) printf("[%d]  pivot failed\n", sol);
#endif
                        qstat = AC_NAN;
                        break;
                    }
                }
                STAMP_END(4);
                // ---- vector + forward passes: affine 5-vector recursions in SGPRs
                STAMP_BEGIN();
                if constexpr (C::CHAIN_SPLIT) {
                    // Every part of stage k owns the rows {part + PARTS s} of the stage's
                    // backward map p_k = h_k + G_k p_{k+1} and the same columns of the forward
                    // map dx_{k+1} = G_k' dx_k + e_k: a chain step is RS short dot products per
                    // lane instead of one whole 5x5 product, and the owning parts' rows meet
                    // in SGPRs through v_readlane.  Same operation order per row as the
                    // single-owner chain (bit-identical).
                    constexpr int RS = (NX + PARTS - 1) / PARTS;
                    const int kv = k < N ? k : 0;
                    const bool own = stage_lane && k < N;
                    double Lo[C::NLO > 0 ? C::NLO : 1], il[NU];
                    if constexpr (NU == 2) {
                        Lo[0] = S.Lc[kv][1]; il[0] = S.Lc[kv][2]; il[1] = S.Lc[kv][3];
                    } else {
#pragma unroll
                        for (int i = 0; i < C::NLO; ++i) Lo[i] = S.Lc[kv][i];
#pragma unroll
                        for (int u = 0; u < NU; ++u) il[u] = S.Lc[kv][C::NLO + u];
                    }
                    // dynamics residual of stage kv (LEAN recomputes it)
                    auto rdyn_v = [&](int i) -> double {
                        if constexpr (LEAN) return rdyn_at(kv, i);
                        else return S.rdyn[kv][i];
                    };
                    int rs[RS];
                    bool rv[RS];
#pragma unroll
                    for (int t = 0; t < RS; ++t) {
                        rv[t] = part + PARTS * t < NX;
                        rs[t] = rv[t] ? part + PARTS * t : NX - 1;
                    }
                    double Wu[NU][NX], y0[NU], c[NX];
                    {
                        double rr[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) rr[i] = rdyn_v(i);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = 0.0;
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += S.P[kv + 1][sym(i, j)] * rr[j];
                            c[i] = a;
                        }
                        double m0u[NU];
#pragma unroll
                        for (int i = 0; i < NU; ++i) {
                            double a = S.q[kv][i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += Fat(kv, j, i) * c[j];
                            m0u[i] = a;
                        }
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            double acc = m0u[u];
#pragma unroll
                            for (int m = 0; m < u; ++m) acc -= Lo[C::lo_idx(u, m)] * y0[m];
                            y0[u] = acc * il[u];
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i)
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                double w = Fat(kv, i, u);
#pragma unroll
                                for (int m = 0; m < u; ++m) w -= Lo[C::lo_idx(u, m)] * Wu[m][i];
                                Wu[u][i] = w * il[u];
                            }
                    }
                    // my rows of the backward map (h_r, G[r][.]) and columns of the forward one
                    double hr[RS], Gr[RS][NX], Gc[RS][NX];
#pragma unroll
                    for (int t = 0; t < RS; ++t) {
                        const int r = rs[t];
                        double a = S.q[kv][NU + r];
#pragma unroll
                        for (int j = 0; j < NX; ++j) a += Fat(kv, j, NU + r) * c[j];
#pragma unroll
                        for (int u = 0; u < NU; ++u) a -= S.Y[kv][u][r] * y0[u];
                        hr[t] = a;
                        double Yr[NU], Wr[NU];
#pragma unroll
                        for (int u = 0; u < NU; ++u) Yr[u] = S.Y[kv][u][r];
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            double w = Fat(kv, r, u);
#pragma unroll
                            for (int m = 0; m < u; ++m) w -= Lo[C::lo_idx(u, m)] * Wr[m];
                            Wr[u] = w * il[u];
                        }
#pragma unroll
                        for (int j = 0; j < NX; ++j) {
                            double acc = Fat(kv, j, NU + r);
#pragma unroll
                            for (int u = 0; u < NU; ++u) acc -= Yr[u] * Wu[u][j];
                            Gr[t][j] = acc;
                            double acc2 = Fat(kv, r, NU + j);
#pragma unroll
                            for (int u = 0; u < NU; ++u) acc2 -= S.Y[kv][u][j] * Wr[u];
                            Gc[t][j] = acc2;
                        }
                    }
                    STAMP_LAP(6);
                    double* const pch = &S.bx[0][0];
                    static_assert((N + 1) * NZ >= N * NX, "chain storage");
                    // Two-stage composed maps (PAIR): p_k = (h_k + G_k h_{k+1}) + G_k G_{k+1} p_{k+2}
                    // on the stages k = N-2, N-4, ... (the chain), then p_k = h_k + G_k p_{k+1} on the
                    // others, all at once; the forward map likewise (dx_{o+1} = Phi_o Phi_{o-1} dx_{o-1}
                    // + Phi_o e_{o-1} + e_o on odd o, then the even stages).  Half the sequential
                    // steps; each composition needs the partner stage's whole map, exchanged
                    // through the barrier-term rows and the pivot scratch, both dead from the
                    // Riccati step to the next barrier pass (which rewrites every barrier entry
                    // but the always-zero slot, restored after the forward pass).
                    constexpr bool PAIR = C::PAIR_CHAINS;
                    constexpr int NSLOT = (N + 1) / 2;  // slots k >> 1 of the publishing stages k <= N - 1
                    double* const XG = &S.dH[0][0];
                    double* const Xh = &S.Msc[0];
                    static_assert(!PAIR || (NSLOT * NX * NX <= (N + 1) * C::NDH && NSLOT * NX <= 128),
                                  "pair exchange storage");
                    // the stage's rows of (M, v) to its exchange slot / composed with the partner's slot
                    auto publish = [&](int sl, const double (&M)[RS][NX], const double (&v)[RS]) {
#pragma unroll
                        for (int t = 0; t < RS; ++t) {
                            if (!rv[t]) continue;
#pragma unroll
                            for (int j = 0; j < NX; ++j) XG[(sl * NX + rs[t]) * NX + j] = M[t][j];
                            Xh[sl * NX + rs[t]] = v[t];
                        }
                    };
                    auto compose = [&](int sl, double (&M)[RS][NX], double (&v)[RS]) {
                        double M2[RS][NX], v2[RS];
#pragma unroll
                        for (int t = 0; t < RS; ++t) {
                            v2[t] = v[t];
#pragma unroll
                            for (int j = 0; j < NX; ++j) M2[t][j] = 0.0;
                        }
#pragma unroll
                        for (int m = 0; m < NX; ++m) {
                            const double hm = Xh[sl * NX + m];
                            double xr[NX];
#pragma unroll
                            for (int j = 0; j < NX; ++j) xr[j] = XG[(sl * NX + m) * NX + j];
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                v2[t] += M[t][m] * hm;
#pragma unroll
                                for (int j = 0; j < NX; ++j) M2[t][j] += M[t][m] * xr[j];
                            }
                        }
#pragma unroll
                        for (int t = 0; t < RS; ++t) {
                            v[t] = v2[t];
#pragma unroll
                            for (int j = 0; j < NX; ++j) M[t][j] = M2[t][j];
                        }
                    };
                    // backward: the stages k = N-1, N-3, ... publish, k = N-2, N-4, ... compose
                    const bool bfix = k >= 1 && k <= N - 1 && ((N - 1 - k) & 1) == 0;
                    if constexpr (PAIR) {
                        if (bfix) publish(k >> 1, Gr, hr);
                        wave_sync();
                        if (k >= 1 && k <= N - 2 && ((N - k) & 1) == 0) compose((k + 1) >> 1, Gr, hr);
                    }
                    double pu[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) pu[i] = S.q[N][NU + i];
                    #pragma unroll
                    for (int kk = PAIR ? N - 2 : N - 1; kk >= 1; kk -= PAIR ? 2 : 1) {  // p_0 is not needed
                        double pn[RS];
#pragma unroll
                        for (int t = 0; t < RS; ++t) {
                            pn[t] = chain_dot<NX>(hr[t], Gr[t], pu);
                        }
                        if constexpr (C::REC_FLAT) {
                            // branch-free record: lanes that do not own the step write to the
                            // dead pivot scratch (the stores then sink below the broadcast)
#ifndef MPCG_REC_SELECT
                            // owner lanes of step kk: the literal mask of stage kk's parts; both
                            // candidate addresses are lane constants offset by the step's stride
                            const unsigned long long OWN = ((1ull << PARTS) - 1) << (kk * PARTS);
                            // dummies in the QP step rows (dead until the forward chain writes them)
                            static_assert((N - 1) * NX + 8 <= (N + 1) * NZ, "record dummies inside the QP step rows");
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                const unsigned off = lds_addr(&S.ddz[0][lane & 7]);
                                const unsigned on = rv[t] ? lds_addr(&pch[rs[t]]) : off;
                                lds_store(sel_lanes(OWN, off, on) + kk * NX * 8, pn[t]);
                            }
#else
#pragma unroll
                            for (int t = 0; t < RS; ++t)
                                *((k == kk && rv[t]) ? &pch[kk * NX + rs[t]] : &S.Msc[64 * (t & 1) + lane]) = pn[t];
#endif
                        } else if (k == kk) {
#pragma unroll
                            for (int t = 0; t < RS; ++t)
                                if (rv[t]) pch[kk * NX + rs[t]] = pn[t];
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) pu[i] = readlane_d(pn[i / PARTS], kk * PARTS + i % PARTS);
                    }
                    wave_sync();
                    if constexpr (PAIR) {
                        // the stages between the chain's: one map applied to the recorded p_{k+1}
                        if (bfix) {
                            const double* src = (k + 1 < N) ? pch + (k + 1) * NX : &S.q[N][NU];
                            double pnx[NX];
#pragma unroll
                            for (int i = 0; i < NX; ++i) pnx[i] = src[i];
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                double a = hr[t];
#pragma unroll
                                for (int j = 0; j < NX; ++j) a += Gr[t][j] * pnx[j];
                                if (rv[t]) pch[k * NX + rs[t]] = a;
                            }
                        }
                        wave_sync();
                    }
                    double pmine[NX];
                    {
                        const double* src = (kv + 1 < N) ? pch + (kv + 1) * NX : &S.q[N][NU];
#pragma unroll
                        for (int i = 0; i < NX; ++i) pmine[i] = src[i];
                    }
                    STAMP_LAP(15);
                    // feedback of stage k: du = K dx + kff; closed loop dx+ = G' dx + e
                    double kf[NU];
                    {
                        double yy[NU];
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            double acc = y0[u];
#pragma unroll
                            for (int i = 0; i < NX; ++i) acc += Wu[u][i] * pmine[i];
                            yy[u] = acc;
                        }
#pragma unroll
                        for (int u = NU - 1; u >= 0; --u) {
                            double acc = -yy[u];
#pragma unroll
                            for (int m = u + 1; m < NU; ++m) acc -= Lo[C::lo_idx(m, u)] * kf[m];
                            kf[u] = acc * il[u];
                        }
                    }
                    double ec[RS];
#pragma unroll
                    for (int t = 0; t < RS; ++t) {
                        double acc = rdyn_v(rs[t]);
#pragma unroll
                        for (int u = 0; u < NU; ++u) acc += Fat(kv, rs[t], u) * kf[u];
                        ec[t] = acc;
                    }
                    // forward: the even stages publish (Phi_k, e_k), the odd stages compose
                    const bool ffix = k <= N - 1 && (k & 1) == 0;
                    if constexpr (PAIR) {
                        if (ffix) publish(k >> 1, Gc, ec);
                        wave_sync();
                        if (k >= 1 && k <= N - 1 && (k & 1)) compose(k >> 1, Gc, ec);
                    }
                    // dx_{kk+1} goes straight to its place in the QP step, ddz[kk + 1]
                    double dxu[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) dxu[i] = 0.0;
                    #pragma unroll
                    for (int kk = PAIR ? 1 : 0; kk < N; kk += PAIR ? 2 : 1) {
                        double dn[RS];
#pragma unroll
                        for (int t = 0; t < RS; ++t) {
                            dn[t] = chain_dot<NX>(ec[t], Gc[t], dxu);
                        }
                        if constexpr (C::REC_FLAT) {
#ifndef MPCG_REC_SELECT
                            // dummies in the box-sum rows (the backward chain's values are read)
                            const unsigned long long OWN = ((1ull << PARTS) - 1) << (kk * PARTS);
                            static_assert((N - 1) * NZ + 8 <= (N + 1) * NZ, "record dummies inside the box-sum rows");
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                const unsigned off = lds_addr(&S.bx[0][lane & 7]);
                                const unsigned on = rv[t] ? lds_addr(&S.ddz[1][NU + rs[t]]) : off;
                                lds_store(sel_lanes(OWN, off, on) + kk * NZ * 8, dn[t]);
                            }
#else
#pragma unroll
                            for (int t = 0; t < RS; ++t)
                                *((k == kk && rv[t]) ? &S.ddz[kk + 1][NU + rs[t]] : &S.Msc[64 * (t & 1) + lane]) = dn[t];
#endif
                        } else if (k == kk) {
#pragma unroll
                            for (int t = 0; t < RS; ++t)
                                if (rv[t]) S.ddz[kk + 1][NU + rs[t]] = dn[t];
                        }
                        if (kk + (PAIR ? 2 : 1) < N) {
#pragma unroll
                            for (int i = 0; i < NX; ++i) dxu[i] = readlane_d(dn[i / PARTS], kk * PARTS + i % PARTS);
                        }
                    }
                    wave_sync();
                    if constexpr (PAIR) {
                        // the even stages: one map applied to the recorded dx_k
                        if (ffix) {
                            double dxs[NX];
#pragma unroll
                            for (int i = 0; i < NX; ++i) dxs[i] = k >= 1 ? S.ddz[k][NU + i] : 0.0;
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                double a = ec[t];
#pragma unroll
                                for (int j = 0; j < NX; ++j) a += Gc[t][j] * dxs[j];
                                if (rv[t]) S.ddz[k + 1][NU + rs[t]] = a;
                            }
                        }
                        // the barrier rows' always-zero slot, overwritten by the exchange (the
                        // rest of the rows is rewritten by the next predictor's barrier pass)
                        for (int e = lane; e <= N; e += 64) S.dH[e][C::NDH - 1] = 0.0;
                        wave_sync();
                    }
                    STAMP_LAP(9);
                    if (own) {
                        double dxm[NX], dxn[NX], du[NU];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            dxm[i] = k >= 1 ? S.ddz[k][NU + i] : 0.0;
                            dxn[i] = S.ddz[k + 1][NU + i];
                        }
#pragma unroll
                        for (int u = 0; u < NU; ++u) du[u] = kf[u];
#pragma unroll
                        for (int j = 0; j < NX; ++j) {
                            double K[NU];
#pragma unroll
                            for (int u = NU - 1; u >= 0; --u) {
                                double acc = -S.Y[k][u][j];
#pragma unroll
                                for (int m = u + 1; m < NU; ++m) acc -= Lo[C::lo_idx(m, u)] * K[m];
                                K[u] = acc * il[u];
                            }
#pragma unroll
                            for (int u = 0; u < NU; ++u) du[u] += K[u] * dxm[j];
                        }
#pragma unroll
                        for (int u = 0; u < NU; ++u) S.ddz[k][u] = du[u];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            if (k == 0) S.ddz[0][NU + i] = 0.0;
                            if constexpr (PIN_SPLIT) continue;
                            double a = pmine[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += S.P[k + 1][sym(i, j)] * dxn[j];
                            if constexpr (LEAN) pinr[i] = a;
                            else S.pin[k][i] = a;
                        }
                        if (k == N - 1) {
#pragma unroll
                            for (int u = 0; u < NU; ++u) S.ddz[N][u] = 0.0;
                        }
                    }
                    if constexpr (PIN_SPLIT) {
                        // the new dynamics multipliers, rows split over the parts like the chains' rows
                        if (k < N) {
                            double dxn[NX];
#pragma unroll
                            for (int i = 0; i < NX; ++i) dxn[i] = S.ddz[k + 1][NU + i];
#pragma unroll
                            for (int t = 0; t < RS; ++t) {
                                if (!rv[t]) continue;
                                const int i = rs[t];
                                double a = pmine[i];
#pragma unroll
                                for (int j = 0; j < NX; ++j) a += S.P[k + 1][sym(i, j)] * dxn[j];
                                S.pin[k][i] = a;
                            }
                        }
                    }
                } else
                {
                    const bool own = stage_lane && k < N;
                    const int kq = own ? k : 0;
                    double Lo[C::NLO > 0 ? C::NLO : 1], il[NU];
                    if constexpr (NU == 2) {
                        Lo[0] = S.Lc[kq][1]; il[0] = S.Lc[kq][2]; il[1] = S.Lc[kq][3];
                    } else {
#pragma unroll
                        for (int i = 0; i < C::NLO; ++i) Lo[i] = S.Lc[kq][i];
#pragma unroll
                        for (int u = 0; u < NU; ++u) il[u] = S.Lc[kq][C::NLO + u];
                    }
                    double G[NX][NX], hv[NX], Wu[NU][NX], y0[NU];
                    double rdv[LEAN ? NX : 1];  // LEAN: recomputed dynamics residual
                    {
                        double c[NX], rr[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            if constexpr (LEAN) rr[i] = rdv[i] = rdyn_at(kq, i);
                            else rr[i] = S.rdyn[kq][i];
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = 0.0;
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += S.P[kq + 1][sym(i, j)] * rr[j];
                            c[i] = a;
                        }
                        double m0[NZ];
#pragma unroll
                        for (int i = 0; i < NZ; ++i) {
                            double a = S.q[kq][i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += Fat(kq, j, i) * c[j];
                            m0[i] = a;
                        }
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            double acc = m0[u];
#pragma unroll
                            for (int m = 0; m < u; ++m) acc -= Lo[C::lo_idx(u, m)] * y0[m];
                            y0[u] = acc * il[u];
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = m0[NU + i];
#pragma unroll
                            for (int u = 0; u < NU; ++u) acc -= S.Y[kq][u][i] * y0[u];
                            hv[i] = acc;
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                double w = Fat(kq, i, u);
#pragma unroll
                                for (int m = 0; m < u; ++m) w -= Lo[C::lo_idx(u, m)] * Wu[m][i];
                                Wu[u][i] = w * il[u];
                            }
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double Yi[NU];
#pragma unroll
                            for (int u = 0; u < NU; ++u) Yi[u] = S.Y[kq][u][i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) {
                                double acc = Fat(kq, j, NU + i);
#pragma unroll
                                for (int u = 0; u < NU; ++u) acc -= Yi[u] * Wu[u][j];
                                G[i][j] = acc;
                            }
                        }
                    }
                    STAMP_LAP(6);
                    // each chain step's value is recorded in LDS by the lane that owns it (a
                    // predicated store off the VALU path) and read back after the chain.  The
                    // register-starved bicycle instance did the selects into registers until round 4;
                    // the records keep six doubles per chain out of its registers: scratch 560 -> 504
                    // B/lane, C3 19.50 -> 18.99 ms (profiles/r04i_ab_*; MPCG_C3_CHAIN_REC=0: A/B)
#ifndef MPCG_C3_CHAIN_REC
#define MPCG_C3_CHAIN_REC 1
#endif
                    constexpr bool CHAIN_REC = !C::COMPACT || MPCG_C3_CHAIN_REC;
                    double pu[NX], pmine[NX];
                    double* const pch = &S.bx[0][0];
                    static_assert((N + 1) * NZ >= N * NX, "chain storage");
#pragma unroll
                    for (int i = 0; i < NX; ++i) { pu[i] = S.q[N][NU + i]; pmine[i] = pu[i]; }
                    #pragma unroll
                    for (int kk = N - 1; kk >= 1; --kk) {  // p_0 is not needed
                        double pn[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = hv[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += G[i][j] * pu[j];
                            pn[i] = a;
                        }
                        if (CHAIN_REC && lane == kk * PARTS) {
#pragma unroll
                            for (int i = 0; i < NX; ++i) pch[kk * NX + i] = pn[i];
                        }
                        const bool mine = !CHAIN_REC && (k == kk - 1) && (part == 0);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            pu[i] = readlane_d(pn[i], kk * PARTS);
                            if constexpr (!CHAIN_REC) pmine[i] = mine ? pu[i] : pmine[i];
                        }
                    }
                    if constexpr (CHAIN_REC) {
                        wave_sync();
                        const double* src = (kq + 1 < N) ? pch + (kq + 1) * NX : &S.q[N][NU];
#pragma unroll
                        for (int i = 0; i < NX; ++i) pmine[i] = src[i];
                    }
                    STAMP_LAP(15);
                    // feedback of stage k: du = K dx + kff; closed loop dx+ = G' dx + e
                    double kf[NU];
                    {
                        double yy[NU];
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            double acc = y0[u];
#pragma unroll
                            for (int i = 0; i < NX; ++i) acc += Wu[u][i] * pmine[i];
                            yy[u] = acc;
                        }
#pragma unroll
                        for (int u = NU - 1; u >= 0; --u) {
                            double acc = -yy[u];
#pragma unroll
                            for (int m = u + 1; m < NU; ++m) acc -= Lo[C::lo_idx(m, u)] * kf[m];
                            kf[u] = acc * il[u];
                        }
                    }
                    double e[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        double acc;
                        if constexpr (LEAN) acc = rdv[i];
                        else acc = S.rdyn[kq][i];
#pragma unroll
                        for (int u = 0; u < NU; ++u) acc += Fat(kq, i, u) * kf[u];
                        e[i] = acc;
                    }
                    // dx_{kk+1} goes straight to its place in the QP step, ddz[kk + 1]
                    double dxu[NX], dxmine[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) { dxu[i] = 0.0; dxmine[i] = 0.0; }
                    #pragma unroll
                    for (int kk = 0; kk < N - 1; ++kk) {  // dx_N comes from stage N - 1's own lane
                        double dn[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = e[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += G[j][i] * dxu[j];
                            dn[i] = a;
                        }
                        if (CHAIN_REC && lane == kk * PARTS) {
#pragma unroll
                            for (int i = 0; i < NX; ++i) S.ddz[kk + 1][NU + i] = dn[i];
                        }
                        const bool mine = !CHAIN_REC && (k == kk + 1) && (part == 0);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            dxu[i] = readlane_d(dn[i], kk * PARTS);
                            if constexpr (!CHAIN_REC) dxmine[i] = mine ? dxu[i] : dxmine[i];
                        }
                    }
                    if constexpr (CHAIN_REC) {
                        wave_sync();
#pragma unroll
                        for (int i = 0; i < NX; ++i) dxmine[i] = (k >= 1 && k < N) ? S.ddz[k][NU + i] : 0.0;
                    }
                    STAMP_LAP(9);
                    if (own) {
                        double du[NU], dxn[NX];
#pragma unroll
                        for (int u = 0; u < NU; ++u) du[u] = kf[u];
#pragma unroll
                        for (int j = 0; j < NX; ++j) {
                            double K[NU];
#pragma unroll
                            for (int u = NU - 1; u >= 0; --u) {
                                double acc = -S.Y[k][u][j];
#pragma unroll
                                for (int m = u + 1; m < NU; ++m) acc -= Lo[C::lo_idx(m, u)] * K[m];
                                K[u] = acc * il[u];
                            }
#pragma unroll
                            for (int u = 0; u < NU; ++u) du[u] += K[u] * dxmine[j];
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double a = e[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += G[j][i] * dxmine[j];
                            dxn[i] = a;
                        }
#pragma unroll
                        for (int u = 0; u < NU; ++u) S.ddz[k][u] = du[u];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            if (!CHAIN_REC || k == 0) S.ddz[k][NU + i] = dxmine[i];  // 0 at k = 0
                            double a = pmine[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) a += S.P[k + 1][sym(i, j)] * dxn[j];
                            if constexpr (LEAN) pinr[i] = a;
                            else S.pin[k][i] = a;
                        }
                        if (k == N - 1) {
#pragma unroll
                            for (int u = 0; u < NU; ++u) S.ddz[N][u] = 0.0;
#pragma unroll
                            for (int i = 0; i < NX; ++i) S.ddz[N][NU + i] = dxn[i];
                        }
                    }
                }
                wave_sync();
                STAMP_END(5);
                // ---- inequality steps, step length, predictor statistics, row update
                STAMP_BEGIN();
                {
                    double ddk[NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) ddk[i] = S.ddz[ks][i];
                    const double smu = sigma_mu;
                    const int ph = phase;
                    // per-row D . ddz of the lane's rows
                    double ddb[BVS];
#pragma unroll
                    for (int j = 0; j < BVS; ++j) ddb[j] = LR.box_on(j) ? S.ddz[k][LR.var(j)] : 0.0;
                    // h rows: D . ddz once per phase (the passes below reuse it)
                    double ddh[HS];
#pragma unroll
                    for (int r = 0; r < HS; ++r) {
                        double v = 0.0;
                        if (LR.h_on(r)) {
                            const int hh = LR.hrow(r);
                            double ga, gb, gc;
                            rowg(hh, ga, gb, gc);
                            v = ga * ddk[X0] + gb * ddk[X1] + gc * ddk[X2];
                            if constexpr (NB == 4) v += C::slack_coef(hh) * ddk[ZS];
                        }
                        ddh[r] = v;
                    }
                    auto ddot = [&](int s) {
                        if (s < HB) return (s & 1) ? ddb[s >> 1] : -ddb[s >> 1];
                        return ddh[s - HB];
                    };
                    auto active = [&](int s) { return s < HB ? LR.box_on(s >> 1) : LR.h_on(s - HB); };
                    // dt = -rin - D ddz; dl = -(rc + l dt) / t
                    auto row_step = [&](int s, double& dt, double& dl) {
                        const double l = R.l[s], t = R.t[s];
                        const double rc = (ph == 0) ? l * t : l * t + R.pr[s] - smu;
                        dt = -R.rin[s] - ddot(s);
                        dl = -(rc + l * dt) * R.it(s);
                    };
                    // step to the boundary: min over rows of -t/dt and -l/dl = 1 / max(-dt/t, -dl/l)
                    // STEP_FORMS: in the predictor rc = l t, so dl = -l (t + dt) / t and a row's
                    // multiplier blocks (dl < 0) exactly when t + dt > 0, at -dl / l = 1 + dt / t: the row's
                    // bound is max(-dt/t, 1 + dt/t) (the second term is <= 0 < the first when it does not
                    // block), no reciprocal of l and no branch; in the corrector the branch on dl < 0 is a
                    // select (the wave computes the reciprocal whenever any lane needs it)
#ifndef MPCG_STEP_FORMS
#define MPCG_STEP_FORMS 1
#endif
                    double rmax = 0.0;
                    if (MPCG_STEP_FORMS && ph == 0) {
#pragma unroll
                        for (int s = 0; s < C::SLOTS; ++s) {
                            if (!active(s)) continue;
                            double dt, dl;
                            row_step(s, dt, dl);
                            const double x = dt * R.it(s);
                            rmax = fmax(rmax, fmax(-x, 1.0 + x));
                        }
                    } else {
#pragma unroll
                        for (int s = 0; s < C::SLOTS; ++s) {
                            if (!active(s)) continue;
                            double dt, dl;
                            row_step(s, dt, dl);
                            rmax = fmax(rmax, -dt * R.it(s));
                            if (MPCG_STEP_FORMS) {
                                const double c = -dl * frcp(R.l[s]);
                                rmax = fmax(rmax, dl < 0.0 ? c : 0.0);
                            } else if (dl < 0.0) {
                                rmax = fmax(rmax, -dl * frcp(R.l[s]));
                            }
                        }
                    }
                    rmax = wave_max(rmax);
                    const double amax = rmax > 0.0 ? frcp(rmax) : 1e300;
                    if (phase == 0) {
                        const double aa = fmin(amax, 1.0);
                        double ca = 0.0;
#pragma unroll
                        for (int s = 0; s < C::SLOTS; ++s) {
                            if (!active(s)) continue;
                            double dt, dl;
                            row_step(s, dt, dl);
                            ca += (R.l[s] + aa * dl) * (R.t[s] + aa * dt);
                            R.pr[s] = dt * dl;
                        }
                        ca = wave_sum(ca);
                        const double mu_aff = ca / C::M_TOTAL;
                        double sig = mu_aff / mu;
                        if (sig > 1.0) sig = 1.0;
                        sig = sig * sig * sig;
                        sigma_mu = sig * mu;
                    } else {
                        alpha = 0.995 * amax;
                        if (alpha > 1.0) alpha = 1.0;
                        if (alpha >= 1e-12) {
                            // rows move with the corrector step (rin, ddz of the current iterate), then
                            // t and lambda are floored at qp_t_min (a compare-select: NaN passes through)
#pragma unroll
                            for (int s = 0; s < C::SLOTS; ++s) {
                                if (!active(s)) continue;
                                double dt, dl;
                                row_step(s, dt, dl);
                                const double tn = R.t[s] + alpha * dt, ln = R.l[s] + alpha * dl;
                                R.t[s] = tn < tmin ? tmin : tn;
                                R.l[s] = ln < tmin ? tmin : ln;
                            }
                        }
                    }
                }
                wave_sync();
                STAMP_END(7);
            }
            if (qstat == AC_NAN) break;
            if (alpha < 1e-12) { qstat = AC_MINSTEP; ++qit; break; }
            // ---- update of the stage variables (rows were updated with the step)
            STAMP_BEGIN();
            if (RES_SPLIT && !LEAN) {
                // every part its variables and dynamics rows (same operations)
                if (k <= N) {
#pragma unroll
                    for (int j = 0; j < BVS; ++j) {
                        const int v = LR.var(j);
                        if (v < NZ) S.dz[k][v] += alpha * S.ddz[k][v];
                    }
                    if (k < N) {
#pragma unroll
                        for (int jd = 0; jd < DRS; ++jd) {
                            const int i = part + PARTS * jd;
                            if (i < NX) S.piq[k][i] += alpha * (S.pin[k][i] - S.piq[k][i]);
                        }
                    }
                }
            } else if (stage_lane) {
#pragma unroll
                for (int i = 0; i < NZ; ++i) S.dz[k][i] += alpha * S.ddz[k][i];
                if (k < N) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        if constexpr (LEAN) S.piq[k][i] += alpha * (pinr[i] - S.piq[k][i]);
                        else S.piq[k][i] += alpha * (S.pin[k][i] - S.piq[k][i]);
                    }
                }
            }
            wave_sync();
            STAMP_END(8);
        }
        wave_sync();
        qp_status = qstat;
        qp_total += qit;
        ++sqp_iter;
        n_maxit += qstat == AC_MAXITER;
        if (qstat != AC_SUCCESS && qstat != AC_MAXITER) {
            acados_status = AC_QP_FAILURE;
            break;
        }
        // FIXED_STEP full step on the primal iterate and on every multiplier
        if (stage_lane) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) S.z[k][i] += S.dz[k][i];
            if (k == N) {
#pragma unroll
                for (int u = 0; u < NU; ++u) S.z[N][u] = 0.0;
            }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.pi_nlp[k][i] = S.piq[k][i];
            }
        }
#pragma unroll
        for (int r = 0; r < HS; ++r)
            if (LR.h_on(r)) R.nlam[r] = R.l[HB + r];
        wave_sync();
        acados_status = AC_SUCCESS;
        // SQP-RTI: the reference's loop stops after a QP that did not succeed
        // (acados_solver_interface.cpp:105); a full SQP call continues after a max-iter QP
        if (!sqp_mode && qstat != AC_SUCCESS) break;
    }

    // ---- completeOneIteration (acados_solver_interface.cpp:162-204)
    double Lk = 0.0;
    if (stage_lane && k < N) {
        double zz[NZ], gd[NZ], Hd[NZ][NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zz[i] = S.z[k][i];
        if constexpr (C::MODEL == 1) Lk = bike::stage_cost(pr, pk, k, zz, gd, Hd, false);
        else Lk = stage_cost<NX>(pr, pk, zz, gd, Hd, false);
    }
    const double pobj = wave_sum(Lk);
    double* xo = io.xtraj + (size_t)sol * (N + 1) * NX;
    for (int e = lane; e < (N + 1) * NX; e += 64) xo[e] = S.z[e / NX][NU + e % NX];
    double* uo = io.utraj + (size_t)sol * N * NU;
    for (int e = lane; e < N * NU; e += 64) uo[e] = S.z[e / NU][e % NU];
    if (io.lam_out) {
        double* lo = io.lam_out + (size_t)sol * N * LAMS;
        for (int e = lane; e < N * NX; e += 64) lo[(size_t)(e / NX) * LAMS + e % NX] = S.pi_nlp[e / NX][e % NX];
        if (k == 0) {
            for (int r = part; r < C::NH; r += PARTS) lo[NX + r] = 0.0;
        } else if (k < N) {
#pragma unroll
            for (int r = 0; r < HS; ++r)
                if (LR.h_on(r)) lo[(size_t)k * LAMS + NX + LR.hrow(r)] = R.nlam[r];
        }
    }
    if (FULL && io.qp_out) {
        double* q = io.qp_out + (size_t)sol * C::QPM;
#pragma unroll
        for (int sl = 0; sl < C::SLOTS; ++sl) {
            q[(2 * sl) * 64 + lane] = R.t[sl];
            q[(2 * sl + 1) * 64 + lane] = R.l[sl];
        }
        for (int e = lane; e < (N + 1) * NZ; e += 64) q[C::QPM_ROWS + e] = (&S.dz[0][0])[e];
        for (int e = lane; e < N * NX; e += 64) q[C::QPM_ROWS + (N + 1) * NZ + e] = (&S.piq[0][0])[e];
    }
    if (FULL && io.stats && lane == 0) {
        double* st = io.stats + (size_t)sol * MPCG_STATS_STRIDE;
        st[0] = nlp_stat;
        st[1] = res_eq;
        st[2] = nlp_ineq;
        st[3] = nlp_comp;
    }
    if (lane == 0) {
        int code = acados_status;
        if (res_eq > pr.res_eq_fail && code == AC_SUCCESS) code = AC_QP_FAILURE;
        if (code == AC_SUCCESS) code = 1;
        else if (code == 1) code = 0;
        io.exit_code[sol] = code;
        io.pobj[sol] = pobj;
        if (io.info) {
            io.info[(size_t)sol * MPCG_INFO_STRIDE + 0] = sqp_iter;
            io.info[(size_t)sol * MPCG_INFO_STRIDE + 1] = qp_total;
            io.info[(size_t)sol * MPCG_INFO_STRIDE + 2] = qp_status;
            io.info[(size_t)sol * MPCG_INFO_STRIDE + 3] = n_maxit;
        }
    }
    STAMP_STORE(stamps, sol);
}

// The batched solve.  queue == NULL or an instance without C::QUEUE: workgroup b solves problem b
// (a grid of `batch` workgroups).  Otherwise a grid of at most the resident workgroups (launch_instance: MPCG_QUEUE) takes the
// problems from the head of a work queue, queue[0], one at a time until it runs past `batch`:
// the hardware deals workgroups to the XCDs round robin and starts a new one only when a slot
// frees, so with a grid of one workgroup per solve each XCD works through a fixed eighth of the
// batch and every solve pays a workgroup launch; here a wave that finishes early takes the next
// solve of the whole batch (the tail).  Every wave leaves the loop on its first
// ticket >= batch; the last workgroup out (queue[1] counts them) zeroes both words for the next
// launch on the same workspace, which the stream orders after this one.
template <class C, bool FULL = false>
__global__ MPCG_KERNEL_ATTR void sqp_kernel(mpcg_problem pr, int batch, mpcg_io io,
                                                    unsigned long long* __restrict__ stamps,
                                                    double* __restrict__ gws, unsigned* __restrict__ queue) {
    if constexpr (!C::QUEUE) {
        (void)queue;
        sqp_solve<C, FULL>(pr, batch, io, stamps, gws, blockIdx.x);
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
            sqp_solve<C, FULL>(pr, batch, io, stamps, gws, sol);
            wave_sync();
        }
        if (q && threadIdx.x == 0 && atomicAdd(&queue[1], 1u) == gridDim.x - 1) {
            atomicExch(&queue[0], 0u);
            atomicExch(&queue[1], 0u);
        }
    }
}

}  // namespace mpcg
