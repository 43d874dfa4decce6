// mpcg_kernels.hip — MI355X (gfx950) kernels of the batched T-MPC++ SQP solve.
//
// One wavefront (64 lanes, one workgroup) solves one (scene, guess) pair:
// the body of one `Solver::solve()` call of the OpenMP fan-out in
// GuidanceConstraints::optimize (guidance_constraints.cpp:304-421), i.e.
// `sqp_iters` acados SQP-RTI iterations (acados_solver_interface.cpp:311-429).
//
// Lane roles inside the wave
//   * stage lanes   lane k in [0, N]: linearisation of shooting stage k (cost,
//                   ERK4 sensitivities + exact Hessian, constraints, MIRROR),
//                   and every per-inequality interior-point operation of stage k
//   * element lanes lane e < 49: one entry (i, j) of the 7x7 Riccati stage
//                   block during the backward factorisation
//   * all lanes     redundant scalar recursions (vector pass, forward pass),
//                   so no LDS round trip sits on those sequential chains
// All QP data of one solve lives in LDS (struct Lds below); stage-indexed
// arrays are stage-minor so stage lanes access consecutive 8-byte words.
// Reductions (max residual, complementarity sum, step length) are xor
// butterflies: bit-identical in every lane, deterministic.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "mpcg.h"
#include "mpcg_device.h"

namespace mpcg {

enum { AC_SUCCESS = 0, AC_NAN = 1, AC_MAXITER = 2, AC_MINSTEP = 3, AC_QP_FAILURE = 4 };

template <int N_, int NL_, int NE_>
struct Cfg {
    static constexpr int N = N_, NL = NL_, NE = NE_;
    static constexpr int NH = NL + NE;
    static constexpr int NR = 2 * NU + 2 * NX + NH;  // inequality rows of stages 1..N-1
    static constexpr int NR0 = 2 * NU;               // stage 0: input bounds only
    static constexpr int M_TOTAL = NR0 + (N - 1) * NR;
};

template <class C>
struct Lds {
    static constexpr int N = C::N, NH = C::NH, NR = C::NR;
    double z[N + 1][NZ];          // NLP iterate [u x] per stage
    double H[N + 1][NZ][NZ];      // MIRROR-regularised Hessian of the Lagrangian
    double g[N + 1][NZ];          // cost gradient
    double F[N][NX][NZ];          // [B A]
    double b[N][NX];              // shooting defect
    double dH[N + 1][13];         // barrier terms: diag(7) + (x,y,psi) block (6)
    double q[N + 1][NZ];          // Newton-system gradient
    double dz[N + 1][NZ];         // QP primal iterate
    double ddz[N + 1][NZ];        // QP primal step
    double pi_nlp[N][NX];         // NLP dynamics multipliers
    double piq[N][NX];            // QP dynamics multipliers
    double pin[N][NX];            // QP multipliers after the Newton step
    double rdyn[N][NX];           // QP dynamics residual
    double P[N + 1][NX][NX];      // Riccati cost-to-go
    double p[N + 1][NX];
    double Lc[N][3];              // chol(Muu)
    double Y[N][NU][NX];          // L^{-1} Mux
    double yv[N][NU];
    double M[NZ][NZ];             // factorisation scratch
    double xinit[NX];
    double lamw[NH][N];           // signed NLP multipliers of h (Hessian weights)
    double Dg[NH][3][N];          // signed h-row gradient over (x, y, psi)
    double rd[NR][N], rt[NR][N], rl[NR][N], rdt[NR][N], rdl[NR][N], rin[NR][N], rrc[NR][N];
    int flag;
};

// Diagnostic per-phase cycle stamps (separate build with -DMPCG_STAMPS; the
// production build compiles them out).  Shares of a phase, not absolute times.
#ifdef MPCG_STAMPS
#define STAMP_DECL unsigned long long st_acc_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_t0_ = 0;
#define STAMP_BEGIN()                                  \
    do {                                               \
        __syncthreads();                               \
        st_t0_ = __builtin_amdgcn_s_memtime();         \
    } while (0)
#define STAMP_END(i)                                           \
    do {                                                       \
        __syncthreads();                                       \
        st_acc_[i] += __builtin_amdgcn_s_memtime() - st_t0_;   \
    } while (0)
#define STAMP_STORE(ptr, sol)                                                      \
    do {                                                                           \
        if ((ptr) && threadIdx.x == 0)                                             \
            for (int i_ = 0; i_ < 10; ++i_) (ptr)[(size_t)(sol) * 10 + i_] = st_acc_[i_]; \
    } while (0)
#else
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(i) do {} while (0)
#define STAMP_STORE(ptr, sol) do {} while (0)
#endif

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---- inequality rows of stage k ------------------------------------------
// r in [0,4): input bounds (a lo, a hi, w lo, w hi); r in [4,14): state
// bounds (x lo, x hi, ...); r >= 14: h row r-14 (one finite side each).
__device__ __forceinline__ int row_var(int r) { return r < 2 * NU ? (r >> 1) : NU + ((r - 2 * NU) >> 1); }
__device__ __forceinline__ double row_sign(int r) { return (r & 1) ? 1.0 : -1.0; }

template <class C>
__device__ __forceinline__ int nrows(int k) { return k == 0 ? C::NR0 : (k < C::N ? C::NR : 0); }

template <class C>
__device__ __forceinline__ double row_dot(const Lds<C>& S, int r, int k, const double* v) {
    if (r < 2 * NU + 2 * NX) return row_sign(r) * v[row_var(r)];
    const int j = r - (2 * NU + 2 * NX);
    return S.Dg[j][0][k] * v[2] + S.Dg[j][1][k] * v[3] + S.Dg[j][2][k] * v[4];
}

// ---- linearisation of stage k (one lane) ----------------------------------
template <class C>
__device__ void linearize_stage(const mpcg_problem& pr, Lds<C>& S, const double* __restrict__ pk, int k,
                                double& res_local) {
    double z[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) z[i] = S.z[k][i];
    double g[NZ], H[NZ][NZ], F[NX][NZ], xn[NX];
    stage_cost(pr, pk, z, g, H, true);
    double pi[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) pi[i] = S.pi_nlp[k][i];
    erk_unicycle(pr, z, pi, xn, F, H);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        const double bi = xn[i] - S.z[k + 1][NU + i];
        S.b[k][i] = bi;
        res_local = fmax(res_local, fabs(bi));
#pragma unroll
        for (int j = 0; j < NZ; ++j) S.F[k][i][j] = F[i][j];
    }
    // input bounds (all stages < N)
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        S.rd[2 * i][k] = z[i] - pr.lbu[i];
        S.rd[2 * i + 1][k] = pr.ubu[i] - z[i];
    }
    if (k >= 1) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            S.rd[2 * NU + 2 * i][k] = z[NU + i] - pr.lbx[i];
            S.rd[2 * NU + 2 * i + 1][k] = pr.ubx[i] - z[NU + i];
        }
        const double x = z[2], y = z[3], psi = z[4];
        // topology halfspaces a1 x + a2 y - b <= 0 (guidance_constraints.py:355-370)
        for (int i = 0; i < C::NL; ++i) {
            const double* c = pk + pr.i_lin0 + 3 * i;
            const double h = c[0] * x + c[1] * y - c[2];
            const int r = 2 * NU + 2 * NX + i;
            S.rd[r][k] = 0.0 - h;  // uh - h
            S.Dg[i][0][k] = c[0];
            S.Dg[i][1][k] = c[1];
            S.Dg[i][2][k] = 0.0;
        }
        // ellipsoids d' R'DR d >= 1 (ellipsoid_constraints.py:435-489), lower side
        const double rdisc = pk[pr.i_disc_r], off = pk[pr.i_disc_off];
        double sp, cp;
        sincos(psi, &sp, &cp);
        const double dxp = -off * sp, dyp = off * cp, dxpp = -off * cp, dypp = -off * sp;
        double hb[6] = {0, 0, 0, 0, 0, 0};  // sum of weighted Hessians on (x,y,psi): xx xy xp yy yp pp
        for (int j = 0; j < C::NE; ++j) {
            const double* o = pk + pr.i_ell0 + 7 * j;
            const double chi = sqrt(o[5]);
            const double ra = o[3] * chi + rdisc + o[6];
            const double rb = o[4] * chi + rdisc + o[6];
            const double D0 = 1.0 / (ra * ra), D1 = 1.0 / (rb * rb);
            double so, co;
            sincos(o[2], &so, &co);
            const double M00 = co * co * D0 + so * so * D1;
            const double M01 = -co * so * D0 + so * co * D1;
            const double M11 = so * so * D0 + co * co * D1;
            const double ddx = x + off * cp - o[0], ddy = y + off * sp - o[1];
            const double Mdx = M00 * ddx + M01 * ddy, Mdy = M01 * ddx + M11 * ddy;
            const double h = ddx * Mdx + ddy * Mdy;
            const int jr = C::NL + j;
            const int r = 2 * NU + 2 * NX + jr;
            S.rd[r][k] = h - 1.0;  // h - lh
            S.Dg[jr][0][k] = -2.0 * Mdx;
            S.Dg[jr][1][k] = -2.0 * Mdy;
            S.Dg[jr][2][k] = -2.0 * (Mdx * dxp + Mdy * dyp);
            const double wgt = S.lamw[jr][k];
            if (wgt != 0.0) {
                const double hxp = 2.0 * (M00 * dxp + M01 * dyp);
                const double hyp = 2.0 * (M01 * dxp + M11 * dyp);
                const double hpp = 2.0 * (dxp * (M00 * dxp + M01 * dyp) + dyp * (M01 * dxp + M11 * dyp)) +
                                   2.0 * (Mdx * dxpp + Mdy * dypp);
                hb[0] += wgt * 2.0 * M00; hb[1] += wgt * 2.0 * M01; hb[2] += wgt * hxp;
                hb[3] += wgt * 2.0 * M11; hb[4] += wgt * hyp; hb[5] += wgt * hpp;
            }
        }
        H[2][2] += hb[0]; H[2][3] += hb[1]; H[3][2] += hb[1];
        H[2][4] += hb[2]; H[4][2] += hb[2];
        H[3][3] += hb[3]; H[3][4] += hb[4]; H[4][3] += hb[4];
        H[4][4] += hb[5];
    }
    mirror7(H, pr.reg_eps);
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        S.g[k][i] = g[i];
#pragma unroll
        for (int j = 0; j < NZ; ++j) S.H[k][i][j] = H[i][j];
    }
}

// ---- one full solve -------------------------------------------------------
template <class C>
__global__ __launch_bounds__(64) void sqp_kernel(mpcg_problem pr, int batch,
                                                 const double* __restrict__ params,
                                                 const double* __restrict__ warm,
                                                 const double* __restrict__ xinit,
                                                 double* __restrict__ xtraj, double* __restrict__ utraj,
                                                 double* __restrict__ pobj_out, int* __restrict__ exit_out,
                                                 int* __restrict__ info_out,
                                                 unsigned long long* __restrict__ stamps) {
    constexpr int N = C::N, NH = C::NH;
    STAMP_DECL
    __shared__ Lds<C> S;
    const int sol = blockIdx.x;
    if (sol >= batch) return;
    const int lane = threadIdx.x;
    const int npar = pr.npar;

    // ---- load warm start (loadWarmstart, acados_solver_interface.cpp:499-509)
    const double* w = warm + (size_t)sol * (N + 1) * NZ;
    for (int e = lane; e < (N + 1) * NZ; e += 64) (&S.z[0][0])[e] = w[e];
    if (lane < NX) S.xinit[lane] = xinit[(size_t)sol * NX + lane];
    for (int e = lane; e < N * NX; e += 64) (&S.pi_nlp[0][0])[e] = 0.0;
    for (int e = lane; e < NH * N; e += 64) (&S.lamw[0][0])[e] = 0.0;
    __syncthreads();
    if (lane < NU) S.z[N][lane] = 0.0;
    __syncthreads();

    int acados_status = AC_SUCCESS, qp_status = AC_SUCCESS, sqp_iter = 0, qp_total = 0;
    double res_eq = 0.0;
    const double* pbase = params + (size_t)sol * N * npar;

    for (int it = 0; it < pr.sqp_iters; ++it) {
        // ================= preparation: linearise =================
        STAMP_BEGIN();
        double resl = 0.0;
        if (lane < N) {
            linearize_stage<C>(pr, S, pbase + (size_t)lane * npar, lane, resl);
        } else if (lane == N) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                S.g[N][i] = 0.0;
#pragma unroll
                for (int j = 0; j < NZ; ++j) S.H[N][i][j] = (i == j && i >= NU) ? pr.reg_eps : 0.0;
            }
        }
        res_eq = wave_max(resl);
        if (lane < NX) S.dz[0][NU + lane] = S.xinit[lane] - S.z[0][NU + lane];
        __syncthreads();
        STAMP_END(0);
        STAMP_BEGIN();

        // ================= feedback: QP (Riccati interior point) =================
        // cold start
        if (lane <= N) {
            const int k = lane;
#pragma unroll
            for (int i = 0; i < NZ; ++i)
                if (!(k == 0 && i >= NU)) S.dz[k][i] = 0.0;
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.piq[k][i] = 0.0;
            }
            const int nr = nrows<C>(k);
            for (int r = 0; r < nr; ++r) {
                const double s = S.rd[r][k];
                const double t = s > pr.qp_thr0 ? s : pr.qp_thr0;
                S.rt[r][k] = t;
                S.rl[r][k] = pr.qp_mu0 / t;
            }
        }
        __syncthreads();
        int qstat = AC_MAXITER, qit = 0;
        STAMP_END(1);
        for (;; ++qit) {
            // ---- residuals
            STAMP_BEGIN();
            double rs = 0.0, re = 0.0, ri = 0.0, comp = 0.0;
            if (lane <= N) {
                const int k = lane;
                double dzk[NZ], r[NZ];
#pragma unroll
                for (int i = 0; i < NZ; ++i) dzk[i] = S.dz[k][i];
#pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    double acc = S.g[k][i];
#pragma unroll
                    for (int j = 0; j < NZ; ++j) acc += S.H[k][i][j] * dzk[j];
                    r[i] = acc;
                }
                if (k < N) {
#pragma unroll
                    for (int m = 0; m < NX; ++m) {
                        const double pm = S.piq[k][m];
#pragma unroll
                        for (int i = 0; i < NZ; ++i) r[i] += S.F[k][m][i] * pm;
                    }
                    double dxn[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        double acc = S.b[k][i] - S.dz[k + 1][NU + i];
#pragma unroll
                        for (int j = 0; j < NZ; ++j) acc += S.F[k][i][j] * dzk[j];
                        dxn[i] = acc;
                        S.rdyn[k][i] = acc;
                        re = fmax(re, fabs(acc));
                    }
                }
                if (k > 0) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) r[NU + i] -= S.piq[k - 1][i];
                }
                const int nr = nrows<C>(k);
                for (int rr = 0; rr < nr; ++rr) {
                    const double l = S.rl[rr][k], t = S.rt[rr][k];
                    if (rr < 2 * NU + 2 * NX) {
                        r[row_var(rr)] += row_sign(rr) * l;
                    } else {
                        const int j = rr - (2 * NU + 2 * NX);
                        r[2] += S.Dg[j][0][k] * l; r[3] += S.Dg[j][1][k] * l; r[4] += S.Dg[j][2][k] * l;
                    }
                    const double rin = row_dot(S, rr, k, dzk) + t - S.rd[rr][k];
                    S.rin[rr][k] = rin;
                    ri = fmax(ri, fabs(rin));
                    comp += l * t;
                }
                const int i0 = (k == N) ? NU : 0, i1 = (k == 0) ? NU : NZ;
#pragma unroll
                for (int i = 0; i < NZ; ++i)
                    if (i >= i0 && i < i1) rs = fmax(rs, fabs(r[i]));
            }
            rs = wave_max(rs); re = wave_max(re); ri = wave_max(ri);
            comp = wave_sum(comp);
            const double mu = comp / C::M_TOTAL;
            if (!(rs < 1e30) || !(re < 1e30) || !(ri < 1e30) || !(mu < 1e16)) { qstat = AC_NAN; break; }
            if (rs < pr.qp_tol && re < pr.qp_tol && ri < pr.qp_tol && mu < pr.qp_tol) { qstat = AC_SUCCESS; break; }
            if (qit >= pr.qp_iter_max) { qstat = AC_MAXITER; break; }
            __syncthreads();
            STAMP_END(2);

            double alpha = 1.0;
            double sigma_mu = 0.0;
            for (int phase = 0; phase < 2; ++phase) {
                // ---- barrier Hessian terms (predictor only) and Newton gradient q
                STAMP_BEGIN();
                if (lane <= N) {
                    const int k = lane;
                    double qk[NZ], dzk[NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) dzk[i] = S.dz[k][i];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) {
                        double acc = S.g[k][i];
#pragma unroll
                        for (int j = 0; j < NZ; ++j) acc += S.H[k][i][j] * dzk[j];
                        qk[i] = acc;
                    }
                    double dd[NZ] = {0, 0, 0, 0, 0, 0, 0};
                    double db[6] = {0, 0, 0, 0, 0, 0};
                    const int nr = nrows<C>(k);
                    for (int rr = 0; rr < nr; ++rr) {
                        const double l = S.rl[rr][k], t = S.rt[rr][k], rin = S.rin[rr][k];
                        double rc;
                        if (phase == 0) {
                            rc = l * t;
                        } else {
                            rc = l * t + S.rdt[rr][k] * S.rdl[rr][k] - sigma_mu;
                        }
                        S.rrc[rr][k] = rc;
                        const double coef = l + (l * rin - rc) / t;
                        const double wgt = l / t;
                        if (rr < 2 * NU + 2 * NX) {
                            const int v = row_var(rr);
                            qk[v] += row_sign(rr) * coef;
                            dd[v] += wgt;
                        } else {
                            const int j = rr - (2 * NU + 2 * NX);
                            const double d0 = S.Dg[j][0][k], d1 = S.Dg[j][1][k], d2 = S.Dg[j][2][k];
                            qk[2] += d0 * coef; qk[3] += d1 * coef; qk[4] += d2 * coef;
                            db[0] += d0 * wgt * d0; db[1] += d0 * wgt * d1; db[2] += d0 * wgt * d2;
                            db[3] += d1 * wgt * d1; db[4] += d1 * wgt * d2; db[5] += d2 * wgt * d2;
                        }
                    }
#pragma unroll
                    for (int i = 0; i < NZ; ++i) S.q[k][i] = qk[i];
                    if (phase == 0) {
#pragma unroll
                        for (int i = 0; i < NZ; ++i) S.dH[k][i] = dd[i];
#pragma unroll
                        for (int i = 0; i < 6; ++i) S.dH[k][NZ + i] = db[i];
                    }
                }
                __syncthreads();
                STAMP_END(3);
                // ---- Riccati factorisation (predictor only; the corrector reuses it)
                STAMP_BEGIN();
                if (phase == 0) {
                    if (lane < NX * NX) {
                        const int i = lane / NX, j = lane % NX;
                        double v = S.H[N][NU + i][NU + j];
                        if (i == j) v += S.dH[N][NU + i];
                        S.P[N][i][j] = v;
                    }
                    if (lane == 0) S.flag = 0;
                    __syncthreads();
                    for (int k = N - 1; k >= 0; --k) {
                        if (lane < NZ * NZ) {
                            const int i = lane / NZ, j = lane % NZ;
                            // t_l = sum_m F[m][i] P[m][l]
                            double tl[NX];
#pragma unroll
                            for (int l = 0; l < NX; ++l) {
                                double acc = 0.0;
#pragma unroll
                                for (int m = 0; m < NX; ++m) acc += S.F[k][m][i] * S.P[k + 1][m][l];
                                tl[l] = acc;
                            }
                            double v = S.H[k][i][j];
                            if (i == j) v += S.dH[k][i];
                            if (i >= 2 && i <= 4 && j >= 2 && j <= 4) {
                                const int a = i - 2, bb = j - 2;
                                const int lo = a < bb ? a : bb, hi = a < bb ? bb : a;
                                const int idx = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
                                v += S.dH[k][NZ + idx];
                            }
#pragma unroll
                            for (int l = 0; l < NX; ++l) v += tl[l] * S.F[k][l][j];
                            S.M[i][j] = v;
                        }
                        __syncthreads();
                        if (lane < NX * NX) {
                            const int i = lane / NX, j = lane % NX;
                            const double m00 = S.M[0][0];
                            const double l00 = sqrt(m00);
                            const double l10 = S.M[1][0] / l00;
                            const double m11 = S.M[1][1] - l10 * l10;
                            const double l11 = sqrt(m11);
                            if (!(m00 > 0.0) || !(m11 > 0.0)) S.flag = 1;
                            const double y0i = S.M[0][NU + i] / l00;
                            const double y1i = (S.M[1][NU + i] - l10 * y0i) / l11;
                            const double y0j = S.M[0][NU + j] / l00;
                            const double y1j = (S.M[1][NU + j] - l10 * y0j) / l11;
                            S.P[k][i][j] = S.M[NU + i][NU + j] - y0i * y0j - y1i * y1j;
                            if (j == 0) { S.Y[k][0][i] = y0i; S.Y[k][1][i] = y1i; }
                            if (lane == 0) { S.Lc[k][0] = l00; S.Lc[k][1] = l10; S.Lc[k][2] = l11; }
                        }
                        __syncthreads();
                    }
                    if (S.flag) { qstat = AC_NAN; break; }
                }
                STAMP_END(4);
                // ---- vector + forward passes.  Lane k owns stage k: it folds its
                // stage block into two affine 5-vector recursions
                //   p_k = h_k + G_k p_{k+1}          (cost-to-go gradient)
                //   dx_{k+1} = Phi_k dx_k + e_k        (closed-loop rollout, Phi_k = G_k')
                // so the sequential chain is one 5x5 mat-vec per stage, carried
                // in SGPRs through v_readlane; everything else is stage-parallel.
                STAMP_BEGIN();
                {
                    const bool own = lane < N;
                    const int k = own ? lane : 0;
                    double Fl[NX][NZ], P1[NX][NX], G[NX][NX], hv[NX], W0[NX], W1[NX], Y0[NX], Y1[NX], rr[NX];
                    const double l00 = S.Lc[k][0], l10 = S.Lc[k][1], l11 = S.Lc[k][2];
                    double y0a, y0b;
                    {
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            rr[i] = S.rdyn[k][i];
                            Y0[i] = S.Y[k][0][i];
                            Y1[i] = S.Y[k][1][i];
#pragma unroll
                            for (int j = 0; j < NZ; ++j) Fl[i][j] = S.F[k][i][j];
#pragma unroll
                            for (int j = 0; j < NX; ++j) P1[i][j] = S.P[k + 1][i][j];
                        }
                        double c[NX], m0[NZ];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = 0.0;
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += P1[i][j] * rr[j];
                            c[i] = acc;
                        }
#pragma unroll
                        for (int i = 0; i < NZ; ++i) {
                            double acc = S.q[k][i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += Fl[j][i] * c[j];
                            m0[i] = acc;
                        }
                        y0a = m0[0] / l00;
                        y0b = (m0[1] - l10 * y0a) / l11;
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            hv[i] = m0[NU + i] - Y0[i] * y0a - Y1[i] * y0b;
                            W0[i] = Fl[i][0] / l00;
                            W1[i] = (Fl[i][1] - l10 * W0[i]) / l11;
                        }
#pragma unroll
                        for (int i = 0; i < NX; ++i)
#pragma unroll
                            for (int j = 0; j < NX; ++j) G[i][j] = Fl[j][NU + i] - Y0[i] * W0[j] - Y1[i] * W1[j];
                    }
                    // backward chain
                    double pu[NX], pmine[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) { pu[i] = S.q[N][NU + i]; pmine[i] = pu[i]; }
                    for (int kk = N - 1; kk >= 0; --kk) {
                        double pn[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = hv[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += G[i][j] * pu[j];
                            pn[i] = acc;
                        }
                        const bool mine = (lane == kk);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            pmine[i] = mine ? pu[i] : pmine[i];
                            pu[i] = readlane_d(pn[i], kk);
                        }
                    }
                    // feedback terms of stage k
                    const double ya = y0a + W0[0] * pmine[0] + W0[1] * pmine[1] + W0[2] * pmine[2] + W0[3] * pmine[3] + W0[4] * pmine[4];
                    const double yb = y0b + W1[0] * pmine[0] + W1[1] * pmine[1] + W1[2] * pmine[2] + W1[3] * pmine[3] + W1[4] * pmine[4];
                    const double kf1 = -yb / l11;
                    const double kf0 = (-ya - l10 * kf1) / l00;
                    double K0[NX], K1[NX], e[NX];
#pragma unroll
                    for (int j = 0; j < NX; ++j) {
                        K1[j] = -Y1[j] / l11;
                        K0[j] = (-Y0[j] - l10 * K1[j]) / l00;
                    }
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        e[i] = rr[i] + Fl[i][0] * kf0 + Fl[i][1] * kf1;
#pragma unroll
                        for (int j = 0; j < NX; ++j) G[i][j] = Fl[i][NU + j] + Fl[i][0] * K0[j] + Fl[i][1] * K1[j];  // Phi
                    }
                    // forward chain
                    double dxu[NX] = {0, 0, 0, 0, 0}, dxmine[NX] = {0, 0, 0, 0, 0};
                    for (int kk = 0; kk < N; ++kk) {
                        double dn[NX];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = e[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += G[i][j] * dxu[j];
                            dn[i] = acc;
                        }
                        const bool mine = (lane == kk);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            dxmine[i] = mine ? dxu[i] : dxmine[i];
                            dxu[i] = readlane_d(dn[i], kk);
                        }
                    }
                    if (own) {
                        double du0 = kf0, du1 = kf1, dxn[NX];
#pragma unroll
                        for (int j = 0; j < NX; ++j) { du0 += K0[j] * dxmine[j]; du1 += K1[j] * dxmine[j]; }
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = e[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += G[i][j] * dxmine[j];
                            dxn[i] = acc;
                        }
                        S.ddz[k][0] = du0;
                        S.ddz[k][1] = du1;
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            S.ddz[k][NU + i] = (k == 0) ? 0.0 : dxmine[i];
                            double acc = pmine[i];
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += P1[i][j] * dxn[j];
                            S.pin[k][i] = acc;
                        }
                        if (k == N - 1) {
                            S.ddz[N][0] = 0.0;
                            S.ddz[N][1] = 0.0;
#pragma unroll
                            for (int i = 0; i < NX; ++i) S.ddz[N][NU + i] = dxn[i];
                        }
                    }
                }
                __syncthreads();
                STAMP_END(5);
                // ---- inequality steps and step length
                STAMP_BEGIN();
                double amax = 1e300;
                if (lane < N) {
                    const int k = lane;
                    double dd[NZ];
#pragma unroll
                    for (int i = 0; i < NZ; ++i) dd[i] = S.ddz[k][i];
                    const int nr = nrows<C>(k);
                    for (int rr = 0; rr < nr; ++rr) {
                        const double t = S.rt[rr][k], l = S.rl[rr][k];
                        const double dt = -S.rin[rr][k] - row_dot(S, rr, k, dd);
                        const double dl = -(S.rrc[rr][k] + l * dt) / t;
                        S.rdt[rr][k] = dt;
                        S.rdl[rr][k] = dl;
                        if (dt < 0.0) amax = fmin(amax, -t / dt);
                        if (dl < 0.0) amax = fmin(amax, -l / dl);
                    }
                }
                amax = wave_min(amax);
                if (phase == 0) {
                    const double aa = fmin(amax, 1.0);
                    double ca = 0.0;
                    if (lane < N) {
                        const int k = lane;
                        const int nr = nrows<C>(k);
                        for (int rr = 0; rr < nr; ++rr)
                            ca += (S.rl[rr][k] + aa * S.rdl[rr][k]) * (S.rt[rr][k] + aa * S.rdt[rr][k]);
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
                }
                __syncthreads();
                STAMP_END(7);
            }
            if (qstat == AC_NAN) break;
            if (alpha < 1e-12) { qstat = AC_MINSTEP; ++qit; break; }
            // ---- update
            STAMP_BEGIN();
            if (lane <= N) {
                const int k = lane;
#pragma unroll
                for (int i = 0; i < NZ; ++i) S.dz[k][i] += alpha * S.ddz[k][i];
                if (k < N) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) S.piq[k][i] += alpha * (S.pin[k][i] - S.piq[k][i]);
                }
                const int nr = nrows<C>(k);
                for (int rr = 0; rr < nr; ++rr) {
                    S.rt[rr][k] += alpha * S.rdt[rr][k];
                    S.rl[rr][k] += alpha * S.rdl[rr][k];
                }
            }
            __syncthreads();
            STAMP_END(8);
        }
        __syncthreads();
        qp_status = qstat;
        qp_total += qit;
        ++sqp_iter;
        if (qstat != AC_SUCCESS && qstat != AC_MAXITER) {
            acados_status = AC_QP_FAILURE;
            break;
        }
        // FIXED_STEP full step on primal and multipliers
        if (lane <= N) {
            const int k = lane;
#pragma unroll
            for (int i = 0; i < NZ; ++i) S.z[k][i] += S.dz[k][i];
            if (k == N) { S.z[N][0] = 0.0; S.z[N][1] = 0.0; }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.pi_nlp[k][i] = S.piq[k][i];
                for (int j = 0; j < NH; ++j) {
                    const double l = (k >= 1) ? S.rl[2 * NU + 2 * NX + j][k] : 0.0;
                    S.lamw[j][k] = (j < C::NL) ? l : -l;  // upper rows +lambda, lower rows -lambda
                }
            }
        }
        __syncthreads();
        acados_status = AC_SUCCESS;
        if (qstat != AC_SUCCESS) break;
    }

    // ---- completeOneIteration (acados_solver_interface.cpp:387-429)
    STAMP_BEGIN();
    double Lk = 0.0;
    if (lane < N) {
        double zk[NZ], gd[NZ], Hd[NZ][NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zk[i] = S.z[lane][i];
        Lk = stage_cost(pr, pbase + (size_t)lane * npar, zk, gd, Hd, false);
    }
    const double pobj = wave_sum(Lk);
    double* xo = xtraj + (size_t)sol * (N + 1) * NX;
    for (int e = lane; e < (N + 1) * NX; e += 64) xo[e] = S.z[e / NX][NU + e % NX];
    double* uo = utraj + (size_t)sol * N * NU;
    for (int e = lane; e < N * NU; e += 64) uo[e] = S.z[e / NU][e % NU];
    if (lane == 0) {
        int code = acados_status;
        if (res_eq > pr.res_eq_fail && code == AC_SUCCESS) code = AC_QP_FAILURE;
        if (code == AC_SUCCESS) code = 1;
        else if (code == 1) code = 0;
        exit_out[sol] = code;
        pobj_out[sol] = pobj;
        if (info_out) {
            info_out[(size_t)sol * MPCG_INFO_STRIDE + 0] = sqp_iter;
            info_out[(size_t)sol * MPCG_INFO_STRIDE + 1] = qp_total;
            info_out[(size_t)sol * MPCG_INFO_STRIDE + 2] = qp_status;
            info_out[(size_t)sol * MPCG_INFO_STRIDE + 3] = 0;
        }
    }
    STAMP_END(9);
    STAMP_STORE(stamps, sol);
}

// ---- planner selection per scene (guidance_constraints.cpp:372-420, 572-590)
__global__ void select_best_kernel(int n_scenes, int G, int N, const double* __restrict__ xtraj,
                                   const double* __restrict__ pobj, const int* __restrict__ exit_code,
                                   const double* __restrict__ prev, double w_cons,
                                   const unsigned char* __restrict__ cons_en,
                                   const unsigned char* __restrict__ prev_sel, double sel_w,
                                   const unsigned char* __restrict__ disabled, int* __restrict__ best,
                                   double* __restrict__ objective) {
    const int sc = blockIdx.x * blockDim.x + threadIdx.x;
    if (sc >= n_scenes) return;
    double best_obj = 1e10;
    int best_i = -1;
    for (int g = 0; g < G; ++g) {
        const int s = sc * G + g;
        double obj = pobj[s];
        if (prev && cons_en && cons_en[s]) {
            // calculateConsistencyCostForSolver (guidance_constraints.cpp:1025-1050)
            double acc = 0.0;
            for (int k = 1; k <= N - 2; ++k) {
                const double dx = xtraj[((size_t)s * (N + 1) + k) * NX + 0] - prev[((size_t)sc * N + k) * 2 + 0];
                const double dy = xtraj[((size_t)s * (N + 1) + k) * NX + 1] - prev[((size_t)sc * N + k) * 2 + 1];
                acc += dx * dx + dy * dy;
            }
            obj -= w_cons * acc;
        }
        if (prev_sel && prev_sel[s]) obj *= sel_w;
        if (objective) objective[s] = obj;
        const bool dis = disabled && disabled[s];
        if (!dis && exit_code[s] == 1 && obj < best_obj) {
            best_obj = obj;
            best_i = g;
        }
    }
    best[sc] = best_i;
}

// ---- dispatch over compiled instances ------------------------------------
static thread_local std::string g_err;
static unsigned long long* g_stamps = nullptr;  // diagnostic stamp buffer (MPCG_STAMPS builds only)

template <class C>
static int launch(const mpcg_problem& pr, int batch, const double* params, const double* warm,
                  const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                  int* info, hipStream_t stream) {
    hipLaunchKernelGGL((sqp_kernel<C>), dim3(batch), dim3(64), 0, stream, pr, batch, params, warm, xinit,
                       xtraj, utraj, pobj, exit_code, info, g_stamps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("sqp_kernel launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

using Fn = int (*)(const mpcg_problem&, int, const double*, const double*, const double*, double*, double*,
                   double*, int*, int*, hipStream_t);

static Fn find_instance(const mpcg_problem& pr) {
    if (pr.rk_steps < 1 || pr.n_seg < 1 || pr.n_seg > 16) return nullptr;
#define MPCG_INST(N_, L_, E_) \
    if (pr.N == N_ && pr.n_lin == L_ && pr.n_ell == E_) return &launch<Cfg<N_, L_, E_>>;
    MPCG_INST(20, 4, 4)    // C1
    MPCG_INST(20, 8, 8)    // C2 (north star)
    MPCG_INST(30, 12, 12)  // C4
    MPCG_INST(10, 2, 2)    // small test instance
#undef MPCG_INST
    return nullptr;
}

}  // namespace mpcg

extern "C" {

int mpcg_abi_version(void) { return MPCG_ABI_VERSION; }

/* diagnostic builds only: device buffer of batch x 10 u64 phase-cycle sums */
void mpcg_debug_set_stamp_buffer(unsigned long long* dev_ptr) { mpcg::g_stamps = dev_ptr; }

const char* mpcg_last_error(void) { return mpcg::g_err.c_str(); }

int mpcg_supported(const mpcg_problem* pr) { return (pr && mpcg::find_instance(*pr)) ? 0 : -1; }

int mpcg_solve_batch_device(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                            const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                            int* info, void* stream) {
    if (!pr || batch < 0) { mpcg::g_err = "invalid arguments"; return -1; }
    if (batch == 0) return 0;
    mpcg::Fn fn = mpcg::find_instance(*pr);
    if (!fn) {
        mpcg::g_err = "no compiled instance for N=" + std::to_string(pr->N) + " n_lin=" + std::to_string(pr->n_lin) +
                      " n_ell=" + std::to_string(pr->n_ell);
        return -2;
    }
    return fn(*pr, batch, params, warm, xinit, xtraj, utraj, pobj, exit_code, info, (hipStream_t)stream);
}

int mpcg_solve_batch_host(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                          const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                          int* info) {
    if (!pr || batch < 0) { mpcg::g_err = "invalid arguments"; return -1; }
    if (batch == 0) return 0;
    const size_t N = pr->N, np = pr->npar;
    const size_t s_par = batch * N * np, s_warm = batch * (N + 1) * MPCG_NVAR, s_xi = (size_t)batch * MPCG_NX;
    const size_t s_xt = batch * (N + 1) * MPCG_NX, s_ut = batch * N * MPCG_NU;
    double *dpar, *dwarm, *dxi, *dxt, *dut, *dpo;
    int *dex, *dinfo;
    size_t dbl = s_par + s_warm + s_xi + s_xt + s_ut + batch;
    if (hipMalloc(&dpar, dbl * sizeof(double)) != hipSuccess) { mpcg::g_err = "hipMalloc failed"; return -3; }
    if (hipMalloc(&dex, (size_t)batch * (1 + MPCG_INFO_STRIDE) * sizeof(int)) != hipSuccess) {
        (void)hipFree(dpar);
        mpcg::g_err = "hipMalloc failed";
        return -3;
    }
    dwarm = dpar + s_par; dxi = dwarm + s_warm; dxt = dxi + s_xi; dut = dxt + s_xt; dpo = dut + s_ut;
    dinfo = dex + batch;
    bool ok = hipMemcpy(dpar, params, s_par * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dwarm, warm, s_warm * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dxi, xinit, s_xi * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    int rc = ok ? mpcg_solve_batch_device(pr, batch, dpar, dwarm, dxi, dxt, dut, dpo, dex, dinfo, nullptr) : -5;
    if (!ok) mpcg::g_err = "host to device copy failed";
    if (rc == 0) {
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) { mpcg::g_err = std::string("solve: ") + hipGetErrorString(e); rc = -4; }
    }
    if (rc == 0) {
        ok = hipMemcpy(xtraj, dxt, s_xt * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(utraj, dut, s_ut * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(pobj, dpo, batch * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(exit_code, dex, batch * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess &&
             (!info || hipMemcpy(info, dinfo, (size_t)batch * MPCG_INFO_STRIDE * sizeof(int),
                                 hipMemcpyDeviceToHost) == hipSuccess);
        if (!ok) { mpcg::g_err = "device to host copy failed"; rc = -5; }
    }
    (void)hipFree(dpar);
    (void)hipFree(dex);
    return rc;
}

int mpcg_select_best_device(int n_scenes, int n_guesses, int N, const double* xtraj, const double* pobj,
                            const int* exit_code, const double* prev_traj, double w_cons,
                            const unsigned char* consistency_enabled, const unsigned char* previously_selected,
                            double selection_weight, const unsigned char* disabled, int* best, double* objective,
                            void* stream) {
    if (n_scenes <= 0) return 0;
    const int T = 64;
    hipLaunchKernelGGL(mpcg::select_best_kernel, dim3((n_scenes + T - 1) / T), dim3(T), 0, (hipStream_t)stream,
                       n_scenes, n_guesses, N, xtraj, pobj, exit_code, prev_traj, w_cons, consistency_enabled,
                       previously_selected, selection_weight, disabled, best, objective);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("select_best launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // extern "C"
