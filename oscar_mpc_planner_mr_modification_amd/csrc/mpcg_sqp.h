// mpcg_sqp.h — the batched SQP-RTI solve kernel (one wavefront per solve).
//
// Reference: one `Solver::solve()` of the OpenMP fan-out in
// GuidanceConstraints::optimize (guidance_constraints.cpp:304-421) =
// `sqp_iters` acados SQP-RTI iterations (acados_solver_interface.cpp:311-429).
//
// Lane layout (PARTS lanes per shooting stage, lane = k * PARTS + part):
//   part 0 of stage k  cost / ERK4 / MIRROR / Riccati stage algebra of stage k,
//                      the box-bound rows of stage k, and (PARTS == 2) the
//                      first h rows
//   parts 1..          the nonlinear-constraint (h) rows of stage k
// Every inequality row keeps its interior-point state (bound gap d, slack t,
// multiplier lambda, predictor product, residual) in REGISTERS of its owner
// lane for the whole solve; only stage blocks live in LDS (~27 KB per solve
// for N=20, so 4 solves per CU — one wavefront per SIMD).
//   element lanes      e < 28 own entry (i >= j) of the 7x7 stage block in the
//                      Riccati factorisation
//   chains             the two 5-vector recursions of each Newton solve run as
//                      affine maps carried in SGPRs through v_readlane.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mpcg.h"
#include "mpcg_device.h"

namespace mpcg {

enum { AC_SUCCESS = 0, AC_NAN = 1, AC_MAXITER = 2, AC_MINSTEP = 3, AC_QP_FAILURE = 4 };

constexpr int NBOX = 2 * NU + 2 * NX;  // box rows of a stage in 1..N-1 (input + state bounds)

__host__ __device__ constexpr int imax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int sym(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

template <int N_, int NL_, int NE_>
struct Cfg {
    static constexpr int N = N_, NL = NL_, NE = NE_;
    static constexpr int NH = NL + NE;
    static constexpr int PARTS = (64 / (N + 1)) >= 3 ? 3 : 2;
    static_assert((N + 1) * PARTS <= 64, "horizon too long for one wavefront");
    // h rows owned by part 0 (only when PARTS == 2, to balance the two lanes)
    static constexpr int H0 = PARTS == 2 ? imax(0, (NH - NBOX) / 2) : 0;
    static constexpr int M_TOTAL = 2 * NU + (N - 1) * (NBOX + NH);
    // h row range of part p
    __host__ __device__ static constexpr int hb(int p) {
        return p == 0 ? 0 : (PARTS == 2 ? H0 : (p == 1 ? 0 : NH / 2));
    }
    __host__ __device__ static constexpr int he(int p) {
        return p == 0 ? H0 : (PARTS == 2 ? NH : (p == 1 ? NH / 2 : NH));
    }
    __host__ __device__ static constexpr int nbox(int p) { return p == 0 ? NBOX : 0; }
    __host__ __device__ static constexpr int nslot(int p) { return nbox(p) + he(p) - hb(p); }
    static constexpr int SLOTS = imax(nslot(0), imax(nslot(1), PARTS > 2 ? nslot(2) : 0));
    static constexpr int HSLOTS = imax(he(0) - hb(0), imax(he(1) - hb(1), PARTS > 2 ? he(2) - hb(2) : 0));
};

template <class C>
struct Lds {
    static constexpr int N = C::N;
    double z[N + 1][NZ];      // NLP iterate [u x]
    double H[N + 1][28];      // MIRROR-regularised Lagrangian Hessian, packed lower triangle
    double g[N + 1][NZ];
    double F[N][NX][NZ];      // [B A]
    double b[N][NX];          // shooting defects
    double dH[N + 1][13];     // barrier terms: diag(7) + (x,y,psi) block (6, packed)
    double q[N + 1][NZ];      // Newton gradient
    double dz[N + 1][NZ];     // QP iterate
    double ddz[N + 1][NZ];    // QP step
    double pi_nlp[N][NX];
    double piq[N][NX];
    double pin[N][NX];
    double rdyn[N][NX];
    double P[N + 1][15];      // Riccati cost-to-go, packed
    double Lc[N][3];
    double Y[N][NU][NX];
    double Dg[N][C::NH][3];   // signed h-row gradients on (x, y, psi)
    double Msc[28];           // factorisation scratch
    double xinit[NX];
    int flag;
};

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

// box row s (0..13): variable and sign (lower bounds -1, upper +1)
__host__ __device__ constexpr int box_var(int s) { return s < 2 * NU ? (s >> 1) : NU + ((s - 2 * NU) >> 1); }
__host__ __device__ constexpr double box_sign(int s) { return (s & 1) ? 1.0 : -1.0; }

// barrier contribution at (i, j), i >= j: diagonal part dh[0..6] plus the
// (x, y, psi) block dh[7..12] packed xx xy xp yy yp pp
__device__ __forceinline__ double dh_at(const double* dh, int i, int j) {
    double v = (i == j) ? dh[i] : 0.0;
    if (i >= 2 && i <= 4 && j >= 2 && j <= 4) {
        const int a = i - 2, c = j - 2;
        v += dh[NZ + ((c == 0) ? a : (c == 1 ? 2 + a : 5))];
    }
    return v;
}

// Per-lane register state of the inequality rows it owns.
template <class C>
struct Rows {
    double d[C::SLOTS], t[C::SLOTS], l[C::SLOTS], rin[C::SLOTS], pr[C::SLOTS];
    double nlam[C::HSLOTS];  // NLP multiplier of the h row (Hessian weight of the next linearisation)
};

// dispatch a generic lambda on the lane's part as a compile-time constant
template <class C, class Fn>
__device__ __forceinline__ void on_part(int part, Fn&& fn) {
    if (part == 0) fn(std::integral_constant<int, 0>{});
    else if (part == 1) fn(std::integral_constant<int, 1>{});
    else if constexpr (C::PARTS > 2) {
        if (part == 2) fn(std::integral_constant<int, 2>{});
    }
}

// row s of part P is active at stage k
template <class C, int P>
__device__ __forceinline__ bool row_active(int s, int k) {
    if (s < C::nbox(P)) return (k == 0) ? (s < 2 * NU) : (k < C::N);
    return k >= 1 && k < C::N;
}

// h values, signed gradients, bound gaps and the multiplier-weighted Hessian
// (on x, y, psi: xx xy xp yy yp pp) of the h rows [hb(P), he(P)) of stage k.
template <class C, int P>
__device__ __forceinline__ void h_rows(const mpcg_problem& pr, const double* __restrict__ pk, const double z[NZ],
                                       Rows<C>& R, double hb6[6], double (*Dg)[3]) {
    const double x = z[2], y = z[3], psi = z[4];
    const double rdisc = pk[pr.i_disc_r], off = pk[pr.i_disc_off];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double dxp = -off * sp, dyp = off * cp, dxpp = -off * cp, dypp = -off * sp;
#pragma unroll
    for (int hh = C::hb(P); hh < C::he(P); ++hh) {
        constexpr int base = C::nbox(P);
        const int s = base + hh - C::hb(P);
        const int hs = hh - C::hb(P);
        if (hh < C::NL) {
            // topology halfspace a1 x + a2 y - b <= 0 (guidance_constraints.py:355-370)
            const double* c = pk + pr.i_lin0 + 3 * hh;
            const double h = c[0] * x + c[1] * y - c[2];
            R.d[s] = 0.0 - h;
            Dg[hh][0] = c[0];
            Dg[hh][1] = c[1];
            Dg[hh][2] = 0.0;
        } else {
            // obstacle ellipsoid d' R'DR d >= 1 (ellipsoid_constraints.py:435-489)
            const double* o = pk + pr.i_ell0 + 7 * (hh - C::NL);
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
            R.d[s] = h - 1.0;
            Dg[hh][0] = -2.0 * Mdx;
            Dg[hh][1] = -2.0 * Mdy;
            Dg[hh][2] = -2.0 * (Mdx * dxp + Mdy * dyp);
            const double wgt = -R.nlam[hs];  // lower-bound row: Hessian weight -lambda
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

template <class C>
__global__ __launch_bounds__(64, 1) void sqp_kernel(mpcg_problem pr, int batch, const double* __restrict__ params,
                                                 const double* __restrict__ warm, const double* __restrict__ xinit,
                                                 double* __restrict__ xtraj, double* __restrict__ utraj,
                                                 double* __restrict__ pobj_out, int* __restrict__ exit_out,
                                                 int* __restrict__ info_out, unsigned long long* __restrict__ stamps) {
    constexpr int N = C::N, PARTS = C::PARTS;
    __shared__ Lds<C> S;
    const int sol = blockIdx.x;
    if (sol >= batch) return;
    const int lane = threadIdx.x;
    const int k = lane / PARTS;          // my stage
    const int part = lane - k * PARTS;   // my part
    const bool stage_lane = (part == 0) && (k <= N);
    const int kc = k < N ? k : N - 1;    // clamped stage for parameter / F access
    const int npar = pr.npar;
    const double* pbase = params + (size_t)sol * N * npar;
    const double* pk = pbase + (size_t)kc * npar;
    (void)stamps;

    Rows<C> R;
#pragma unroll
    for (int s = 0; s < C::HSLOTS; ++s) R.nlam[s] = 0.0;

    // ---- load warm start (loadWarmstart, acados_solver_interface.cpp:499-509)
    const double* w = warm + (size_t)sol * (N + 1) * NZ;
    for (int e = lane; e < (N + 1) * NZ; e += 64) (&S.z[0][0])[e] = w[e];
    if (lane < NX) S.xinit[lane] = xinit[(size_t)sol * NX + lane];
    for (int e = lane; e < N * NX; e += 64) (&S.pi_nlp[0][0])[e] = 0.0;
    __syncthreads();
    if (lane < NU) S.z[N][lane] = 0.0;
    __syncthreads();

    int acados_status = AC_SUCCESS, qp_status = AC_SUCCESS, sqp_iter = 0, qp_total = 0;
    double res_eq = 0.0;

    for (int it = 0; it < pr.sqp_iters; ++it) {
        // =============== preparation: linearise every stage ===============
        double zk[NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zk[i] = S.z[k <= N ? k : N][i];
        double hb6[6] = {0, 0, 0, 0, 0, 0};
        if (k >= 1 && k < N) {
            on_part<C>(part, [&](auto Pc) {
                constexpr int P = decltype(Pc)::value;
                h_rows<C, P>(pr, pk, zk, R, hb6, S.Dg[k]);
            });
        }
        // fold the h-row Hessian terms of parts 1.. into part 0 (fixed order)
        {
            double acc[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) acc[i] = hb6[i];
#pragma unroll
            for (int p = 1; p < PARTS; ++p)
#pragma unroll
                for (int i = 0; i < 6; ++i) acc[i] += __shfl_down(hb6[i], p);
#pragma unroll
            for (int i = 0; i < 6; ++i) hb6[i] = acc[i];
        }
        double resl = 0.0;
        if (stage_lane && k < N) {
            double g[NZ], H[NZ][NZ], F[NX][NZ], xn[NX], pi[NX];
            stage_cost(pr, pk, zk, g, H, true);
#pragma unroll
            for (int i = 0; i < NX; ++i) pi[i] = S.pi_nlp[k][i];
            erk_unicycle(pr, zk, pi, xn, F, H);
            H[2][2] += hb6[0]; H[2][3] += hb6[1]; H[3][2] += hb6[1];
            H[2][4] += hb6[2]; H[4][2] += hb6[2];
            H[3][3] += hb6[3]; H[3][4] += hb6[4]; H[4][3] += hb6[4];
            H[4][4] += hb6[5];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double bi = xn[i] - S.z[k + 1][NU + i];
                S.b[k][i] = bi;
                resl = fmax(resl, fabs(bi));
#pragma unroll
                for (int j = 0; j < NZ; ++j) S.F[k][i][j] = F[i][j];
            }
            // box rows: input bounds on every stage < N, state bounds on 1..N-1
#pragma unroll
            for (int s = 0; s < NBOX; ++s) {
                const int v = box_var(s);
                const double lo = v < NU ? pr.lbu[v] : pr.lbx[v - NU];
                const double hi = v < NU ? pr.ubu[v] : pr.ubx[v - NU];
                R.d[s] = (s & 1) ? hi - zk[v] : zk[v] - lo;
            }
            mirror7(H, pr.reg_eps);
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                S.g[k][i] = g[i];
#pragma unroll
                for (int j = 0; j <= i; ++j) S.H[k][sym(i, j)] = H[i][j];
            }
        } else if (stage_lane && k == N) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                S.g[N][i] = 0.0;
#pragma unroll
                for (int j = 0; j <= i; ++j) S.H[N][sym(i, j)] = (i == j && i >= NU) ? pr.reg_eps : 0.0;
            }
        }
        res_eq = wave_max(resl);
        if (lane < NX) S.dz[0][NU + lane] = S.xinit[lane] - S.z[0][NU + lane];
        __syncthreads();

        // =============== feedback: QP by Riccati interior point ===============
        // cold start
        on_part<C>(part, [&](auto Pc) {
            constexpr int P = decltype(Pc)::value;
#pragma unroll
            for (int s = 0; s < C::nslot(P); ++s) {
                const double t0 = R.d[s] > pr.qp_thr0 ? R.d[s] : pr.qp_thr0;
                R.t[s] = t0;
                R.l[s] = pr.qp_mu0 / t0;
                R.pr[s] = 0.0;
            }
        });
        if (stage_lane) {
#pragma unroll
            for (int i = 0; i < NZ; ++i)
                if (!(k == 0 && i >= NU)) S.dz[k][i] = 0.0;
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.piq[k][i] = 0.0;
            }
        }
        __syncthreads();
        int qstat = AC_MAXITER, qit = 0;
        double Hdz[NZ];  // part 0: H_k dz_k of the current iterate
        for (;; ++qit) {
            // ---- residuals
            double dzk[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) dzk[i] = S.dz[k <= N ? k : N][i];
            double rs = 0.0, re = 0.0, ri = 0.0, comp = 0.0;
            double rbox[NZ] = {0, 0, 0, 0, 0, 0, 0}, rh[3] = {0, 0, 0};
            if (k <= N) {
                on_part<C>(part, [&](auto Pc) {
                    constexpr int P = decltype(Pc)::value;
#pragma unroll
                    for (int s = 0; s < C::nslot(P); ++s) {
                        if (!row_active<C, P>(s, k)) continue;
                        double dot;
                        if (s < C::nbox(P)) {
                            dot = box_sign(s) * dzk[box_var(s)];
                            rbox[box_var(s)] += box_sign(s) * R.l[s];
                        } else {
                            const int hh = C::hb(P) + s - C::nbox(P);
                            const double a = S.Dg[k][hh][0], bq = S.Dg[k][hh][1], c = S.Dg[k][hh][2];
                            dot = a * dzk[2] + bq * dzk[3] + c * dzk[4];
                            rh[0] += a * R.l[s]; rh[1] += bq * R.l[s]; rh[2] += c * R.l[s];
                        }
                        const double rin = dot + R.t[s] - R.d[s];
                        R.rin[s] = rin;
                        ri = fmax(ri, fabs(rin));
                        comp += R.l[s] * R.t[s];
                    }
                });
            }
            {
                double acc[3] = {rh[0], rh[1], rh[2]};
#pragma unroll
                for (int p = 1; p < PARTS; ++p)
#pragma unroll
                    for (int i = 0; i < 3; ++i) acc[i] += __shfl_down(rh[i], p);
                rbox[2] += acc[0]; rbox[3] += acc[1]; rbox[4] += acc[2];
            }
            if (stage_lane) {
                double r[NZ];
#pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    double acc = 0.0;
#pragma unroll
                    for (int j = 0; j < NZ; ++j) acc += S.H[k][sym(i, j)] * dzk[j];
                    Hdz[i] = acc;
                    r[i] = acc + S.g[k][i] + rbox[i];
                }
                if (k < N) {
#pragma unroll
                    for (int m = 0; m < NX; ++m) {
                        const double pm = S.piq[k][m];
#pragma unroll
                        for (int i = 0; i < NZ; ++i) r[i] += S.F[k][m][i] * pm;
                    }
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        double acc = S.b[k][i] - S.dz[k + 1][NU + i];
#pragma unroll
                        for (int j = 0; j < NZ; ++j) acc += S.F[k][i][j] * dzk[j];
                        S.rdyn[k][i] = acc;
                        re = fmax(re, fabs(acc));
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
            rs = wave_max(rs);
            re = wave_max(re);
            ri = wave_max(ri);
            comp = wave_sum(comp);
            const double mu = comp / C::M_TOTAL;
            if (!(rs < 1e30) || !(re < 1e30) || !(ri < 1e30) || !(mu < 1e16)) { qstat = AC_NAN; break; }
            if (rs < pr.qp_tol && re < pr.qp_tol && ri < pr.qp_tol && mu < pr.qp_tol) { qstat = AC_SUCCESS; break; }
            if (qit >= pr.qp_iter_max) { qstat = AC_MAXITER; break; }
            __syncthreads();

            double alpha = 1.0, sigma_mu = 0.0;
            for (int phase = 0; phase < 2; ++phase) {
                // ---- barrier terms + Newton gradient
                {
                    double qb[NZ] = {0, 0, 0, 0, 0, 0, 0}, dd[NZ] = {0, 0, 0, 0, 0, 0, 0};
                    double qh[3] = {0, 0, 0}, dbh[6] = {0, 0, 0, 0, 0, 0};
                    if (k <= N) {
                        on_part<C>(part, [&](auto Pc) {
                            constexpr int P = decltype(Pc)::value;
#pragma unroll
                            for (int s = 0; s < C::nslot(P); ++s) {
                                if (!row_active<C, P>(s, k)) continue;
                                const double l = R.l[s], t = R.t[s];
                                const double rc = (phase == 0) ? l * t : l * t + R.pr[s] - sigma_mu;
                                const double coef = l + (l * R.rin[s] - rc) / t;
                                const double wgt = l / t;
                                if (s < C::nbox(P)) {
                                    qb[box_var(s)] += box_sign(s) * coef;
                                    dd[box_var(s)] += wgt;
                                } else {
                                    const int hh = C::hb(P) + s - C::nbox(P);
                                    const double a = S.Dg[k][hh][0], bq = S.Dg[k][hh][1], c = S.Dg[k][hh][2];
                                    qh[0] += a * coef; qh[1] += bq * coef; qh[2] += c * coef;
                                    dbh[0] += a * wgt * a; dbh[1] += a * wgt * bq; dbh[2] += a * wgt * c;
                                    dbh[3] += bq * wgt * bq; dbh[4] += bq * wgt * c; dbh[5] += c * wgt * c;
                                }
                            }
                        });
                    }
                    double aq[3] = {qh[0], qh[1], qh[2]}, ab[6];
#pragma unroll
                    for (int i = 0; i < 6; ++i) ab[i] = dbh[i];
#pragma unroll
                    for (int p = 1; p < PARTS; ++p) {
#pragma unroll
                        for (int i = 0; i < 3; ++i) aq[i] += __shfl_down(qh[i], p);
                        if (phase == 0) {
#pragma unroll
                            for (int i = 0; i < 6; ++i) ab[i] += __shfl_down(dbh[i], p);
                        }
                    }
                    if (stage_lane) {
#pragma unroll
                        for (int i = 0; i < NZ; ++i) S.q[k][i] = Hdz[i] + S.g[k][i] + qb[i];
                        S.q[k][2] += aq[0]; S.q[k][3] += aq[1]; S.q[k][4] += aq[2];
                        if (phase == 0) {
#pragma unroll
                            for (int i = 0; i < NZ; ++i) S.dH[k][i] = dd[i];
#pragma unroll
                            for (int i = 0; i < 6; ++i) S.dH[k][NZ + i] = ab[i];
                        }
                    }
                }
                __syncthreads();
                // ---- Riccati factorisation (predictor only; the corrector reuses it)
                if (phase == 0) {
                    if (lane < 15) {
                        int i = 0;
                        while ((i + 1) * (i + 2) / 2 <= lane) ++i;
                        const int j = lane - i * (i + 1) / 2;
                        S.P[N][lane] = S.H[N][sym(NU + i, NU + j)] + dh_at(S.dH[N], NU + i, NU + j);
                    }
                    if (lane == 0) S.flag = 0;
                    // element lane -> (ei, ej), ei >= ej, of the 7x7 block
                    int ei = 0;
                    if (lane < 28) {
                        while ((ei + 1) * (ei + 2) / 2 <= lane) ++ei;
                    }
                    const int ej = lane < 28 ? lane - ei * (ei + 1) / 2 : 0;
                    // barrier terms of entry (ei, ej): diagonal part and (x,y,psi) block part
                    const int dhd = (ei == ej) ? ei : -1;
                    int dhb = -1;
                    if (ei >= 2 && ei <= 4 && ej >= 2 && ej <= 4) {
                        const int a = ei - 2, c = ej - 2;
                        dhb = NZ + ((c == 0) ? a : (c == 1 ? 2 + a : 5));
                    }
                    __syncthreads();
                    for (int kk = N - 1; kk >= 0; --kk) {
                        if (lane < 28) {
                            double Pm[15];
#pragma unroll
                            for (int e = 0; e < 15; ++e) Pm[e] = S.P[kk + 1][e];
                            double fi[NX], fj[NX];
#pragma unroll
                            for (int m = 0; m < NX; ++m) { fi[m] = S.F[kk][m][ei]; fj[m] = S.F[kk][m][ej]; }
                            double v = S.H[kk][lane] + (dhd >= 0 ? S.dH[kk][dhd] : 0.0) + (dhb >= 0 ? S.dH[kk][dhb] : 0.0);
#pragma unroll
                            for (int m = 0; m < NX; ++m) {
                                double tm = 0.0;
#pragma unroll
                                for (int l = 0; l < NX; ++l) tm += Pm[sym(m, l)] * fj[l];
                                v += fi[m] * tm;
                            }
                            S.Msc[lane] = v;
                        }
                        __syncthreads();
                        if (lane < 15) {
                            int i = 0;
                            while ((i + 1) * (i + 2) / 2 <= lane) ++i;
                            const int j = lane - i * (i + 1) / 2;
                            const double m00 = S.Msc[0], m10 = S.Msc[1], m11 = S.Msc[2];
                            const double l00 = sqrt(m00);
                            const double l10 = m10 / l00;
                            const double r11 = m11 - l10 * l10;
                            const double l11 = sqrt(r11);
                            if (!(m00 > 0.0) || !(r11 > 0.0)) S.flag = 1;
                            const double y0i = S.Msc[sym(NU + i, 0)] / l00;
                            const double y1i = (S.Msc[sym(NU + i, 1)] - l10 * y0i) / l11;
                            const double y0j = S.Msc[sym(NU + j, 0)] / l00;
                            const double y1j = (S.Msc[sym(NU + j, 1)] - l10 * y0j) / l11;
                            S.P[kk][lane] = S.Msc[sym(NU + i, NU + j)] - y0i * y0j - y1i * y1j;
                            if (j == 0) { S.Y[kk][0][i] = y0i; S.Y[kk][1][i] = y1i; }
                            if (lane == 0) { S.Lc[kk][0] = l00; S.Lc[kk][1] = l10; S.Lc[kk][2] = l11; }
                        }
                        __syncthreads();
                    }
                    if (S.flag) { qstat = AC_NAN; break; }
                }
                // ---- vector + forward passes: affine 5-vector recursions in SGPRs
                {
                    const bool own = stage_lane && k < N;
                    const int kq = own ? k : 0;
                    double Fl[NX][NZ], P1[15], G[NX][NX], hv[NX], W0[NX], W1[NX], Y0[NX], Y1[NX], rr[NX];
                    const double l00 = S.Lc[kq][0], l10 = S.Lc[kq][1], l11 = S.Lc[kq][2];
                    double y0a, y0b;
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        rr[i] = S.rdyn[kq][i];
                        Y0[i] = S.Y[kq][0][i];
                        Y1[i] = S.Y[kq][1][i];
#pragma unroll
                        for (int j = 0; j < NZ; ++j) Fl[i][j] = S.F[kq][i][j];
                    }
#pragma unroll
                    for (int e = 0; e < 15; ++e) P1[e] = S.P[kq + 1][e];
                    {
                        double c[NX], m0[NZ];
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            double acc = 0.0;
#pragma unroll
                            for (int j = 0; j < NX; ++j) acc += P1[sym(i, j)] * rr[j];
                            c[i] = acc;
                        }
#pragma unroll
                        for (int i = 0; i < NZ; ++i) {
                            double acc = S.q[kq][i];
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
                        const bool mine = (k == kk) && (part == 0);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            pmine[i] = mine ? pu[i] : pmine[i];
                            pu[i] = readlane_d(pn[i], kk * PARTS);
                        }
                    }
                    const double ya = y0a + W0[0] * pmine[0] + W0[1] * pmine[1] + W0[2] * pmine[2] + W0[3] * pmine[3] +
                                      W0[4] * pmine[4];
                    const double yb = y0b + W1[0] * pmine[0] + W1[1] * pmine[1] + W1[2] * pmine[2] + W1[3] * pmine[3] +
                                      W1[4] * pmine[4];
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
                        for (int j = 0; j < NX; ++j) G[i][j] = Fl[i][NU + j] + Fl[i][0] * K0[j] + Fl[i][1] * K1[j];
                    }
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
                        const bool mine = (k == kk) && (part == 0);
#pragma unroll
                        for (int i = 0; i < NX; ++i) {
                            dxmine[i] = mine ? dxu[i] : dxmine[i];
                            dxu[i] = readlane_d(dn[i], kk * PARTS);
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
                            for (int j = 0; j < NX; ++j) acc += P1[sym(i, j)] * dxn[j];
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
                // ---- inequality steps and step length (dt, dl recomputed where needed)
                double amax = 1e300;
                double ddk[NZ];
#pragma unroll
                for (int i = 0; i < NZ; ++i) ddk[i] = S.ddz[k < N ? k : N][i];
                const double smu = sigma_mu;
                const int ph = phase;
                auto row_step = [&](auto Pc, int s, double& dt, double& dl) {
                    constexpr int P = decltype(Pc)::value;
                    double dot;
                    if (s < C::nbox(P)) {
                        dot = box_sign(s) * ddk[box_var(s)];
                    } else {
                        const int hh = C::hb(P) + s - C::nbox(P);
                        dot = S.Dg[k][hh][0] * ddk[2] + S.Dg[k][hh][1] * ddk[3] + S.Dg[k][hh][2] * ddk[4];
                    }
                    const double l = R.l[s], t = R.t[s];
                    const double rc = (ph == 0) ? l * t : l * t + R.pr[s] - smu;
                    dt = -R.rin[s] - dot;
                    dl = -(rc + l * dt) / t;
                };
                if (k < N) {
                    on_part<C>(part, [&](auto Pc) {
                        constexpr int P = decltype(Pc)::value;
#pragma unroll
                        for (int s = 0; s < C::nslot(P); ++s) {
                            if (!row_active<C, P>(s, k)) continue;
                            double dt, dl;
                            row_step(Pc, s, dt, dl);
                            if (dt < 0.0) amax = fmin(amax, -R.t[s] / dt);
                            if (dl < 0.0) amax = fmin(amax, -R.l[s] / dl);
                        }
                    });
                }
                amax = wave_min(amax);
                if (phase == 0) {
                    const double aa = fmin(amax, 1.0);
                    double ca = 0.0;
                    if (k < N) {
                        on_part<C>(part, [&](auto Pc) {
                            constexpr int P = decltype(Pc)::value;
#pragma unroll
                            for (int s = 0; s < C::nslot(P); ++s) {
                                if (!row_active<C, P>(s, k)) continue;
                                double dt, dl;
                                row_step(Pc, s, dt, dl);
                                ca += (R.l[s] + aa * dl) * (R.t[s] + aa * dt);
                                R.pr[s] = dt * dl;
                            }
                        });
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
                    if (alpha >= 1e-12 && k < N) {
                        // row update with the corrector step (before dz moves: rin and
                        // ddz belong to the current iterate)
                        on_part<C>(part, [&](auto Pc) {
                            constexpr int P = decltype(Pc)::value;
#pragma unroll
                            for (int s = 0; s < C::nslot(P); ++s) {
                                if (!row_active<C, P>(s, k)) continue;
                                double dt, dl;
                                row_step(Pc, s, dt, dl);
                                R.t[s] += alpha * dt;
                                R.l[s] += alpha * dl;
                            }
                        });
                    }
                }
                __syncthreads();
            }
            if (qstat == AC_NAN) break;
            if (alpha < 1e-12) { qstat = AC_MINSTEP; ++qit; break; }
            // ---- update of the stage variables (rows were updated with the step)
            if (stage_lane) {
#pragma unroll
                for (int i = 0; i < NZ; ++i) S.dz[k][i] += alpha * S.ddz[k][i];
                if (k < N) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) S.piq[k][i] += alpha * (S.pin[k][i] - S.piq[k][i]);
                }
            }
            __syncthreads();
        }
        __syncthreads();
        qp_status = qstat;
        qp_total += qit;
        ++sqp_iter;
        if (qstat != AC_SUCCESS && qstat != AC_MAXITER) {
            acados_status = AC_QP_FAILURE;
            break;
        }
        // FIXED_STEP full step on the primal iterate and on every multiplier
        if (stage_lane) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) S.z[k][i] += S.dz[k][i];
            if (k == N) { S.z[N][0] = 0.0; S.z[N][1] = 0.0; }
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; ++i) S.pi_nlp[k][i] = S.piq[k][i];
            }
        }
        if (k >= 1 && k < N) {
            on_part<C>(part, [&](auto Pc) {
                constexpr int P = decltype(Pc)::value;
#pragma unroll
                for (int s = C::nbox(P); s < C::nslot(P); ++s) R.nlam[s - C::nbox(P)] = R.l[s];
            });
        }
        __syncthreads();
        acados_status = AC_SUCCESS;
        if (qstat != AC_SUCCESS) break;
    }

    // ---- completeOneIteration (acados_solver_interface.cpp:387-429)
    double Lk = 0.0;
    if (stage_lane && k < N) {
        double zz[NZ], gd[NZ], Hd[NZ][NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zz[i] = S.z[k][i];
        Lk = stage_cost(pr, pk, zz, gd, Hd, false);
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
}

}  // namespace mpcg
