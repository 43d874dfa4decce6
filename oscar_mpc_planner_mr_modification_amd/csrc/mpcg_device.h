// mpcg_device.h — per-stage device functions of the T-MPC++ SQP backend
// (gfx950, fp64 VALU).  One lane evaluates one shooting stage.
//
// Reference semantics (paths relative to the reference repo):
//   stage cost   solver_definition.py:19-34 over mpc_base.py:47-60,
//                contouring.py:140-174 (stage_idx=1), consistency_module.py:229-250,
//                glued spline spline.py:28-86
//   constraints  guidance_constraints.py:355-370 then ellipsoid_constraints.py:435-489
//   slack model  solver_model.py:274-298 (slack state last, constant in time),
//                its MPCBase weight slack^2 (generate_jackalsimulator_solver.py:69-89)
//   dynamics     solver_model.py:207-214 integrated by acados ERK (4 stages,
//                3 steps) with exact first/second-order sensitivities
//                (generate_acados_solver.py:148-157)
//   MIRROR       regularize_method "MIRROR" (generate_acados_solver.py:157)
#pragma once
#include <hip/hip_runtime.h>

#include "mpcg.h"

namespace mpcg {

constexpr int NU = MPCG_NU;

// ---------------------------------------------------------------------------
// fp64 reciprocal / reciprocal square root: the hardware estimate
// (v_rcp_f64 / v_rsq_f64) refined by two Newton steps, within an ulp of the
// correctly rounded result at a third of the latency of the IEEE division /
// square-root expansions.  Arguments are finite and non-zero (positive for
// frsq) wherever they are used.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double frcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

__device__ __forceinline__ double frsq(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    return y * fma(-h * y, y, 1.5);
}

// sqrt for x > 0
__device__ __forceinline__ double fsqrt_pos(double x) { return x * frsq(x); }

// ---------------------------------------------------------------------------
// sin and cos of one argument: quadrant n = rint(2x / pi), r = x - n pi/2 by two
// fused steps (pi/2 as a double pair), then the fdlibm kernel polynomials on
// [-pi/4, pi/4].  Within ~1 ulp of the correctly rounded values for
// |x| < 2^20 pi/2 (the angles of this path are headings and steering angles of
// order one); beyond that the reduction error grows with n.  Unlike the ROCm
// device library's sincos it has no large-argument (Payne-Hanek) branch, whose
// registers the linearisation lane otherwise reserves through its jets (the
// bicycle instance spilled on it).  __host__ too: tests/test_device_math checks
// it against the C library on the host.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ void fsincos(double x, double* s, double* c) {
    const double n = rint(x * 0x1.45f306dc9c883p-1);     // 2 / pi
    double r = fma(-n, 0x1.921fb54442d18p+0, x);           // pi/2, leading double
    r = fma(-n, 0x1.1a62633145c07p-54, r);                 // pi/2 - leading double
    r = n == 0.0 ? x : r;
    const double z = r * r;
    // __kernel_sin: r + r^3 (S1 + z (S2 + ... S6))
    const double ps = 0x1.111111110f8a6p-7 + z * (-0x1.a01a019c161d5p-13 + z * (0x1.71de357b1fe7dp-19 +
                      z * (-0x1.ae5e68a2b9cebp-26 + z * 0x1.5d93a5acfd57cp-33)));
    double sr = r + (r * z) * (-0x1.5555555555549p-3 + z * ps);
    sr = fabs(r) < 0x1p-27 ? r : sr;                       // sin r = r there (and sin(-0) = -0)
    // __kernel_cos: w + (((1 - w) - z/2) + z^2 (C1 + z (C2 + ... C6))), w = 1 - z/2
    const double pc = 0x1.555555555554cp-5 + z * (-0x1.6c16c16c15177p-10 + z * (0x1.a01a019cb159p-16 +
                      z * (-0x1.27e4f809c52adp-22 + z * (0x1.1ee9ebdb4b1c4p-29 + z * -0x1.8fae9be8838d4p-37))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + (z * z) * pc);
    const long q = (long)n & 3;
    const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}

// atan and atan2 after fdlibm's s_atan / e_atan2: |x| reduced to one of the intervals
// around 0, 1/2, 1, 3/2, infinity (one quotient, through the reciprocal), the odd
// polynomial, the interval's atan as a double pair; quadrants and special values by
// selects, no branches.  Within ~2 ulp of the C library (tests/test_device_math).
template <class RCP>
__host__ __device__ __forceinline__ double fatan_abs(double ax, RCP rcp) {
    // ax = |x| (may be +inf)
    const int id = ax < 0.4375 ? -1 : (ax < 0.6875 ? 0 : (ax < 1.1875 ? 1 : (ax < 2.4375 ? 2 : 3)));
    const double num = id == 0 ? 2.0 * ax - 1.0 : (id == 1 ? ax - 1.0 : (id == 2 ? ax - 1.5 : -1.0));
    const double den = id == 0 ? 2.0 + ax : (id == 1 ? ax + 1.0 : (id == 2 ? 1.0 + 1.5 * ax : ax));
    double x = id < 0 ? ax : num * rcp(den);
    x = (id == 3 && !(ax < 0x1p66)) ? -0.0 : x;  // atan(huge or inf) = pi/2
    const double z = x * x, w = z * z;
    const double s1 = z * (0.333333333333329318027 + w * (0.142857142725034663711 + w * (0.0909088713343650656196 +
                      w * (0.0666107313738753120669 + w * (0.0497687799461593236017 + w * 0.0162858201153657823623)))));
    const double s2 = w * (-0.199999999998764832476 + w * (-0.111111104054623557880 + w * (-0.0769187620504482999495 +
                      w * (-0.0583357013379057348645 + w * -0.0365315727442169155270))));
    const double hi = id == 0 ? 4.63647609000806093515e-01 : (id == 1 ? 7.85398163397448278999e-01 :
                      (id == 2 ? 9.82793723247329054082e-01 : 1.57079632679489655800e+00));
    const double lo = id == 0 ? 2.26987774529616870924e-17 : (id == 1 ? 3.06161699786838301793e-17 :
                      (id == 2 ? 1.39033110312309984516e-17 : 6.12323399573676603587e-17));
    return id < 0 ? x - x * (s1 + s2) : hi - ((x * (s1 + s2) - lo) - x);
}
// the reciprocal of the quotient: frcp on the device (FRcp), the division on the host (tests)
struct FRcp {
    __device__ double operator()(double d) const { return frcp(d); }
};
template <class RCP>
__host__ __device__ __forceinline__ double fatan(double x, RCP rcp) {
    const double a = fatan_abs(fabs(x), rcp);
    return x < 0.0 ? -a : (x == 0.0 ? x : a);
}
// atan2(y, x) for finite arguments, not both zero
template <class RCP>
__host__ __device__ __forceinline__ double fatan2(double y, double x, RCP rcp) {
    const double ax = fabs(x), ay = fabs(y);
    const double z = fatan_abs(ax == 0.0 ? INFINITY : ay * rcp(ax), rcp);  // atan |y / x|
    constexpr double PI = 3.1415926535897931160e+00, PI_LO = 1.2246467991473531772e-16;
    const double r = (__builtin_signbit(x) && ax != 0.0) ? PI - (z - PI_LO) : z;
    return __builtin_signbit(y) ? -r : r;
}

// tan through fsincos (within ~3 ulp; cos(x) != 0 for the steering angles it is used on)
__device__ __forceinline__ double ftan(double x) {
    double s, c;
    fsincos(x, &s, &c);
    return s * frcp(c);
}

// ---------------------------------------------------------------------------
// glued spline of spline.py:39-58: for both axes the glued position G and the
// glued segment-derivative D, each with first and second s-derivatives.
// ---------------------------------------------------------------------------
struct SplineJets {
    double Gx[3], Gy[3], Dx[3], Dy[3];
};

__device__ __forceinline__ void seg_jets(const double* __restrict__ c, double t, double P[4]) {
    // c = (a, b, c, d); P = (P, P', P'', P''')
    double a = c[0], b = c[1], cc = c[2], d = c[3];
    P[0] = ((a * t + b) * t + cc) * t + d;
    P[1] = (3.0 * a * t + 2.0 * b) * t + cc;
    P[2] = 6.0 * a * t + 2.0 * b;
    P[3] = 6.0 * a;
}

__device__ inline void spline_jets(const mpcg_problem& pr, const double* __restrict__ p, double s,
                                   SplineJets& J) {
    const int M = pr.n_seg;
    const double* base = p + pr.i_spline0;
    double Px[4], Py[4];
    {
        const double* seg = base + 9 * (M - 1);
        double t = s - seg[8];
        seg_jets(seg, t, Px);
        seg_jets(seg + 4, t, Py);
    }
    double Vx[3] = {Px[0], Px[1], Px[2]}, Wx[3] = {Px[1], Px[2], Px[3]};
    double Vy[3] = {Py[0], Py[1], Py[2]}, Wy[3] = {Py[1], Py[2], Py[3]};
    for (int k = M - 1; k >= 1; --k) {
        // lambda_k uses the start of segment k (spline.py:37)
        const double sk = base[9 * k + 8];
        const double e = exp((s - sk + 0.02) / 0.1);
        const double l0 = e < 0x1p1000 ? frcp(1.0 + e) : 0.0;  // 1 / (1 + inf) = 0, as the oracle
        const double l1 = -10.0 * l0 * (1.0 - l0);
        const double l2 = 100.0 * l0 * (1.0 - l0) * (1.0 - 2.0 * l0);
        const double* seg = base + 9 * (k - 1);
        const double t = s - seg[8];
        seg_jets(seg, t, Px);
        seg_jets(seg + 4, t, Py);
        const double m0 = 1.0 - l0;
        // glued value and its derivatives
        double a0 = Px[0] - Vx[0], a1 = Px[1] - Vx[1];
        Vx[2] = l2 * a0 + 2.0 * l1 * a1 + l0 * Px[2] + m0 * Vx[2];
        Vx[1] = l1 * a0 + l0 * Px[1] + m0 * Vx[1];
        Vx[0] = l0 * Px[0] + m0 * Vx[0];
        a0 = Py[0] - Vy[0]; a1 = Py[1] - Vy[1];
        Vy[2] = l2 * a0 + 2.0 * l1 * a1 + l0 * Py[2] + m0 * Vy[2];
        Vy[1] = l1 * a0 + l0 * Py[1] + m0 * Vy[1];
        Vy[0] = l0 * Py[0] + m0 * Vy[0];
        // glued segment derivative and its derivatives
        a0 = Px[1] - Wx[0]; a1 = Px[2] - Wx[1];
        Wx[2] = l2 * a0 + 2.0 * l1 * a1 + l0 * Px[3] + m0 * Wx[2];
        Wx[1] = l1 * a0 + l0 * Px[2] + m0 * Wx[1];
        Wx[0] = l0 * Px[1] + m0 * Wx[0];
        a0 = Py[1] - Wy[0]; a1 = Py[2] - Wy[1];
        Wy[2] = l2 * a0 + 2.0 * l1 * a1 + l0 * Py[3] + m0 * Wy[2];
        Wy[1] = l1 * a0 + l0 * Py[2] + m0 * Wy[1];
        Wy[0] = l0 * Py[1] + m0 * Wy[0];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        J.Gx[i] = Vx[i]; J.Gy[i] = Vy[i]; J.Dx[i] = Wx[i]; J.Dy[i] = Wy[i];
    }
}

// ---------------------------------------------------------------------------
// stage cost L(z; p), gradient and Hessian (z = [a, w, x, y, psi, v, s (, slack)])
// ---------------------------------------------------------------------------
template <int NX>
__device__ inline double stage_cost(const mpcg_problem& pr, const double* __restrict__ p,
                                    const double z[NU + NX], double g[NU + NX], double H[NU + NX][NU + NX],
                                    bool derivs) {
    constexpr int NZ = NU + NX;
    const double a = z[0], w = z[1], x = z[2], y = z[3], v = z[5], s = z[6];
    const double wa = p[pr.i_w_acc], ww = p[pr.i_w_ang], wv = p[pr.i_w_vel], vref = p[pr.i_v_ref];
    const double wc = p[pr.i_w_contour], wl = p[pr.i_w_lag];
    double L = wa * a * a + ww * w * w + wv * (v - vref) * (v - vref);
    SplineJets J;
    spline_jets(pr, p, s, J);
    const double rsq = J.Dx[0] * J.Dx[0] + J.Dy[0] * J.Dy[0];
    const double ir = frsq(rsq);
    const double tx = J.Dx[0] * ir, ty = J.Dy[0] * ir;
    const double ex = x - J.Gx[0], ey = y - J.Gy[0];
    const double ec = ty * ex - tx * ey;  // contour error (contouring.py:166)
    const double el = tx * ex + ty * ey;  // lag error (contouring.py:167)
    L += wl * el * el + wc * ec * ec;
    double wcn = 0.0, dxp = 0.0, dyp = 0.0;
    if (pr.i_cons_w >= 0) {
        wcn = p[pr.i_cons_w];
        dxp = x - p[pr.i_prev_x];
        dyp = y - p[pr.i_prev_y];
        L += wcn * (dxp * dxp + dyp * dyp);
    }
    double wsl = 0.0, sl = 0.0;
    if constexpr (NX > 5) {
        wsl = p[pr.i_w_slack];
        sl = z[NU + 5];
        L += wsl * sl * sl;
    }
    if (!derivs) return L;
    const double r1 = tx * J.Dx[1] + ty * J.Dy[1];
    const double tx1 = (J.Dx[1] - tx * r1) * ir, ty1 = (J.Dy[1] - ty * r1) * ir;
    const double r2 = tx1 * J.Dx[1] + ty1 * J.Dy[1] + tx * J.Dx[2] + ty * J.Dy[2];
    const double tx2 = (J.Dx[2] - 2.0 * tx1 * r1 - tx * r2) * ir;
    const double ty2 = (J.Dy[2] - 2.0 * ty1 * r1 - ty * r2) * ir;
    const double Gx1 = J.Gx[1], Gy1 = J.Gy[1], Gx2 = J.Gx[2], Gy2 = J.Gy[2];
    // d(e)/d(x, y, s) and the s-row of the second derivatives
    const double dc[3] = {ty, -tx, ty1 * ex - tx1 * ey - ty * Gx1 + tx * Gy1};
    const double dl[3] = {tx, ty, tx1 * ex + ty1 * ey - tx * Gx1 - ty * Gy1};
    const double hc_s[3] = {ty1, -tx1, ty2 * ex - tx2 * ey - 2.0 * ty1 * Gx1 + 2.0 * tx1 * Gy1 - ty * Gx2 + tx * Gy2};
    const double hl_s[3] = {tx1, ty1, tx2 * ex + ty2 * ey - 2.0 * tx1 * Gx1 - 2.0 * ty1 * Gy1 - tx * Gx2 - ty * Gy2};
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        g[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NZ; ++j) H[i][j] = 0.0;
    }
    g[0] = 2.0 * wa * a; H[0][0] = 2.0 * wa;
    g[1] = 2.0 * ww * w; H[1][1] = 2.0 * ww;
    g[5] = 2.0 * wv * (v - vref); H[5][5] = 2.0 * wv;
    constexpr int ids[3] = {2, 3, 6};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        g[ids[i]] += 2.0 * (wl * el * dl[i] + wc * ec * dc[i]);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            // second derivatives of e vanish on the (x,y)x(x,y) block
            double hl = (i == 2) ? hl_s[j] : ((j == 2) ? hl_s[i] : 0.0);
            double hc = (i == 2) ? hc_s[j] : ((j == 2) ? hc_s[i] : 0.0);
            H[ids[i]][ids[j]] += 2.0 * (wl * (dl[i] * dl[j] + el * hl) + wc * (dc[i] * dc[j] + ec * hc));
        }
    }
    if (pr.i_cons_w >= 0) {
        g[2] += 2.0 * wcn * dxp; g[3] += 2.0 * wcn * dyp;
        H[2][2] += 2.0 * wcn; H[3][3] += 2.0 * wcn;
    }
    if constexpr (NX > 5) {
        g[NU + 5] = 2.0 * wsl * sl;
        H[NU + 5][NU + 5] = 2.0 * wsl;
    }
    return L;
}

// ---------------------------------------------------------------------------
// acados ERK4 (rk_steps steps over dt) of the contouring unicycle
// x' = (v cos psi, v sin psi, w, a, v).  psi and v are affine in time inside
// a shooting interval (psi_e = psi + tau_e w, v_e = v + tau_e a at every RK
// stage argument), so the discrete map is exactly
//   x+ = x + sum_e h b_e v_e cos(psi_e), y+ likewise with sin, s+ = s + sum_e h b_e v_e,
//   psi+ = psi + dt w, v+ = v + dt a,
// and its exact Jacobian / second-order adjoint follow in closed form.
// Outputs F = [B A] (nx x nz), xn, and (if pi != nullptr) H += Hess(pi' x+).
// The slack state (nx 6) has zero dynamics: x+ = slack, a unit row.
// ---------------------------------------------------------------------------
// Coefficients of a and v in the s+ row of the ERK4 map (s' = v, v' = a): RK4 integrates the
// quadratic s(t) = s + v t + a t^2 / 2 exactly, so they are dt^2 / 2 and dt; the kernel uses them
// for the [B A] rows it does not store, and erk_unicycle writes the same values.
__device__ __forceinline__ void erk_srow(const mpcg_problem& pr, double& sa, double& sv) {
    sa = 0.5 * pr.dt * pr.dt;
    sv = pr.dt;
}

template <int NX>
__device__ inline void erk_unicycle(const mpcg_problem& pr, const double z[NU + NX], const double* pi,
                                    double xn[NX], double F[NX][NU + NX], double H[NU + NX][NU + NX]) {
    constexpr int NZ = NU + NX;
    const double a = z[0], w = z[1], psi = z[4], v = z[5];
    const int ns = pr.rk_steps;
    const double h = pr.dt / ns;
    // c_q = (0, 1/2, 1/2, 1), b_q = (1, 2, 2, 1)/6
    double sx = 0.0, sy = 0.0, ss = 0.0;
    // d/d(a, w, psi, v) of sum b v_e cos, sum b v_e sin, sum b v_e
    double jx[4] = {0, 0, 0, 0}, jy[4] = {0, 0, 0, 0}, js[4] = {0, 0, 0, 0};
    // Hessian accumulators over (a, w, psi, v)
    double hq[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) hq[i][j] = 0.0;
    const double pix = pi ? pi[0] : 0.0, piy = pi ? pi[1] : 0.0;
    double cpsi, spsi;
    sincos(psi, &spsi, &cpsi);
    for (int st = 0; st < ns; ++st) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double cq = (q == 0) ? 0.0 : ((q == 3) ? 1.0 : 0.5);
            const double bq = ((q == 0 || q == 3) ? 1.0 : 2.0) * h / 6.0;
            const double tau = (st + cq) * h;
            double sw, cw;
            sincos(tau * w, &sw, &cw);
            const double ce = cpsi * cw - spsi * sw;  // cos(psi + tau w)
            const double se = spsi * cw + cpsi * sw;  // sin(psi + tau w)
            const double ve = v + tau * a;
            sx += bq * ve * ce;
            sy += bq * ve * se;
            ss += bq * ve;
            // d psi_e = (0, tau, 1, 0), d v_e = (tau, 0, 0, 1) over (a, w, psi, v)
            const double dcx_p = -ve * se, dcx_v = ce;   // d(v cos)/d(psi_e, v_e)
            const double dcy_p = ve * ce, dcy_v = se;    // d(v sin)/d(psi_e, v_e)
            jx[0] += bq * dcx_v * tau; jx[1] += bq * dcx_p * tau; jx[2] += bq * dcx_p; jx[3] += bq * dcx_v;
            jy[0] += bq * dcy_v * tau; jy[1] += bq * dcy_p * tau; jy[2] += bq * dcy_p; jy[3] += bq * dcy_v;
            if (pi) {
                // second derivatives of pix v cos + piy v sin in (psi_e, v_e)
                const double hpp = bq * (-pix * ve * ce - piy * ve * se);
                const double hpv = bq * (-pix * se + piy * ce);
                const double rp[4] = {0.0, tau, 1.0, 0.0};
                const double rv[4] = {tau, 0.0, 0.0, 1.0};
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        hq[i][j] += hpp * rp[i] * rp[j] + hpv * (rp[i] * rv[j] + rv[i] * rp[j]);
            }
        }
    }
    erk_srow(pr, js[0], js[3]);
    const double T = pr.dt;
    xn[0] = z[2] + sx;
    xn[1] = z[3] + sy;
    xn[2] = psi + T * w;
    xn[3] = v + T * a;
    xn[4] = z[6] + ss;
    // F = d x+ / d z, z = [a, w, x, y, psi, v, s]
#pragma unroll
    for (int i = 0; i < NX; ++i)
#pragma unroll
        for (int j = 0; j < NZ; ++j) F[i][j] = 0.0;
    constexpr int zi[4] = {0, 1, 4, 5};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        F[0][zi[j]] = jx[j];
        F[1][zi[j]] = jy[j];
        F[4][zi[j]] = js[j];
    }
    F[0][2] = 1.0; F[1][3] = 1.0; F[4][6] = 1.0;
    F[2][1] = T; F[2][4] = 1.0;
    F[3][0] = T; F[3][5] = 1.0;
#pragma unroll
    for (int i = 5; i < NX; ++i) {
        xn[i] = z[NU + i];
        F[i][NU + i] = 1.0;
    }
    if (pi) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) H[zi[i]][zi[j]] += hq[i][j];
    }
}

// ---------------------------------------------------------------------------
// MIRROR: H <- V f(D) V', f(d) = eps if |d| <= eps else |d|, cyclic Jacobi
// on the nz x nz stage block.  Rotations on exactly-zero couplings are skipped,
// so decoupled sub-blocks (e.g. {a,w,psi,v} vs {x,y,s} with a zero disc
// offset) cost only their own rotations.
// ---------------------------------------------------------------------------
// dia_extra: squared diagonal of a decoupled block handled outside (it enters
// the convergence test exactly as in the full-size sweep)
// NA: the leading NA x NA block of the NZ x NZ array is mirrored in place
// (NA < NZ: the trailing rows / columns are decoupled and handled by the caller)
// MPCG_MIRROR_RR=1: the round-robin (parallel) Jacobi ordering below, A/B only -- measured slower
// (profiles/r03q_ab.jsonl: C2 11.97 -> 12.04 ms, C1 +1.6 %, C5 +1.3 %, JS +1.2 %; C4 -1.0 %) and its
// different rounding moved one C5 copy of 8,192 to another exit (1602: QP failure in the oracle,
// success on the GPU; profiles/r03q_rr_fullsize.log)
#ifndef MPCG_MIRROR_RR
#define MPCG_MIRROR_RR 0
#endif
// round-robin schedule of n (even) players: pair i of round r (players n - 1 and r, then
// (r + i, r - i) mod n - 1), lower / higher index
__host__ __device__ constexpr int rr_a(int n, int r, int i) { return i == 0 ? n - 1 : (r + i) % (n - 1); }
__host__ __device__ constexpr int rr_b(int n, int r, int i) { return i == 0 ? r : (r - i + n - 1) % (n - 1); }
__host__ __device__ constexpr int rr_lo(int n, int r, int i) { return rr_a(n, r, i) < rr_b(n, r, i) ? rr_a(n, r, i) : rr_b(n, r, i); }
__host__ __device__ constexpr int rr_hi(int n, int r, int i) { return rr_a(n, r, i) < rr_b(n, r, i) ? rr_b(n, r, i) : rr_a(n, r, i); }
template <int NZ, int NA = NZ>
__device__ inline void mirror(double A[NZ][NZ], double eps, double dia_extra = 0.0) {
    // Cyclic Jacobi on the symmetric part, one-sided rotation updates on the
    // upper triangle (a_pp -= t a_pq, a_qq += t a_pq, off-diagonal pairs with
    // tau = s / (1 + c)); V accumulates the eigenvectors.  Then
    // A = V diag(f(d)) V' with f(d) = eps if |d| <= eps else |d|.
    double V[NA][NA];
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            V[i][j] = (i == j) ? 1.0 : 0.0;
            if (j > i) A[i][j] = 0.5 * (A[i][j] + A[j][i]);
        }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0, dia = 0.0;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            dia += A[i][i] * A[i][i];
            if (i == NA - 1) dia += dia_extra;
#pragma unroll
            for (int j = i + 1; j < NA; ++j) off += A[i][j] * A[i][j];
        }
        if (off <= 1e-32 * dia || off < 1e-300) break;
#if MPCG_MIRROR_RR
        // round-robin (parallel) ordering: the pairs of a round are disjoint, so their rotation
        // parameters depend only on the round's starting entries and their reciprocal / square
        // root chains run side by side; the rotations are then applied one after the other
        constexpr int NPL = NA + (NA & 1), NPR = NPL / 2;
#pragma unroll
        for (int rd = 0; rd < NPL - 1; ++rd) {
            double tr[NPR], snr[NPR], taur[NPR];
            bool on[NPR];
#pragma unroll
            for (int i = 0; i < NPR; ++i) {
                const int p = rr_lo(NPL, rd, i), q = rr_hi(NPL, rd, i);
                on[i] = false;
                if (q >= NA) continue;  // the bye of an odd count
                const double apq = A[p][q];
                on[i] = fabs(apq) >= 1e-300;
                const double theta = 0.5 * (A[q][q] - A[p][p]) * frcp(on[i] ? apq : 1.0);
                const double at = fabs(theta);
                double t = at < 1e150 ? frcp(at + fsqrt_pos(fma(at, at, 1.0))) : 0.5 * frcp(at);
                t = theta >= 0.0 ? t : -t;
                const double c = frsq(fma(t, t, 1.0));
                tr[i] = t;
                snr[i] = t * c;
                taur[i] = snr[i] * frcp(1.0 + c);
            }
#pragma unroll
            for (int i = 0; i < NPR; ++i) {
                const int p = rr_lo(NPL, rd, i), q = rr_hi(NPL, rd, i);
                if (q >= NA || !on[i]) continue;
                const double apq = A[p][q], t = tr[i], sn = snr[i], tau = taur[i];
                A[p][p] -= t * apq;
                A[q][q] += t * apq;
                A[p][q] = 0.0;
#pragma unroll
                for (int r = 0; r < NA; ++r) {
                    if (r == p || r == q) continue;
                    double& arp = r < p ? A[r][p] : A[p][r];
                    double& arq = r < q ? A[r][q] : A[q][r];
                    const double g = arp, h = arq;
                    arp = g - sn * fma(g, tau, h);
                    arq = h + sn * fma(-h, tau, g);
                }
#pragma unroll
                for (int r = 0; r < NA; ++r) {
                    const double g = V[r][p], h = V[r][q];
                    V[r][p] = g - sn * fma(g, tau, h);
                    V[r][q] = h + sn * fma(-h, tau, g);
                }
            }
        }
        continue;
#endif
#pragma unroll
        for (int p = 0; p < NA - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < NA; ++q) {
                const double apq = A[p][q];
                if (fabs(apq) >= 1e-300) {
                    const double theta = 0.5 * (A[q][q] - A[p][p]) * frcp(apq);
                    const double at = fabs(theta);
                    // t = 1 / (|theta| + sqrt(theta^2 + 1)); ~1 / (2 |theta|) once theta^2 would overflow
                    double t = at < 1e150 ? frcp(at + fsqrt_pos(fma(at, at, 1.0))) : 0.5 * frcp(at);
                    t = theta >= 0.0 ? t : -t;
                    const double c = frsq(fma(t, t, 1.0)), sn = t * c;
                    const double tau = sn * frcp(1.0 + c);
                    A[p][p] -= t * apq;
                    A[q][q] += t * apq;
                    A[p][q] = 0.0;
#pragma unroll
                    for (int r = 0; r < NA; ++r) {
                        if (r == p || r == q) continue;
                        double& arp = r < p ? A[r][p] : A[p][r];
                        double& arq = r < q ? A[r][q] : A[q][r];
                        const double g = arp, h = arq;
                        arp = g - sn * fma(g, tau, h);
                        arq = h + sn * fma(-h, tau, g);
                    }
#pragma unroll
                    for (int r = 0; r < NA; ++r) {
                        const double g = V[r][p], h = V[r][q];
                        V[r][p] = g - sn * fma(g, tau, h);
                        V[r][q] = h + sn * fma(-h, tau, g);
                    }
                }
            }
    }
    double d[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        double di = A[i][i];
        d[i] = (di >= -eps && di <= eps) ? eps : fabs(di);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = i; j < NA; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < NA; ++k) acc += V[i][k] * d[k] * V[j][k];
            A[i][j] = acc;
            A[j][i] = acc;
        }
}

// The sweeps of mirror() with the eigenvector rows split over the PARTS lanes of a stage: every
// part applies the same rotations to its own copy of A (symmetrised upper triangle, from the
// stage's part 0), and part p accumulates only the rows p, p + PARTS, ... of V (Vr[t] = row
// p + PARTS t; rows past NA stay unused).  Per entry the operations of mirror(): bit-identical.
template <int NZ, int NA, int PARTS>
__device__ inline void mirror_rows(double A[NZ][NZ], double (&Vr)[(NA + PARTS - 1) / PARTS][NA], int part,
                                   double dia_extra) {
    constexpr int RV = (NA + PARTS - 1) / PARTS;
#pragma unroll
    for (int t = 0; t < RV; ++t)
#pragma unroll
        for (int j = 0; j < NA; ++j) Vr[t][j] = (part + PARTS * t == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0, dia = 0.0;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            dia += A[i][i] * A[i][i];
            if (i == NA - 1) dia += dia_extra;
#pragma unroll
            for (int j = i + 1; j < NA; ++j) off += A[i][j] * A[i][j];
        }
        if (off <= 1e-32 * dia || off < 1e-300) break;
#pragma unroll
        for (int p = 0; p < NA - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < NA; ++q) {
                const double apq = A[p][q];
                if (fabs(apq) >= 1e-300) {
                    const double theta = 0.5 * (A[q][q] - A[p][p]) * frcp(apq);
                    const double at = fabs(theta);
                    double t = at < 1e150 ? frcp(at + fsqrt_pos(fma(at, at, 1.0))) : 0.5 * frcp(at);
                    t = theta >= 0.0 ? t : -t;
                    const double c = frsq(fma(t, t, 1.0)), sn = t * c;
                    const double tau = sn * frcp(1.0 + c);
                    A[p][p] -= t * apq;
                    A[q][q] += t * apq;
                    A[p][q] = 0.0;
#pragma unroll
                    for (int r = 0; r < NA; ++r) {
                        if (r == p || r == q) continue;
                        double& arp = r < p ? A[r][p] : A[p][r];
                        double& arq = r < q ? A[r][q] : A[q][r];
                        const double g = arp, h = arq;
                        arp = g - sn * fma(g, tau, h);
                        arq = h + sn * fma(-h, tau, g);
                    }
#pragma unroll
                    for (int r = 0; r < RV; ++r) {
                        const double g = Vr[r][p], h = Vr[r][q];
                        Vr[r][p] = g - sn * fma(g, tau, h);
                        Vr[r][q] = h + sn * fma(-h, tau, g);
                    }
                }
            }
    }
}
// mirror()'s reconstruction A = V diag(f(d)) V' from the eigenvalues on A's diagonal
template <int NZ, int NA>
__device__ inline void mirror_rebuild(double A[NZ][NZ], const double (&V)[NA][NA], double eps) {
    double d[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        double di = A[i][i];
        d[i] = (di >= -eps && di <= eps) ? eps : fabs(di);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = i; j < NA; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < NA; ++k) acc += V[i][k] * d[k] * V[j][k];
            A[i][j] = acc;
            A[j][i] = acc;
        }
}

}  // namespace mpcg
