// mpcg_bicycle.h — C3 stage functions on the device (gfx950, fp64 VALU):
// BicycleModel2ndOrderCurvatureAware + MPCBase(a, w, slack) +
// CurvatureAwareContouring; the decomp halfspaces are the kernel's slack rows.
//
// Reference semantics (paths relative to the reference repo):
//   model      solver_model.py:355-396 (bicycle, integrated states x y psi v delta,
//              beta = atan(l_r / (l_r + l_f) tan delta), l_r = l_f = 2.79 / 2),
//              :398-437 (the CA spline update s+ = s + R atan2(vt, R - e_c - vn),
//              R = fmax(1 / curvature, 1e5)); integrated by forces_discrete_dynamics
//              (:11-36): RK4 over integrator_step (pr.rk_steps steps)
//   cost       mpc_base.py:47-60 + curvature_aware_contouring.py:48-105, the terminal
//              terms at stage N-1 as Forces applies them (generate_forces_solver.py:50-59)
//   spline     spline.py:4-86 (glued value, derivative and second derivative)
//
// z = [a, w, slack, x, y, psi, v, delta, s].  Every nonlinear piece depends on
// at most five stage variables, so derivatives come from second-order jets
// over five local variables (value, gradient, packed Hessian: 21 doubles);
// functions of the path coordinate s alone are carried as one-dimensional
// jets (f, f', f'') and lifted into the stage jets.
#pragma once
#include <hip/hip_runtime.h>

#include "mpcg.h"
#include "mpcg_device.h"

namespace mpcg {
namespace bike {

constexpr int NUB = 3, NXB = 6, NZB = NUB + NXB;
constexpr int ZA = 0, ZW = 1, ZSL = 2, ZX = 3, ZY = 4, ZPSI = 5, ZV = 6, ZDELTA = 7, ZS = 8;
constexpr double LR = 2.79 / 2.0;          // solver_model.py:383-386
constexpr double RATIO = LR / (LR + LR);
constexpr double PI_D = 3.14159265358979323846;

__host__ __device__ constexpr int tri(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// ---- one-dimensional jets in s: (f, f', f'')
struct S1 {
    double v, d, dd;
};
__device__ __forceinline__ S1 s1_mul(S1 a, S1 b) { return {a.v * b.v, a.d * b.v + a.v * b.d, a.dd * b.v + 2.0 * a.d * b.d + a.v * b.dd}; }
__device__ __forceinline__ S1 s1_fn(S1 a, double f, double f1, double f2) { return {f, f1 * a.d, f1 * a.dd + f2 * a.d * a.d}; }
__device__ __forceinline__ S1 s1_inv(S1 a) { const double i = frcp(a.v); return s1_fn(a, i, -i * i, 2.0 * i * i * i); }

// ---- second-order jets over five local variables
struct J5 {
    double v, g[5], h[15];
};
__device__ __forceinline__ J5 jconst(double c) {
    J5 r;
    r.v = c;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.g[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 15; ++i) r.h[i] = 0.0;
    return r;
}
__device__ __forceinline__ J5 jvar(int i, double x) {
    J5 r = jconst(x);
    r.g[i] = 1.0;
    return r;
}
// a one-dimensional s-jet lifted into variable i
__device__ __forceinline__ J5 jlift(S1 a, int i) {
    J5 r = jconst(a.v);
    r.g[i] = a.d;
    r.h[tri(i, i)] = a.dd;
    return r;
}
// f(a): f' = f1, f'' = f2
__device__ __forceinline__ J5 jfn(const J5& a, double f, double f1, double f2) {
    J5 r;
    r.v = f;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.g[i] = f1 * a.g[i];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) r.h[tri(i, j)] = f1 * a.h[tri(i, j)] + f2 * a.g[i] * a.g[j];
    return r;
}
// f(a, b): partials fa, fb, faa, fab, fbb
__device__ __forceinline__ J5 jfn2(const J5& a, const J5& b, double f, double fa, double fb, double faa, double fab,
                                   double fbb) {
    J5 r;
    r.v = f;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.g[i] = fa * a.g[i] + fb * b.g[i];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j)
            r.h[tri(i, j)] = fa * a.h[tri(i, j)] + fb * b.h[tri(i, j)] + faa * a.g[i] * a.g[j] +
                             fab * (a.g[i] * b.g[j] + b.g[i] * a.g[j]) + fbb * b.g[i] * b.g[j];
    return r;
}
__device__ __forceinline__ J5 operator+(const J5& a, const J5& b) { return jfn2(a, b, a.v + b.v, 1.0, 1.0, 0.0, 0.0, 0.0); }
__device__ __forceinline__ J5 operator-(const J5& a, const J5& b) { return jfn2(a, b, a.v - b.v, 1.0, -1.0, 0.0, 0.0, 0.0); }
__device__ __forceinline__ J5 operator*(const J5& a, const J5& b) { return jfn2(a, b, a.v * b.v, b.v, a.v, 0.0, 1.0, 0.0); }
__device__ __forceinline__ J5 operator*(double c, const J5& a) { return jfn(a, c * a.v, c, 0.0); }
__device__ __forceinline__ J5 operator+(const J5& a, double c) { return jfn(a, a.v + c, 1.0, 0.0); }
__device__ __forceinline__ J5 jsq(const J5& a) { return jfn(a, a.v * a.v, 2.0 * a.v, 2.0); }
__device__ __forceinline__ J5 jinv(const J5& a) { const double i = frcp(a.v); return jfn(a, i, -i * i, 2.0 * i * i * i); }
__device__ __forceinline__ J5 jcos(const J5& a, double c, double s) { return jfn(a, c, -s, -c); }
__device__ __forceinline__ J5 jsin(const J5& a, double c, double s) { return jfn(a, s, c, -s); }
__device__ __forceinline__ J5 jatan2(const J5& y, const J5& x) {
    const double r2 = x.v * x.v + y.v * y.v, ir2 = frcp(r2), ir4 = ir2 * ir2;
    return jfn2(y, x, fatan2(y.v, x.v, FRcp{}), x.v * ir2, -y.v * ir2, -2.0 * x.v * y.v * ir4, (y.v * y.v - x.v * x.v) * ir4,
                2.0 * x.v * y.v * ir4);
}

// Glued spline of spline.py:28-58 for one axis: value P, derivative D and
// second derivative Z, each a jet in s (segment values glued with the sigmoids).
struct PathJets {
    S1 P[2], D[2], Z[2];
};
__device__ inline void path_jets(const mpcg_problem& pr, const double* __restrict__ p, double s, PathJets& J) {
    const int M = pr.n_seg;
    const double* base = p + pr.i_spline0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        // segment M-1: P, P', P'', P'''
        const double* c = base + 9 * (M - 1) + 4 * ax;
        double t = s - base[9 * (M - 1) + 8];
        double q0 = ((c[0] * t + c[1]) * t + c[2]) * t + c[3], q1 = (3.0 * c[0] * t + 2.0 * c[1]) * t + c[2];
        double q2 = 6.0 * c[0] * t + 2.0 * c[1], q3 = 6.0 * c[0];
        S1 P = {q0, q1, q2}, D = {q1, q2, q3}, Z = {q2, q3, 0.0};
        for (int k = M - 1; k >= 1; --k) {
            const double e = exp((s - base[9 * k + 8] + 0.02) / 0.1);
            const double l0 = e < 0x1p1000 ? frcp(1.0 + e) : 0.0;  // 1 / (1 + inf) = 0, as the oracle
            const double l1 = -10.0 * l0 * (1.0 - l0);
            const double l2 = 100.0 * l0 * (1.0 - l0) * (1.0 - 2.0 * l0);
            const double m0 = 1.0 - l0;
            c = base + 9 * (k - 1) + 4 * ax;
            t = s - base[9 * (k - 1) + 8];
            q0 = ((c[0] * t + c[1]) * t + c[2]) * t + c[3];
            q1 = (3.0 * c[0] * t + 2.0 * c[1]) * t + c[2];
            q2 = 6.0 * c[0] * t + 2.0 * c[1];
            q3 = 6.0 * c[0];
            // glue (l * A + (1 - l) * Q) with its first two s-derivatives, A = segment k-1
            auto glue = [&](S1 Q, double a0, double a1, double a2) -> S1 {
                return {l0 * a0 + m0 * Q.v, l1 * (a0 - Q.v) + l0 * a1 + m0 * Q.d,
                        l2 * (a0 - Q.v) + 2.0 * l1 * (a1 - Q.d) + l0 * a2 + m0 * Q.dd};
            };
            P = glue(P, q0, q1, q2);
            D = glue(D, q1, q2, q3);
            Z = glue(Z, q2, q3, 0.0);
        }
        J.P[ax] = P;
        J.D[ax] = D;
        J.Z[ax] = Z;
    }
}

// unit tangent t = D / |D| (spline.py:72-77) as s-jets
__device__ __forceinline__ void tangent(const PathJets& J, S1& tx, S1& ty) {
    const S1 r2 = {J.D[0].v * J.D[0].v + J.D[1].v * J.D[1].v, 2.0 * (J.D[0].v * J.D[0].d + J.D[1].v * J.D[1].d),
                   2.0 * (J.D[0].d * J.D[0].d + J.D[0].v * J.D[0].dd + J.D[1].d * J.D[1].d + J.D[1].v * J.D[1].dd)};
    const double ir = frsq(r2.v);  // 1 / sqrt
    const S1 inr = s1_fn(r2, ir, -0.5 * ir * ir * ir, 0.75 * ir * ir * ir * ir * ir);
    tx = s1_mul(J.D[0], inr);
    ty = s1_mul(J.D[1], inr);
}

// ---------------------------------------------------------------------------
// stage cost of stage k: MPCBase(a, w, slack) + CA contouring (+ terminal terms
// at k = N-1).  Jet variables: 0 x, 1 y, 2 psi, 3 v, 4 s.
// ---------------------------------------------------------------------------
__device__ inline double stage_cost(const mpcg_problem& pr, const double* __restrict__ p, int k,
                                    const double z[NZB], double g[NZB], double H[NZB][NZB], bool derivs) {
    const double wa = p[pr.i_w_acc], ww = p[pr.i_w_ang], ws = p[pr.i_w_slack];
    const double wc = p[pr.i_w_contour], wv = p[pr.i_w_vel], vref = p[pr.i_v_ref];
    const double a = z[ZA], w = z[ZW], sl = z[ZSL];
    PathJets PJ;
    path_jets(pr, p, z[ZS], PJ);
    S1 tx1, ty1;
    tangent(PJ, tx1, ty1);
    const J5 x = jvar(0, z[ZX]), y = jvar(1, z[ZY]), psi = jvar(2, z[ZPSI]), v = jvar(3, z[ZV]);
    const J5 tx = jlift(tx1, 4), ty = jlift(ty1, 4);
    const J5 ex = x - jlift(PJ.P[0], 4), ey = y - jlift(PJ.P[1], 4);
    // projection_ratio = 1 / (1 - ((x - px) ddx + (y - py) ddy))  (curvature_aware_contouring.py:83-84)
    const J5 proj = jinv((-1.0) * (ex * jlift(PJ.Z[0], 4) + ey * jlift(PJ.Z[1], 4)) + 1.0);
    double sp, cp;
    fsincos(z[ZPSI], &sp, &cp);
    // s_dot = v (cos psi tx + sin psi ty) projection_ratio  (:85)
    const J5 sdot = (v * (jcos(psi, cp, sp) * tx + jsin(psi, cp, sp) * ty)) * proj;
    const J5 cerr2 = jsq(ex) + jsq(ey);  // (:88)
    const J5 verr2 = jsq(sdot + (-vref));
    J5 L = wc * cerr2 + wv * verr2;      // (:90-91)
    if (k == pr.N - 1) {                 // terminal terms (:94-103)
        const double wta = p[pr.i_w_tangle], tc = p[pr.i_w_tcont];
        const J5 pa = jatan2(ty, tx);
        // haar_difference_without_abs = fmod(a1 - a2 + pi, 2 pi) - pi (util/math.py:10-11)
        const J5 d = psi - pa + PI_D;
        const J5 ae = jfn(d, fmod(d.v, 2.0 * PI_D), 1.0, 0.0) + (-PI_D);
        L = L + wta * jsq(ae) + (tc * wc) * cerr2 + (tc * wv) * verr2;
    }
    const double Lv = wa * a * a + ww * w * w + ws * sl * sl + L.v;
    if (!derivs) return Lv;
#pragma unroll
    for (int i = 0; i < NZB; ++i) {
        g[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NZB; ++j) H[i][j] = 0.0;
    }
    g[ZA] = 2.0 * wa * a; H[ZA][ZA] = 2.0 * wa;
    g[ZW] = 2.0 * ww * w; H[ZW][ZW] = 2.0 * ww;
    g[ZSL] = 2.0 * ws * sl; H[ZSL][ZSL] = 2.0 * ws;
    constexpr int zi[5] = {ZX, ZY, ZPSI, ZV, ZS};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        g[zi[i]] = L.g[i];
#pragma unroll
        for (int j = 0; j < 5; ++j) H[zi[i]][zi[j]] = L.h[tri(i, j)];
    }
    return Lv;
}

// ---------------------------------------------------------------------------
// Discrete map of one shooting interval: RK4 (pr.rk_steps steps over dt) of the
// five bicycle states, then the CA spline update.  Outputs xn, the rows of
// [B A] of x+, y+, psi+ and s+ without the slack column (written straight to
// `F`, LDS in the kernel; the rows of v+ = v + dt a and delta+ = delta + dt w
// are known) and Hs = Hess(pi' x+) packed without the slack row / column (lower triangle,
// tri(fc(i), fc(j)); the slack couples to nothing): the stage's LDS Hessian block, so that
// the 36 entries are not held in registers through the spline update.
// RK jets over 0 a, 1 w, 2 psi, 3 v, 4 delta; x and y enter the integrated
// positions additively (x+ = x + dX, y+ = y + dY), so dp = (dX, dY) in the update.
// Written to keep few jets live at once (the linearisation lane's registers):
// F rows and the psi Hessian leave before the update is evaluated.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void discrete(const mpcg_problem& pr, const double* __restrict__ p, const double z[NZB],
                                const double* pi, double xn[NXB], double (*F)[NZB - 1], double* Hs) {
    const int ns = pr.rk_steps;
    const double h = pr.dt / ns;
    // v' = a and delta' = w are integrated exactly (v_q = v + tau a, delta_q = delta + tau w at
    // every RK stage argument), so their jets stay sparse; psi, dX, dY carry the nonlinearity.
    J5 psi = jvar(2, z[ZPSI]), dX = jconst(0.0), dY = jconst(0.0);
    for (int st = 0; st < ns; ++st) {
        // the step's increments go straight into dX, dY and the psi accumulator
        J5 kp, psin = psi;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double cq = (q == 0) ? 0.0 : ((q == 3) ? 1.0 : 0.5);
            const double wq = ((q == 0 || q == 3) ? 1.0 : 2.0) * h / 6.0;
            const double tau = (st + cq) * h;
            const J5 pq = q ? psi + (cq * h) * kp : psi;
            J5 vq = jvar(3, z[ZV] + tau * z[ZA]);
            vq.g[0] = tau;
            J5 dq = jvar(4, z[ZDELTA] + tau * z[ZW]);
            dq.g[1] = tau;
            // beta = atan(ratio tan delta)
            const double td = ftan(dq.v);
            const double rt = RATIO * td, ib = frcp(1.0 + rt * rt);
            // d beta / d delta and d2 beta / d delta2 through rt = ratio tan(delta)
            const double rt1 = RATIO * (1.0 + td * td), rt2 = RATIO * 2.0 * td * (1.0 + td * td);
            const J5 beta = jfn(dq, fatan(rt, FRcp{}), ib * rt1, ib * rt2 - 2.0 * rt * ib * ib * rt1 * rt1);
            const J5 ang = pq + beta;
            double sa, ca, sb, cb;
            fsincos(ang.v, &sa, &ca);
            fsincos(beta.v, &sb, &cb);
            dX = dX + wq * (vq * jcos(ang, ca, sa));
            dY = dY + wq * (vq * jsin(ang, ca, sa));
            kp = ((1.0 / LR) * vq) * jsin(beta, cb, sb);
            psin = psin + wq * kp;
        }
        psi = psin;
    }
    constexpr int ri[5] = {ZA, ZW, ZPSI, ZV, ZDELTA};
    // rows x+, y+, psi+, v+ = v + dt a, delta+ = delta + dt w
    xn[0] = z[ZX] + dX.v;
    xn[1] = z[ZY] + dY.v;
    xn[2] = psi.v;
    xn[3] = z[ZV] + pr.dt * z[ZA];
    xn[4] = z[ZDELTA] + pr.dt * z[ZW];
    // compact column of z variable j (the slack column is not stored)
    constexpr auto fc = [](int j) { return j < ZSL ? j : j - 1; };
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < NZB - 1; ++j) F[i][j] = 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        F[0][fc(ri[j])] = dX.g[j];
        F[1][fc(ri[j])] = dY.g[j];
        F[2][fc(ri[j])] = psi.g[j];
    }
    F[0][fc(ZX)] = 1.0;
    F[1][fc(ZY)] = 1.0;
    const double p2 = pi ? pi[2] : 0.0;
    constexpr auto hc = [](int i, int j) { return tri(i < ZSL ? i : i - 1, j < ZSL ? j : j - 1); };
#pragma unroll
    for (int i = 0; i < (NZB - 1) * NZB / 2; ++i) Hs[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Hs[hc(ri[i], ri[j])] = p2 * psi.h[tri(i, j)];

    // ---- CA spline update (solver_model.py:409-437); local jets 0 x, 1 y, 2 s, 3 dpx, 4 dpy
    PathJets PJ;
    path_jets(pr, p, z[ZS], PJ);
    S1 tx1, ty1;
    tangent(PJ, tx1, ty1);
    const S1 c2 = {PJ.Z[0].v * PJ.Z[0].v + PJ.Z[1].v * PJ.Z[1].v,
                   2.0 * (PJ.Z[0].v * PJ.Z[0].d + PJ.Z[1].v * PJ.Z[1].d),
                   2.0 * (PJ.Z[0].d * PJ.Z[0].d + PJ.Z[0].v * PJ.Z[0].dd + PJ.Z[1].d * PJ.Z[1].d + PJ.Z[1].v * PJ.Z[1].dd)};
    // R = fmax(1 / |Z|, 1e5) = fmax(c2^-1/2, 1e5)
    const double irc = frsq(c2.v);
    S1 R1 = s1_fn(c2, irc, -0.5 * irc * irc * irc, 0.75 * irc * irc * irc * irc * irc);
    if (!(R1.v > 1e5)) R1 = {1e5, 0.0, 0.0};
    const J5 x = jvar(0, z[ZX]), y = jvar(1, z[ZY]), dpx = jvar(3, dX.v), dpy = jvar(4, dY.v);
    const J5 tx = jlift(tx1, 2), ty = jlift(ty1, 2), R = jlift(R1, 2);
    const J5 ec = ty * (x - jlift(PJ.P[0], 2)) - tx * (y - jlift(PJ.P[1], 2));  // (:423)
    const J5 vt = dpx * tx + dpy * ty;                                         // (:429)
    const J5 vn = dpx * ty - dpy * tx;                                         // (:430)
    const J5 G = jvar(2, z[ZS]) + R * jatan2(vt, R - ec - vn);                 // (:435-437)
    xn[5] = G.v;
#pragma unroll
    for (int j = 0; j < NZB - 1; ++j) F[3][j] = 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) F[3][fc(ri[j])] = G.g[3] * dX.g[j] + G.g[4] * dY.g[j];
    F[3][fc(ZX)] = G.g[0];
    F[3][fc(ZY)] = G.g[1];
    F[3][fc(ZS)] = G.g[2];
    if (!pi) return;
    const double ps = pi[5];
    const double cX = pi[0] + ps * G.g[3], cY = pi[1] + ps * G.g[4];
    // (a, w, psi, v, delta) block: second derivatives of dX, dY and the update's (dpx, dpy) block
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double gxi = ps * (G.h[tri(3, 3)] * dX.g[i] + G.h[tri(4, 3)] * dY.g[i]);
        const double gyi = ps * (G.h[tri(4, 3)] * dX.g[i] + G.h[tri(4, 4)] * dY.g[i]);
#pragma unroll
        for (int j = 0; j <= i; ++j)
            Hs[hc(ri[i], ri[j])] += cX * dX.h[tri(i, j)] + cY * dY.h[tri(i, j)] + gxi * dX.g[j] + gyi * dY.g[j];
    }
    // (x, y, s) block and its coupling with (a, w, psi, v, delta) through (dpx, dpy)
    constexpr int ui[3] = {ZX, ZY, ZS};
#pragma unroll
    for (int m = 0; m < 3; ++m) {
#pragma unroll
        for (int n = 0; n <= m; ++n) Hs[hc(ui[m], ui[n])] += ps * G.h[tri(m, n)];
        const double c3 = ps * G.h[tri(3, m)], c4 = ps * G.h[tri(4, m)];
#pragma unroll
        for (int j = 0; j < 5; ++j) Hs[hc(ui[m], ri[j])] += c3 * dX.g[j] + c4 * dY.g[j];
    }
}

}  // namespace bike
}  // namespace mpcg
