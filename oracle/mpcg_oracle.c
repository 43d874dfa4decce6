/*
 * mpcg_oracle.c — CPU restatement (plain C99) of the reference's per-guess
 * SQP solve.  TEST INFRASTRUCTURE ONLY: see mpcg_oracle.h for scope, the
 * reference lines each routine follows, and the pinning status.
 *
 * Deliberately written as the most literal, loop-per-formula C: dense 7x7
 * stage blocks, Jacobi eigen-decomposition, textbook Riccati recursion.  It
 * shares no source with the HIP kernels it checks.
 */
#include "mpcg_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX ORC_NX
#define NU ORC_NU
#define NZ ORC_NZ
#define BIGBOUND 1e15 /* generate_acados_solver.py:17-24 maps +-inf to +-1e15 */

/* acados return codes (acados/utils/types.h) */
enum { AC_SUCCESS = 0, AC_NAN = 1, AC_MAXITER = 2, AC_MINSTEP = 3, AC_QP_FAILURE = 4 };

/* ------------------------------------------------------------------ */
/* Glued cubic spline (spline.py:4-86)                                 */
/* ------------------------------------------------------------------ */

#ifndef ORC_BICYCLE_CA
/* value and first two s-derivatives of the sigmoid glue weight
 * lambda_k(s) = 1 / (1 + exp((s - s_k + 0.02) / 0.1))        (spline.py:37) */
static void glue_weight(double s, double sk, double *l0, double *l1, double *l2) {
    double e = exp((s - sk + 0.02) / 0.1);
    double l = 1.0 / (1.0 + e);
    *l0 = l;
    *l1 = -10.0 * l * (1.0 - l);
    *l2 = 100.0 * l * (1.0 - l) * (1.0 - 2.0 * l);
}

/* For one axis: G = glued position (spline.py:39-44) and D = glued segment
 * derivative (spline.py:46-51), each with its first two s-derivatives. */
static void spline_axis(const orc_problem *pr, const double *p, double s, int axis,
                        const double (*lam)[3], double G[3], double D[3]) {
    int M = pr->n_seg;
    double Pj[ORC_MAX_SEG][4]; /* P, P', P'', P''' of each segment */
    for (int j = 0; j < M; j++) {
        const double *c = p + pr->i_spline0 + 9 * j + 4 * axis;
        double t = s - p[pr->i_spline0 + 9 * j + 8];
        double a = c[0], b = c[1], cc = c[2], d = c[3];
        Pj[j][0] = a * t * t * t + b * t * t + cc * t + d;
        Pj[j][1] = 3.0 * a * t * t + 2.0 * b * t + cc;
        Pj[j][2] = 6.0 * a * t + 2.0 * b;
        Pj[j][3] = 6.0 * a;
    }
    double V[3] = {Pj[M - 1][0], Pj[M - 1][1], Pj[M - 1][2]};
    double W[3] = {Pj[M - 1][1], Pj[M - 1][2], Pj[M - 1][3]};
    for (int k = M - 1; k >= 1; k--) {
        double l0 = lam[k][0], l1 = lam[k][1], l2 = lam[k][2];
        const double *A = Pj[k - 1];
        double nV0 = l0 * A[0] + (1.0 - l0) * V[0];
        double nV1 = l1 * (A[0] - V[0]) + l0 * A[1] + (1.0 - l0) * V[1];
        double nV2 = l2 * (A[0] - V[0]) + 2.0 * l1 * (A[1] - V[1]) + l0 * A[2] + (1.0 - l0) * V[2];
        double nW0 = l0 * A[1] + (1.0 - l0) * W[0];
        double nW1 = l1 * (A[1] - W[0]) + l0 * A[2] + (1.0 - l0) * W[1];
        double nW2 = l2 * (A[1] - W[0]) + 2.0 * l1 * (A[2] - W[1]) + l0 * A[3] + (1.0 - l0) * W[2];
        V[0] = nV0; V[1] = nV1; V[2] = nV2;
        W[0] = nW0; W[1] = nW1; W[2] = nW2;
    }
    memcpy(G, V, sizeof V);
    memcpy(D, W, sizeof W);
}

#endif

#ifdef ORC_BICYCLE_CA
#define SLACK_IDX 2 /* the slack input of BicycleModel2ndOrderCurvatureAware (solver_model.py:364) */
#else
#define SLACK_IDX (NU + NX - 1)
#endif

#ifdef ORC_BICYCLE_CA
#include "orc_bicycle_ca.inc"
#else
void orc_ca_update(const orc_problem *pr, const double *z, const double *I, const double *p,
                   double *g, double *grad, double *hess) {
    (void)pr; (void)z; (void)I; (void)p; (void)grad; (void)hess;
    *g = 0.0;
}

void orc_stage_cost_k(const orc_problem *pr, int k, const double *z, const double *p,
                      double *Lout, double *grad, double *hess) {
    (void)k;
    orc_stage_cost(pr, z, p, Lout, grad, hess);
}

/* ------------------------------------------------------------------ */
/* Stage cost (solver_definition.py:19-34)                            */
/* ------------------------------------------------------------------ */
void orc_stage_cost(const orc_problem *pr, const double *z, const double *p,
                    double *Lout, double *grad, double *hess) {
    double a = z[0], w = z[1], x = z[2], y = z[3], v = z[5], s = z[6];
    double g[NZ] = {0}, H[NZ][NZ];
    memset(H, 0, sizeof H);
    double L = 0.0;

    /* MPCBase weights (mpc_base.py:47-60; cost functions as configured in
     * generate_jackalsimulator_solver.py:47-53) */
    double wa = p[pr->i_w_acc], ww = p[pr->i_w_ang];
    double wv = p[pr->i_w_vel], vref = p[pr->i_v_ref];
    L += wa * a * a;
    g[0] += 2.0 * wa * a; H[0][0] += 2.0 * wa;
    L += ww * w * w;
    g[1] += 2.0 * ww * w; H[1][1] += 2.0 * ww;
    L += wv * (v - vref) * (v - vref);
    g[5] += 2.0 * wv * (v - vref); H[5][5] += 2.0 * wv;
#if ORC_NX > 5
    /* slack weight (generate_jackalsimulator_solver.py:78) */
    if (pr->i_w_slack >= 0) {
        double ws = p[pr->i_w_slack], sl = z[NU + 5];
        L += ws * sl * sl;
        g[NU + 5] += 2.0 * ws * sl; H[NU + 5][NU + 5] += 2.0 * ws;
    }
#endif

    /* Contouring (contouring.py:140-174), stage_idx=1 => no terminal terms */
    double lam[ORC_MAX_SEG][3];
    for (int k = 1; k < pr->n_seg; k++)
        glue_weight(s, p[pr->i_spline0 + 9 * k + 8], &lam[k][0], &lam[k][1], &lam[k][2]);
    double Gx[3], Dx[3], Gy[3], Dy[3];
    spline_axis(pr, p, s, 0, (const double (*)[3])lam, Gx, Dx);
    spline_axis(pr, p, s, 1, (const double (*)[3])lam, Gy, Dy);
    /* unit tangent t = D/|D| (spline.py:72-77) and its s-derivatives */
    double r = sqrt(Dx[0] * Dx[0] + Dy[0] * Dy[0]);
    double tx = Dx[0] / r, ty = Dy[0] / r;
    double r1 = tx * Dx[1] + ty * Dy[1];
    double tx1 = (Dx[1] - tx * r1) / r, ty1 = (Dy[1] - ty * r1) / r;
    double r2 = tx1 * Dx[1] + ty1 * Dy[1] + tx * Dx[2] + ty * Dy[2];
    double tx2 = (Dx[2] - 2.0 * tx1 * r1 - tx * r2) / r;
    double ty2 = (Dy[2] - 2.0 * ty1 * r1 - ty * r2) / r;
    double ex = x - Gx[0], ey = y - Gy[0];
    double wc = p[pr->i_w_contour], wl = p[pr->i_w_lag];

    /* contour error e_c = ty*ex - tx*ey, lag error e_l = tx*ex + ty*ey (contouring.py:166-167) */
    double ec = ty * ex - tx * ey;
    double el = tx * ex + ty * ey;
    /* gradients over (x, y, s) */
    double dec[3] = {ty, -tx, ty1 * ex - tx1 * ey - ty * Gx[1] + tx * Gy[1]};
    double del[3] = {tx, ty, tx1 * ex + ty1 * ey - tx * Gx[1] - ty * Gy[1]};
    /* second derivatives over (x, y, s) */
    double hec[3][3] = {{0, 0, ty1}, {0, 0, -tx1},
                        {ty1, -tx1, ty2 * ex - tx2 * ey - 2.0 * ty1 * Gx[1] + 2.0 * tx1 * Gy[1] - ty * Gx[2] + tx * Gy[2]}};
    double hel[3][3] = {{0, 0, tx1}, {0, 0, ty1},
                        {tx1, ty1, tx2 * ex + ty2 * ey - 2.0 * tx1 * Gx[1] - 2.0 * ty1 * Gy[1] - tx * Gx[2] - ty * Gy[2]}};
    static const int ids[3] = {2, 3, 6};
    L += wl * el * el;
    L += wc * ec * ec;
    for (int i = 0; i < 3; i++) {
        g[ids[i]] += 2.0 * wl * el * del[i] + 2.0 * wc * ec * dec[i];
        for (int j = 0; j < 3; j++)
            H[ids[i]][ids[j]] += 2.0 * wl * (del[i] * del[j] + el * hel[i][j]) +
                                 2.0 * wc * (dec[i] * dec[j] + ec * hec[i][j]);
    }

    /* Consistency (consistency_module.py:229-250) */
    if (pr->i_cons_w >= 0) {
        double wcn = p[pr->i_cons_w];
        double dx = x - p[pr->i_prev_x], dy = y - p[pr->i_prev_y];
        L += wcn * (dx * dx + dy * dy);
        g[2] += 2.0 * wcn * dx; g[3] += 2.0 * wcn * dy;
        H[2][2] += 2.0 * wcn; H[3][3] += 2.0 * wcn;
    }
    *Lout = L;
    if (grad) memcpy(grad, g, sizeof g);
    if (hess) memcpy(hess, H, sizeof H);
}

#endif /* ORC_BICYCLE_CA */

/* ------------------------------------------------------------------ */
/* Constraints h(z) (solver_definition.py:37-49)                      */
/* ------------------------------------------------------------------ */
int orc_nx(void) { return ORC_NX; }
int orc_nu(void) { return ORC_NU; }

int orc_num_h(const orc_problem *pr) { return pr->n_lin + pr->n_ell + pr->n_scen; }

void orc_h_bounds(const orc_problem *pr, double *lh, double *uh) {
    /* guidance_constraints.py:343-353: (-inf, 0]; ellipsoid_constraints.py:421-433: [1, inf) */
    for (int i = 0; i < pr->n_lin; i++) { lh[i] = -BIGBOUND; uh[i] = 0.0; }
    for (int j = 0; j < pr->n_ell; j++) { lh[pr->n_lin + j] = 1.0; uh[pr->n_lin + j] = BIGBOUND; }
    /* scenario_constraints.py:55-65: (-inf, 0] */
    for (int i = 0; i < pr->n_scen; i++) { lh[pr->n_lin + pr->n_ell + i] = -BIGBOUND; uh[pr->n_lin + pr->n_ell + i] = 0.0; }
}

void orc_stage_constraints(const orc_problem *pr, const double *z, const double *p,
                           double *h, double *jac, double *hess) {
    int nh = orc_num_h(pr);
    double x = z[NU + 0], y = z[NU + 1], psi = z[NU + 2];
    memset(jac, 0, sizeof(double) * nh * NZ);
    if (hess) memset(hess, 0, sizeof(double) * nh * NZ * NZ);
    /* topology halfspaces a1 x + a2 y - b <= 0 (guidance_constraints.py:355-370) */
    for (int i = 0; i < pr->n_lin; i++) {
        const double *c = p + pr->i_lin0 + 3 * i;
        h[i] = c[0] * x + c[1] * y - c[2];
        jac[i * NZ + NU + 0] = c[0];
        jac[i * NZ + NU + 1] = c[1];
    }
    /* obstacle ellipsoids d' R' D R d >= 1 (ellipsoid_constraints.py:435-489), one disc */
    double rd = pr->i_disc_r >= 0 ? p[pr->i_disc_r] : 0.0, off = pr->i_disc_off >= 0 ? p[pr->i_disc_off] : 0.0;
    double cp = cos(psi), sp = sin(psi);
    double dxp = -off * sp, dyp = off * cp;       /* d(disc)/dpsi */
    double dxpp = -off * cp, dypp = -off * sp;    /* d2(disc)/dpsi2 */
    for (int j = 0; j < pr->n_ell; j++) {
        const double *o = p + pr->i_ell0 + 7 * j;
        double chi = sqrt(o[5]);
        double ra = o[3] * chi + rd + o[6];
        double rb = o[4] * chi + rd + o[6];
        double D0 = 1.0 / (ra * ra), D1 = 1.0 / (rb * rb);
        double c = cos(o[2]), s = sin(o[2]);
        double M00 = c * c * D0 + s * s * D1;
        double M01 = -c * s * D0 + s * c * D1;
        double M11 = s * s * D0 + c * c * D1;
        double dx = x + off * cp - o[0];
        double dy = y + off * sp - o[1];
        double Mdx = M00 * dx + M01 * dy, Mdy = M01 * dx + M11 * dy;
        int r = pr->n_lin + j;
        h[r] = dx * Mdx + dy * Mdy;
        jac[r * NZ + NU + 0] = 2.0 * Mdx;
        jac[r * NZ + NU + 1] = 2.0 * Mdy;
        jac[r * NZ + NU + 2] = 2.0 * (Mdx * dxp + Mdy * dyp);
        if (hess) {
            double *Hr = hess + (size_t)r * NZ * NZ;
            Hr[(NU + 0) * NZ + NU + 0] = 2.0 * M00; Hr[(NU + 0) * NZ + NU + 1] = 2.0 * M01;
            Hr[(NU + 1) * NZ + NU + 0] = 2.0 * M01; Hr[(NU + 1) * NZ + NU + 1] = 2.0 * M11;
            double hxp = 2.0 * (M00 * dxp + M01 * dyp);
            double hyp = 2.0 * (M01 * dxp + M11 * dyp);
            Hr[(NU + 0) * NZ + NU + 2] = hxp; Hr[(NU + 2) * NZ + NU + 0] = hxp;
            Hr[(NU + 1) * NZ + NU + 2] = hyp; Hr[(NU + 2) * NZ + NU + 1] = hyp;
            Hr[(NU + 2) * NZ + NU + 2] = 2.0 * (dxp * (M00 * dxp + M01 * dyp) + dyp * (M01 * dxp + M11 * dyp)) +
                             2.0 * (Mdx * dxpp + Mdy * dypp);
        }
    }
    /* scenario halfspaces a1 xd + a2 yd - (b + slack) <= 0 at the disc position
     * (x, y) + R(psi) (offset, 0) (scenario_constraints.py:64-94); C3: the decomp
     * halfspaces, same formula (decomp_constraints.py:68-98) */
    for (int i = 0; i < pr->n_scen; i++) {
        const double *c = p + pr->i_scen0 + 3 * i;
        int r = pr->n_lin + pr->n_ell + i;
        double sl = (NX > 5) ? z[SLACK_IDX] : 0.0;
        h[r] = c[0] * (x + off * cp) + c[1] * (y + off * sp) - (c[2] + sl);
        jac[r * NZ + NU + 0] = c[0];
        jac[r * NZ + NU + 1] = c[1];
        jac[r * NZ + NU + 2] = c[0] * dxp + c[1] * dyp;
        if (NX > 5) jac[r * NZ + SLACK_IDX] = -1.0;
        if (hess) hess[(size_t)r * NZ * NZ + (NU + 2) * NZ + NU + 2] = c[0] * dxpp + c[1] * dypp;
    }
}

#ifndef ORC_BICYCLE_CA
/* ------------------------------------------------------------------ */
/* Dynamics (solver_model.py:207-214)                                  */
/* ------------------------------------------------------------------ */
void orc_dynamics(const double *z, double *f, double *jac, double *hess) {
    double a = z[0], w = z[1], psi = z[4], v = z[5];
    double c = cos(psi), s = sin(psi);
    f[0] = v * c; f[1] = v * s; f[2] = w; f[3] = a; f[4] = v;
    for (int i = 5; i < NX; i++) f[i] = 0.0; /* slack: constant (solver_model.py:287-294) */
    if (jac) {
        memset(jac, 0, sizeof(double) * NX * NZ);
        jac[0 * NZ + 4] = -v * s; jac[0 * NZ + 5] = c;
        jac[1 * NZ + 4] = v * c;  jac[1 * NZ + 5] = s;
        jac[2 * NZ + 1] = 1.0;
        jac[3 * NZ + 0] = 1.0;
        jac[4 * NZ + 5] = 1.0;
    }
    if (hess) {
        memset(hess, 0, sizeof(double) * NX * NZ * NZ);
        hess[0 * NZ * NZ + 4 * NZ + 4] = -v * c;
        hess[0 * NZ * NZ + 4 * NZ + 5] = -s; hess[0 * NZ * NZ + 5 * NZ + 4] = -s;
        hess[1 * NZ * NZ + 4 * NZ + 4] = -v * s;
        hess[1 * NZ * NZ + 4 * NZ + 5] = c; hess[1 * NZ * NZ + 5 * NZ + 4] = c;
    }
}

#endif

/* ------------------------------------------------------------------ */
/* acados ERK (4 stages, rk_steps steps) with forward sensitivities and */
/* the exact second-order adjoint (generate_acados_solver.py:148-150,   */
/* hessian_approx EXACT :155)                                           */
/* ------------------------------------------------------------------ */
#define ORC_MAX_EVAL 64
#define NXI ORC_NXI
/* ERK over the NXI integrated states (all of them except C3's spline state,
 * do_not_use_integration_for_last_n_states, solver_model.py:66-78, 366);
 * C3 then applies the CA spline update (model_discrete_dynamics) on top.
 * p: the stage parameters (read by the C3 update only, may be NULL otherwise). */
void orc_discrete(const orc_problem *pr, const double *z, const double *p, double *xnext, double *A,
                  double *B, const double *adj, double *hess) {
    int ns = pr->rk_steps;
    double h = pr->dt / ns;
    double y[NXI], S[NXI][NZ];
    static const double cst[4] = {0.0, 0.5, 0.5, 1.0};
    static const double wgt[4] = {1.0 / 6.0, 2.0 / 6.0, 2.0 / 6.0, 1.0 / 6.0};
    double W[ORC_MAX_EVAL][NZ];           /* f argument (z-order) of each evaluation */
    double Se[ORC_MAX_EVAL][NXI][NZ];     /* d(integrated state argument)/dz */
    double Je[ORC_MAX_EVAL][NXI][NZ];     /* df/dz' at the argument */
    for (int i = 0; i < NXI; i++) {
        y[i] = z[NU + i];
        for (int j = 0; j < NZ; j++) S[i][j] = (j == NU + i) ? 1.0 : 0.0;
    }
    int e = 0;
    for (int st = 0; st < ns; st++) {
        double k[4][NXI], dk[4][NXI][NZ];
        for (int q = 0; q < 4; q++, e++) {
            /* argument y + c_q h k_{q-1}; inputs and non-integrated states held */
            for (int i = 0; i < NU; i++) W[e][i] = z[i];
            for (int i = NXI; i < NX; i++) W[e][NU + i] = z[NU + i];
            for (int i = 0; i < NXI; i++) {
                W[e][NU + i] = y[i] + (q ? cst[q] * h * k[q - 1][i] : 0.0);
                for (int j = 0; j < NZ; j++)
                    Se[e][i][j] = S[i][j] + (q ? cst[q] * h * dk[q - 1][i][j] : 0.0);
            }
            double J[NXI * NZ];
            orc_dynamics(W[e], k[q], J, NULL);
            for (int i = 0; i < NXI; i++)
                for (int j = 0; j < NZ; j++) Je[e][i][j] = J[i * NZ + j];
            /* dk = Jx * Se + Ju * [I 0] (+ the held states' columns) */
            for (int i = 0; i < NXI; i++)
                for (int j = 0; j < NZ; j++) {
                    double acc = (j < NU) ? J[i * NZ + j] : 0.0;
                    for (int m = 0; m < NXI; m++) acc += J[i * NZ + NU + m] * Se[e][m][j];
                    for (int m = NXI; m < NX; m++) acc += (j == NU + m) ? J[i * NZ + NU + m] : 0.0;
                    dk[q][i][j] = acc;
                }
        }
        for (int i = 0; i < NXI; i++) {
            y[i] += h * (wgt[0] * k[0][i] + wgt[1] * k[1][i] + wgt[2] * k[2][i] + wgt[3] * k[3][i]);
            for (int j = 0; j < NZ; j++)
                S[i][j] += h * (wgt[0] * dk[0][i][j] + wgt[1] * dk[1][i][j] + wgt[2] * dk[2][i][j] + wgt[3] * dk[3][i][j]);
        }
    }
    for (int i = 0; i < NXI; i++) {
        xnext[i] = y[i];
        for (int j = 0; j < NX; j++) A[i * NX + j] = S[i][NU + j];
        for (int j = 0; j < NU; j++) B[i * NU + j] = S[i][j];
    }
    double yb[NXI];
    for (int i = 0; i < NXI; i++) yb[i] = adj ? adj[i] : 0.0;
#ifdef ORC_BICYCLE_CA
    /* the CA spline update g(z, I) at I = the integrated states (solver_model.py:409-437) */
    enum { NG = NZ + NXI };
    double gv, gg[NG], gh[NG * NG];
    orc_ca_update(pr, z, y, p, &gv, gg, (adj && hess) ? gh : NULL);
    xnext[NX - 1] = gv;
    for (int j = 0; j < NZ; j++) {
        double acc = gg[j];
        for (int i = 0; i < NXI; i++) acc += gg[NZ + i] * S[i][j];
        if (j < NU) B[(NX - 1) * NU + j] = acc;
        else A[(NX - 1) * NX + j - NU] = acc;
    }
    /* the update's own adjoint flows into the integrated states */
    if (adj)
        for (int i = 0; i < NXI; i++) yb[i] += adj[NX - 1] * gg[NZ + i];
#endif
    if (!adj || !hess) return;
    memset(hess, 0, sizeof(double) * NZ * NZ);
#ifdef ORC_BICYCLE_CA
    /* adj_s * Wg' Hess(g) Wg, Wg = d(z, I)/dz = [I_nz; S] */
    {
        double Wg[NG][NZ];
        for (int r = 0; r < NG; r++)
            for (int j = 0; j < NZ; j++) Wg[r][j] = r < NZ ? (r == j ? 1.0 : 0.0) : S[r - NZ][j];
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NZ; j++) {
                double acc = 0.0;
                for (int m = 0; m < NG; m++)
                    for (int n = 0; n < NG; n++) acc += Wg[m][i] * gh[m * NG + n] * Wg[n][j];
                hess[i * NZ + j] += adj[NX - 1] * acc;
            }
    }
#endif
    /* reverse sweep: ybar = adjoint of the step output; kbar_q = adjoint of k_q */
    for (int st = ns - 1; st >= 0; st--) {
        double kb[4][NXI];
        int e0 = 4 * st;
        for (int q = 3; q >= 0; q--) {
            for (int i = 0; i < NXI; i++) kb[q][i] = h * wgt[q] * yb[i];
            if (q < 3) { /* k_q feeds the argument of k_{q+1} with factor c_{q+1} h */
                for (int i = 0; i < NXI; i++) {
                    double acc = 0.0;
                    for (int m = 0; m < NXI; m++) acc += Je[e0 + q + 1][m][NU + i] * kb[q + 1][m];
                    kb[q][i] += cst[q + 1] * h * acc;
                }
            }
        }
        double ybn[NXI];
        for (int i = 0; i < NXI; i++) {
            double acc = yb[i];
            for (int q = 0; q < 4; q++)
                for (int m = 0; m < NXI; m++) acc += Je[e0 + q][m][NU + i] * kb[q][m];
            ybn[i] = acc;
        }
        /* second-order terms: sum_q We' Hess(kbar_q' f) We, We = d[u; y_arg; held]/dz */
        for (int q = 0; q < 4; q++) {
            int ee = e0 + q;
            double Hf[NXI * NZ * NZ], f[NXI], Hm[NZ][NZ], Wm[NZ][NZ];
            orc_dynamics(W[ee], f, NULL, Hf);
            for (int i = 0; i < NZ; i++)
                for (int j = 0; j < NZ; j++) {
                    double acc = 0.0;
                    for (int m = 0; m < NXI; m++) acc += kb[q][m] * Hf[m * NZ * NZ + i * NZ + j];
                    Hm[i][j] = acc;
                }
            for (int i = 0; i < NZ; i++)
                for (int j = 0; j < NZ; j++)
                    Wm[i][j] = (i < NU || i - NU >= NXI) ? (i == j ? 1.0 : 0.0) : Se[ee][i - NU][j];
            for (int i = 0; i < NZ; i++)
                for (int j = 0; j < NZ; j++) {
                    double acc = 0.0;
                    for (int m = 0; m < NZ; m++)
                        for (int n = 0; n < NZ; n++) acc += Wm[m][i] * Hm[m][n] * Wm[n][j];
                    hess[i * NZ + j] += acc;
                }
        }
        memcpy(yb, ybn, sizeof yb);
    }
}

void orc_erk4(const orc_problem *pr, const double *z, double *xnext, double *A, double *B,
              const double *adj, double *hess) {
    orc_discrete(pr, z, NULL, xnext, A, B, adj, hess);
}

/* ------------------------------------------------------------------ */
/* MIRROR regularisation (regularize_method "MIRROR",                  */
/* generate_acados_solver.py:157): H = V f(D) V', f(d)=eps if |d|<=eps  */
/* else |d|.  Eigen-decomposition by cyclic Jacobi.                     */
/* ------------------------------------------------------------------ */
void orc_mirror(int n, double *H, double eps) {
    double a[NZ][NZ], V[NZ][NZ], d[NZ];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            a[i][j] = 0.5 * (H[i * n + j] + H[j * n + i]);
            V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 50; sweep++) {
        double off = 0.0, dia = 0.0;
        for (int i = 0; i < n; i++) {
            dia += a[i][i] * a[i][i];
            for (int j = i + 1; j < n; j++) off += a[i][j] * a[i][j];
        }
        if (off <= 1e-32 * dia || off < 1e-300) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                double apq = a[p][q];
                if (fabs(apq) < 1e-300) continue;
                double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
                double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; k++) { /* columns p, q */
                    double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) { /* rows p, q */
                    double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < n; i++) {
        double di = a[i][i];
        if (di >= -eps && di <= eps) di = eps;
        else if (di < 0.0) di = -di;
        d[i] = di;
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double acc = 0.0;
            for (int k = 0; k < n; k++) acc += V[i][k] * d[k] * V[j][k];
            H[i * n + j] = acc;
        }
}

/* Arithmetic forms: three builds of the same interior-point algorithm that differ only in
 * rounding (which operation forms and which summation order).  They matter only where an
 * exit decision rests on rounding (C5's dual-degenerate QPs, DESIGN.md §3.2: the
 * convergence test there reads a residual made of cancelling multipliers of 1e13 and more).
 *
 * ORC_FORMS 1 (default): HPIPM's / BLASFEO's own forms, none taken from the GPU kernel
 *   (HPIPM and BLASFEO are acados submodules at a commit the reference does not pin; the
 *   forms are restated from their published sources, version unpinned):
 *   - Cholesky of the input block as BLASFEO's dpotrf_l: l_jj = sqrt(d), inv_diag_j =
 *     1 / l_jj, sub-diagonal entries and the triangular solves multiplied by inv_diag;
 *   - barrier terms through t_inv = 1 / t (HPIPM compute_Gamma_gamma: Gamma = t_inv lam);
 *   - the row residual res_d = D.dz + t - d (HPIPM res_compute: the constraint product
 *     first, then t and d added);
 *   - the step to the boundary as HPIPM compute_alpha: alpha = min over rows of -t/dt and
 *     -lam/dlam (one division per blocking row);
 *   - the stationarity residual in HPIPM's evaluation order, res_g = (H dz + g) + (lam_u -
 *     lam_l) on the box rows + D' lam of the general rows (row order) + [B A]' pi - pi_prev
 *     (BLASFEO's gemv kernels block the sums by four; that association is not restated).
 * ORC_FORMS 0 (-DORC_LITERAL): the literal forms -- divisions, row-order sums -- the second
 *   kernel-agnostic build.
 * ORC_FORMS 2 (-DORC_KERNEL_FORMS, diagnostic only): the GPU kernel's forms, including its
 *   wavefront layout (the 2x2 pivot's 1/l11 = l00 / sqrt(det), 1 / max(-dt/t, -dl/l), the
 *   h rows' stationarity sums folded per lane part).  Not used as the parity reference: a
 *   build that copies the kernel's association is partly self-agreement.
 * Records: scripts/parity_full.py (rounding-decided = the two kernel-agnostic builds part),
 * tests/test_rounding_record.py. */
#if defined(ORC_LITERAL)
#define ORC_FORMS 0
#elif defined(ORC_KERNEL_FORMS)
#define ORC_FORMS 2
#else
#define ORC_FORMS 1
#endif
#define KF (ORC_FORMS >= 1) /* t_inv, res_d = D.dz + t - d, inv_diag Cholesky (HPIPM / BLASFEO) */
#define KK (ORC_FORMS == 2) /* the kernel's own forms */

/* ------------------------------------------------------------------ */
/* OCP-QP: Riccati-based Mehrotra primal-dual interior point            */
/* (PARTIAL_CONDENSING_HPIPM with cond_N = N, qp_tol 1e-5, iter_max 50:  */
/* generate_acados_solver.py:162-173).  Inequalities D z <= d, one      */
/* sided; +-1e15 bounds are dropped.  x0 is eliminated (fixed).         */
/* ------------------------------------------------------------------ */
typedef struct {
    double H[NZ][NZ], g[NZ];
    double A[NX][NX], B[NX][NU], b[NX];
    int ni;
    double (*D)[NZ];
    double *d, *t, *lam, *dt, *dl, *dt_aff, *dl_aff, *rin, *rc;
    int *hrow; /* >=0: index of the h-row this inequality came from (sign in hsgn) */
    int *hsgn;
    /* Riccati storage */
    double L[NU][NU], Y[NU][NX], P[NX][NX], p[NX], y[NU];
    double il[NU];  /* reciprocal pivots 1/L_ii (default build, nu 2) */
    /* square-root Riccati (qp_ric_alg 1): the state block of the stage's Cholesky factor, P = Lx Lx' */
    double Lx[NX][NX];
    double Hh[NZ][NZ], q[NZ];
    double dz[NZ], ddz[NZ], pi[NX], pin[NX];
    /* iterative refinement (qp_itref_corr_max): the iterate's stationarity residual, the
     * linear KKT residual of the step (stationarity, dynamics; rows in ld / lm) and the
     * unrefined step */
    double rg[NZ], lg[NZ], lb[NX], ddz0[NZ], pin0[NX];
    double *ld, *lm;
} qp_stage;

typedef struct {
    int N;
    qp_stage *st; /* N+1 */
    /* the Riccati recursion's form and its pivot rule (orc_problem.qp_ric_alg, qp_pivot_zero), and
     * HPIPM's lq_fact switch: lq_fact 1 -> after an inaccurate Cholesky factorisation (the predictor's
     * linear residual above 1e-5) the QP's remaining factorisations are LQ ones (force_lq) */
    int ric_sqrt, pivot_zero, lq_fact, force_lq;
} qp_ws;

/* stationarity residual of stage k on its free variables */
static void qp_residuals(qp_ws *w, double *rs, double *re, double *ri, double *mu, int *mtot, double *cmx) {
    int N = w->N;
    double s_max = 0.0, e_max = 0.0, i_max = 0.0, comp = 0.0, c_max = 0.0;
    int m = 0;
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w->st[k];
        double r[NZ];
        for (int i = 0; i < NZ; i++) {
            double acc = S->g[i];
            for (int j = 0; j < NZ; j++) acc += S->H[i][j] * S->dz[j];
            r[i] = acc;
        }
        if (k < N) {
            for (int i = 0; i < NZ; i++) {
                double acc = 0.0;
                for (int m2 = 0; m2 < NX; m2++)
                    acc += (i < NU ? S->B[m2][i] : S->A[m2][i - NU]) * S->pi[m2];
                r[i] += acc;
            }
        }
        if (k > 0)
            for (int i = 0; i < NX; i++) r[NU + i] -= w->st[k - 1].pi[i];
        for (int c = 0; c < S->ni; c++) {
            for (int i = 0; i < NZ; i++) r[i] += S->D[c][i] * S->lam[c];
            double acc;
            if (KF) {
                /* kernel: rin = D.dz + t - gap */
                double dd = 0.0;
                for (int i = 0; i < NZ; i++) dd += S->D[c][i] * S->dz[i];
                acc = dd + S->t[c] - S->d[c];
            } else {
                acc = S->t[c] - S->d[c];
                for (int i = 0; i < NZ; i++) acc += S->D[c][i] * S->dz[i];
            }
            S->rin[c] = acc;
            if (fabs(acc) > i_max) i_max = fabs(acc);
            comp += S->lam[c] * S->t[c];
            if (fabs(S->lam[c] * S->t[c]) > c_max) c_max = fabs(S->lam[c] * S->t[c]);
            m++;
        }
        if (KF) {
            /* box multipliers as upper - lower per variable (HPIPM res_compute: lam_u - lam_l,
             * added at the box index) */
            double rbox[NZ];
            for (int i = 0; i < NZ; i++) {
                double lo = 0.0, hi = 0.0;
                for (int c = 0; c < S->ni; c++)
                    if (S->hrow[c] < 0 && S->D[c][i] != 0.0) { if (S->D[c][i] > 0) hi = S->lam[c]; else lo = S->lam[c]; }
                rbox[i] = hi - lo;
            }
            if (KK) {
                /* diagnostic kernel-forms build: (H dz + g) + (box + the h rows' sums per lane
                 * part folded part 0 + part 1 + part 2), then + F' pi term by term, - pi_prev */
#ifdef ORC_BICYCLE_CA
                const int parts = 2; /* the kernel's bicycle instances run two parts (MPCG_PARTS_BIKE) */
#else
                const int parts = (64 / (N + 1)) >= 3 ? 3 : 2; /* Cfg::PARTS_MAX */
#endif
                double rh[3][NZ];
                memset(rh, 0, sizeof rh);
                for (int c = 0; c < S->ni; c++) {
                    if (S->hrow[c] < 0) continue;
                    const int pp = S->hrow[c] % parts;
                    for (int i = 0; i < NZ; i++) rh[pp][i] += S->D[c][i] * S->lam[c];
                }
                for (int i = 0; i < NZ; i++) {
                    double acc = rh[0][i];
                    for (int pp = 1; pp < parts; pp++) acc += rh[pp][i];
                    rbox[i] += acc;
                }
                for (int i = 0; i < NZ; i++) {
                    double a = 0.0;
                    for (int j = 0; j < NZ; j++) a += S->H[i][j] * S->dz[j];
                    r[i] = a + S->g[i] + rbox[i];
                }
            } else {
                /* HPIPM's order: res_g = (H dz + g) (BLASFEO symv: the product, then beta y),
                 * + box, + D' lam over the general rows in row order */
                for (int i = 0; i < NZ; i++) {
                    double a = 0.0;
                    for (int j = 0; j < NZ; j++) a += S->H[i][j] * S->dz[j];
                    r[i] = a + S->g[i] + rbox[i];
                }
                for (int c = 0; c < S->ni; c++) {
                    if (S->hrow[c] < 0) continue;
                    for (int i = 0; i < NZ; i++) r[i] += S->D[c][i] * S->lam[c];
                }
            }
            if (k < N)
                for (int m2 = 0; m2 < NX; m2++)
                    for (int i = 0; i < NZ; i++) r[i] += (i < NU ? S->B[m2][i] : S->A[m2][i - NU]) * S->pi[m2];
            if (k > 0)
                for (int i = 0; i < NX; i++) r[NU + i] -= w->st[k - 1].pi[i];
        }
        int i0 = (k == N) ? NU : 0, i1 = (k == 0) ? NU : NZ;
        for (int i = i0; i < i1; i++)
            if (fabs(r[i]) > s_max) s_max = fabs(r[i]);
        memcpy(S->rg, r, sizeof r);
        if (getenv("ORC_DEBUG3")) {
            for (int i = i0; i < i1; i++) {
                if (fabs(r[i]) < 1e-7) continue;
                double hz = 0.0, dl = 0.0, fp = 0.0, bx = 0.0, mx = 0.0;
                for (int j = 0; j < NZ; j++) hz += S->H[i][j] * S->dz[j];
                for (int c = 0; c < S->ni; c++) { double v = S->D[c][i] * S->lam[c]; if (S->hrow[c] < 0) bx += v; else dl += v; if (fabs(v) > mx) mx = fabs(v); }
                if (k < N) for (int m2 = 0; m2 < NX; m2++) fp += (i < NU ? S->B[m2][i] : S->A[m2][i - NU]) * S->pi[m2];
                double pp = (k > 0 && i >= NU) ? w->st[k - 1].pi[i - NU] : 0.0;
                fprintf(stderr, "      k %d var %d r %.3e | Hdz %.6e g %.6e box %.6e hrows %.6e (max term %.3e) Fpi %.6e pprev %.6e\n", k, i, r[i], hz, S->g[i], bx, dl, mx, fp, pp);
            }
        }
        if (k < N) {
            qp_stage *S1 = &w->st[k + 1];
            for (int i = 0; i < NX; i++) {
                double acc = S->b[i] - S1->dz[NU + i];
                for (int j = 0; j < NX; j++) acc += S->A[i][j] * S->dz[NU + j];
                for (int j = 0; j < NU; j++) acc += S->B[i][j] * S->dz[j];
                if (fabs(acc) > e_max) e_max = fabs(acc);
            }
        }
    }
    *rs = s_max; *re = e_max; *ri = i_max;
    *mtot = m;
    *mu = m ? comp / m : 0.0;
    *cmx = c_max;
}

/* dynamics residual r_k = A dx_k + B du_k + b_k - dx_{k+1} */
static void dyn_res(qp_ws *w, int k, double r[NX]) {
    qp_stage *S = &w->st[k], *S1 = &w->st[k + 1];
    for (int i = 0; i < NX; i++) {
        double acc = S->b[i] - S1->dz[NU + i];
        for (int j = 0; j < NX; j++) acc += S->A[i][j] * S->dz[NU + j];
        for (int j = 0; j < NU; j++) acc += S->B[i][j] * S->dz[j];
        r[i] = acc;
    }
}

/* BLASFEO dpotrf_l of the leading n x n block of M (row stride NZ) into L, with the inverse diagonal
 * in il: column j's pivot d = M_jj - sum_m L_jm^2; d > 0: L_jj = sqrt(d), il_j = 1 / L_jj, else (with
 * pivot_zero) L_jj = il_j = 0 -- the column below is multiplied by il_j, so a non-positive pivot zeroes
 * its column and the factorisation goes on.  literal: divisions by L_jj instead of the inverse (a zero
 * pivot then gives a zero column too).  Returns -1 on a non-positive pivot without pivot_zero. */
static int potrf_l(int n, double (*M)[NZ], double (*L)[NZ], double *il, int pivot_zero) {
    for (int j = 0; j < n; j++) {
        double d = M[j][j];
        for (int m = 0; m < j; m++) d -= L[j][m] * L[j][m];
        double ljj = 0.0, inv = 0.0;
        if (d > 0.0) {
            ljj = sqrt(d);
            inv = 1.0 / ljj;
        } else if (!pivot_zero) {
            return -1;
        }
        L[j][j] = ljj;
        il[j] = inv;
        for (int i = j + 1; i < n; i++) {
            double acc = M[i][j];
            for (int m = 0; m < j; m++) acc -= L[i][m] * L[j][m];
            L[i][j] = KF ? acc * inv : (ljj != 0.0 ? acc / ljj : 0.0);
        }
        for (int i = 0; i < j; i++) L[i][j] = 0.0;
    }
    return 0;
}

static void lq_stage(qp_stage *S, const qp_stage *S1, int terminal, double (*L)[NZ]);

/* Square-root Riccati factorisation (HPIPM square_root_alg 1, which acados selects by default:
 * acados_template's qp_solver_ric_alg 1 -- restated, version unpinned): the cost-to-go
 * is carried as its Cholesky factor, P_k = Lx_k Lx_k'.  Per stage, AL = F_k' Lx_{k+1} (BLASFEO
 * dtrmm_rlnn), M = Hh_k + AL AL' (dsyrk), and one Cholesky of the whole nz x nz block M (dpotrf_l):
 * its input block gives L and the inverse pivots, its off-diagonal block Y' = Lxu, its state block
 * Lx_k.  The terminal stage factorises its state block.  With pivot_zero a non-positive pivot -- of the
 * input or of the state block -- continues with a zero column (BLASFEO); P is also formed (Lx Lx') for
 * the diagnostics that read it. */
static int riccati_factor_sqrt(qp_ws *w) {
    int N = w->N;
    qp_stage *SN = &w->st[N];
    {
        double M[NZ][NZ], L[NZ][NZ], il[NZ];
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) M[i][j] = SN->Hh[NU + i][NU + j];
        if (w->force_lq) lq_stage(SN, NULL, 1, L);
        else if (potrf_l(NX, M, L, il, w->pivot_zero)) return -1;
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) SN->Lx[i][j] = L[i][j];
    }
    for (int k = N - 1; k >= 0; k--) {
        qp_stage *S = &w->st[k], *S1 = &w->st[k + 1];
        double AL[NZ][NX], M[NZ][NZ], L[NZ][NZ], il[NZ];
        /* AL = BAbt Lx_{k+1}: BAbt[i][m] = F[m][i], Lx lower triangular */
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NX; j++) {
                double acc = 0.0;
                for (int m = j; m < NX; m++) acc += (i < NU ? S->B[m][i] : S->A[m][i - NU]) * S1->Lx[m][j];
                AL[i][j] = acc;
            }
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j <= i; j++) {
                double acc = 0.0;
                for (int m = 0; m < NX; m++) acc += AL[i][m] * AL[j][m];
                M[i][j] = S->Hh[i][j] + acc;
                M[j][i] = M[i][j];
            }
        if (w->force_lq) {
            lq_stage(S, S1, 0, L);
            for (int i = 0; i < NZ; i++) il[i] = 1.0 / L[i][i];
        } else if (potrf_l(NZ, M, L, il, w->pivot_zero)) {
            return -1;
        }
        for (int i = 0; i < NU; i++) {
            for (int j = 0; j < NU; j++) S->L[i][j] = L[i][j];
            S->il[i] = il[i];
        }
        for (int i = 0; i < NU; i++)
            for (int j = 0; j < NX; j++) S->Y[i][j] = L[NU + j][i];
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) S->Lx[i][j] = L[NU + i][NU + j];
    }
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w->st[k];
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) {
                double acc = 0.0;
                for (int m = 0; m <= (i < j ? i : j); m++) acc += S->Lx[i][m] * S->Lx[j][m];
                S->P[i][j] = acc;
            }
    }
    return 0;
}

/* Lower-triangular L with positive diagonal and L L' = W W' for the n x m (m >= n) matrix W (row stride
 * ld): Householder LQ (LAPACK dgelqf's reflections, the diagonal made positive as HPIPM's _pd kernels
 * return it).  The factor the Cholesky of W W' would give, without forming W W' -- no cancellation, no
 * failing pivot */
static void lq_lower(int n, int m, double *W, int ld, double (*L)[NZ]) {
    for (int i = 0; i < n; i++) {
        double *wi = W + (size_t)i * ld;
        double nrm = 0.0;
        for (int j = i; j < m; j++) nrm += wi[j] * wi[j];
        nrm = sqrt(nrm);
        if (nrm > 0.0) {
            const double alpha = wi[i] > 0.0 ? -nrm : nrm;
            /* v = w_i[i:] - alpha e_0, H = I - 2 v v' / (v' v); applied to rows i..n-1 from the right */
            double v[ORC_MAX_NZW];
            double vv = 0.0;
            for (int j = i; j < m; j++) { v[j] = wi[j] - (j == i ? alpha : 0.0); vv += v[j] * v[j]; }
            if (vv > 0.0) {
                for (int r = i; r < n; r++) {
                    double *wr = W + (size_t)r * ld;
                    double dot = 0.0;
                    for (int j = i; j < m; j++) dot += wr[j] * v[j];
                    const double f = 2.0 * dot / vv;
                    for (int j = i; j < m; j++) wr[j] -= f * v[j];
                }
            }
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < NZ; j++) L[i][j] = 0.0;
    for (int j = 0; j < n; j++) {
        const double s = W[(size_t)j * ld + j] < 0.0 ? -1.0 : 1.0;  /* positive diagonal: flip column j */
        for (int i = j; i < n; i++) L[i][j] = s * W[(size_t)i * ld + j];
    }
}

/* HPIPM's LQ factorisation of one stage (d_ocp_qp_fact_lq_solve_kkt_step, square-root form): the stage's
 * factor from the wide matrix [chol(H_k) | sqrt(lam_c / t_c) D_c' for every inequality row | F_k' Lx_{k+1}]
 * (the Hessian's Cholesky, the barrier of each row, the propagated cost-to-go factor): L L' = M as in the
 * Cholesky path, computed without forming M.  n = nz (k < N) or nx (stage N, its state block, no rows) */
static void lq_stage(qp_stage *S, const qp_stage *S1, int terminal, double (*L)[NZ]) {
    const int n = terminal ? NX : NZ, off = terminal ? NU : 0;
    double Hs[NZ][NZ], Lh[NZ][NZ], il[NZ];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) Hs[i][j] = S->H[off + i][off + j];
    potrf_l(n, Hs, Lh, il, 1);
    const int m = n + (terminal ? 0 : S->ni) + (terminal ? 0 : NX);
    static __thread double W[NZ * ORC_MAX_NZW];
    for (int i = 0; i < n; i++) {
        double *wi = W + (size_t)i * ORC_MAX_NZW;
        for (int j = 0; j < m; j++) wi[j] = 0.0;
        for (int j = 0; j <= i; j++) wi[j] = Lh[i][j];
    }
    if (!terminal) {
        for (int c = 0; c < S->ni; c++) {
            const double sw = sqrt(S->lam[c] * (1.0 / S->t[c]));
            for (int i = 0; i < NZ; i++) W[(size_t)i * ORC_MAX_NZW + n + c] = S->D[c][i] * sw;
        }
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NX; j++) {
                double acc = 0.0;
                for (int q = j; q < NX; q++) acc += (i < NU ? S->B[q][i] : S->A[q][i - NU]) * S1->Lx[q][j];
                W[(size_t)i * ORC_MAX_NZW + n + S->ni + j] = acc;
            }
    }
    lq_lower(n, m, W, ORC_MAX_NZW, L);
}

/* P_{k} v as the square-root form applies it: Lx (Lx' v) (BLASFEO dtrmv_ltn, then dtrmv_lnn) */
static void lx_apply(const qp_stage *S, const double *v, double *out) {
    double t[NX];
    for (int i = 0; i < NX; i++) {
        double acc = 0.0;
        for (int m = i; m < NX; m++) acc += S->Lx[m][i] * v[m];
        t[i] = acc;
    }
    for (int i = 0; i < NX; i++) {
        double acc = 0.0;
        for (int m = 0; m <= i; m++) acc += S->Lx[i][m] * t[m];
        out[i] = acc;
    }
}

/* Riccati factorisation of the barrier-augmented Hessians Hh. returns 0 ok */
static int riccati_factor(qp_ws *w) {
    if (w->ric_sqrt) return riccati_factor_sqrt(w);
    int N = w->N;
    qp_stage *SN = &w->st[N];
    for (int i = 0; i < NX; i++)
        for (int j = 0; j < NX; j++) SN->P[i][j] = SN->Hh[NU + i][NU + j];
    for (int k = N - 1; k >= 0; k--) {
        qp_stage *S = &w->st[k], *S1 = &w->st[k + 1];
        double F[NX][NZ], PF[NX][NZ], M[NZ][NZ];
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NZ; j++) F[i][j] = (j < NU) ? S->B[i][j] : S->A[i][j - NU];
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NZ; j++) {
                double acc = 0.0;
                for (int m = 0; m < NX; m++) acc += S1->P[i][m] * F[m][j];
                PF[i][j] = acc;
            }
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NZ; j++) {
                double acc = S->Hh[i][j];
                for (int m = 0; m < NX; m++) acc += F[m][i] * PF[m][j];
                M[i][j] = acc;
            }
        if (KK && NU == 2) {
            /* kernel forms: both reciprocal square roots from the block entries,
             * 1/l11 = l00 / sqrt(m00 m11 - m10^2) */
            const double m00 = M[0][0], m10 = M[1][0], m11 = M[1][1];
            const double det = fma(m00, m11, -(m10 * m10));
            if (!w->pivot_zero && (!(m00 > 0.0) || !(det > 0.0))) return -1;
            /* pivot_zero: the kernel's BLASFEO rule -- a non-positive first pivot gives a zero first
             * column (l10 = 0, the second pivot is then m11 itself); a non-positive second pivot
             * (det / m00 <= 0) a zero second column */
            const double il00 = m00 > 0.0 ? 1.0 / sqrt(m00) : 0.0;
            const double l00 = m00 * il00;
            const double il11 = m00 > 0.0 ? (det > 0.0 ? l00 * (1.0 / sqrt(det)) : 0.0) : (m11 > 0.0 ? 1.0 / sqrt(m11) : 0.0);
            S->L[0][0] = l00; S->L[1][0] = m10 * il00; S->L[0][1] = 0.0;
            S->il[0] = il00; S->il[1] = il11;
            S->L[1][1] = il11 != 0.0 ? 1.0 / il11 : 0.0;
            for (int j = 0; j < NX; j++) {
                S->Y[0][j] = M[0][NU + j] * S->il[0];
                S->Y[1][j] = (M[1][NU + j] - S->L[1][0] * S->Y[0][j]) * S->il[1];
            }
            for (int i = 0; i < NX; i++)
                for (int j = 0; j < NX; j++)
                    S->P[i][j] = M[NU + i][NU + j] - S->Y[0][i] * S->Y[0][j] - S->Y[1][i] * S->Y[1][j];
            continue;
        }
        /* Cholesky of Muu (L L' = Muu).  HPIPM forms: BLASFEO dpotrf_l (sqrt, inv_diag = 1 /
         * l_jj, entries multiplied by inv_diag); kernel forms: inv_diag = 1 / sqrt(d) first,
         * l_jj = d inv_diag; literal: sqrt and divisions.  A pivot <= 0 fails the QP (NaN
         * status): BLASFEO would continue with a zero inverse, DESIGN.md §2.2. */
        for (int j = 0; j < NU; j++) {
            double d = M[j][j];
            for (int m = 0; m < j; m++) d -= S->L[j][m] * S->L[j][m];
            if (!(d > 0.0) && w->pivot_zero) {
                /* BLASFEO dpotrf's non-positive pivot: zero diagonal, zero inverse, the column below
                 * multiplied by that zero; the factorisation goes on */
                S->L[j][j] = 0.0;
                S->il[j] = 0.0;
                for (int i = j + 1; i < NU; i++) S->L[i][j] = 0.0;
                for (int i = 0; i < j; i++) S->L[i][j] = 0.0;
                continue;
            }
            if (!(d > 0.0)) return -1;
            if (KK) {
                S->il[j] = 1.0 / sqrt(d);
                d = d * S->il[j];
            } else {  /* (a positive pivot here: the non-positive ones took the zero column above) */
                d = sqrt(d);
                S->il[j] = 1.0 / d;
            }
            S->L[j][j] = d;
            for (int i = j + 1; i < NU; i++) {
                double acc = M[i][j];
                for (int m = 0; m < j; m++) acc -= S->L[i][m] * S->L[j][m];
                S->L[i][j] = KF ? acc * S->il[j] : acc / d;
            }
            for (int i = 0; i < j; i++) S->L[i][j] = 0.0;
        }
        /* Y = L^{-1} Mux */
        for (int j = 0; j < NX; j++)
            for (int i = 0; i < NU; i++) {
                double acc = M[i][NU + j];
                for (int m = 0; m < i; m++) acc -= S->L[i][m] * S->Y[m][j];
                S->Y[i][j] = KF ? acc * S->il[i] : (S->L[i][i] != 0.0 ? acc / S->L[i][i] : 0.0);
            }
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) {
                double acc = M[NU + i][NU + j];
                for (int m = 0; m < NU; m++) acc -= S->Y[m][i] * S->Y[m][j];
                S->P[i][j] = acc;
            }
    }
    return 0;
}

/* vector pass + forward substitution for gradient q (in S->q) and the
 * current dynamics residuals; writes ddz (step) and pin (new dynamics
 * multipliers) */
static void riccati_solve_r(qp_ws *w, double (*r)[NX]);
static void riccati_solve(qp_ws *w) {
    double r[ORC_MAX_N][NX];
    for (int k = 0; k < w->N; k++) dyn_res(w, k, r[k]);
    riccati_solve_r(w, r);
}

/* the same for the dynamics right-hand sides r (the iterative refinement's) */
static void riccati_solve_r(qp_ws *w, double (*r)[NX]) {
    int N = w->N;
    qp_stage *SN = &w->st[N];
    for (int i = 0; i < NX; i++) SN->p[i] = SN->q[NU + i];
    for (int k = N - 1; k >= 0; k--) {
        qp_stage *S = &w->st[k], *S1 = &w->st[k + 1];
        double v[NX], m[NZ];
        if (w->ric_sqrt) {
            /* HPIPM (square root): Lx (Lx' b) + p */
            double Pb[NX];
            lx_apply(S1, r[k], Pb);
            for (int i = 0; i < NX; i++) v[i] = Pb[i] + S1->p[i];
        } else {
            for (int i = 0; i < NX; i++) {
                double acc = S1->p[i];
                for (int j = 0; j < NX; j++) acc += S1->P[i][j] * r[k][j];
                v[i] = acc;
            }
        }
        for (int i = 0; i < NZ; i++) {
            double acc = S->q[i];
            for (int j = 0; j < NX; j++) acc += (i < NU ? S->B[j][i] : S->A[j][i - NU]) * v[j];
            m[i] = acc;
        }
        for (int i = 0; i < NU; i++) { /* y = L^{-1} m_u */
            double acc = m[i];
            for (int q = 0; q < i; q++) acc -= S->L[i][q] * S->y[q];
            S->y[i] = KF ? acc * S->il[i] : (S->L[i][i] != 0.0 ? acc / S->L[i][i] : 0.0);
        }
        for (int i = 0; i < NX; i++) {
            double acc = m[NU + i];
            for (int q = 0; q < NU; q++) acc -= S->Y[q][i] * S->y[q];
            S->p[i] = acc;
        }
    }
    /* forward */
    double dx[NX] = {0};
    for (int k = 0; k < N; k++) {
        qp_stage *S = &w->st[k], *S1 = &w->st[k + 1];
        /* du = -L^{-T} (Y dx + y) */
        double c[NU], du[NU];
        for (int i = 0; i < NU; i++) {
            c[i] = S->y[i];
            for (int j = 0; j < NX; j++) c[i] += S->Y[i][j] * dx[j];
        }
        for (int i = NU - 1; i >= 0; i--) { /* L' du = -c */
            double acc = -c[i];
            for (int q = i + 1; q < NU; q++) acc -= S->L[q][i] * du[q];
            du[i] = KF ? acc * S->il[i] : (S->L[i][i] != 0.0 ? acc / S->L[i][i] : 0.0);
        }
        for (int i = 0; i < NU; i++) S->ddz[i] = du[i];
        for (int i = 0; i < NX; i++) S->ddz[NU + i] = (k == 0) ? 0.0 : dx[i];
        double dxn[NX];
        for (int i = 0; i < NX; i++) {
            double acc = r[k][i];
            for (int j = 0; j < NU; j++) acc += S->B[i][j] * du[j];
            for (int j = 0; j < NX; j++) acc += S->A[i][j] * dx[j];
            dxn[i] = acc;
        }
        if (w->ric_sqrt) {
            double Pd[NX];
            lx_apply(S1, dxn, Pd);
            for (int i = 0; i < NX; i++) S->pin[i] = Pd[i] + S1->p[i];
        } else {
            for (int i = 0; i < NX; i++) {
                double acc = S1->p[i];
                for (int j = 0; j < NX; j++) acc += S1->P[i][j] * dxn[j];
                S->pin[i] = acc;
            }
        }
        memcpy(dx, dxn, sizeof dx);
    }
    for (int i = 0; i < NU; i++) SN->ddz[i] = 0.0;
    for (int i = 0; i < NX; i++) SN->ddz[NU + i] = dx[i];
}

/* gradient of the Newton system for complementarity targets rc */
static void build_q(qp_ws *w) {
    for (int k = 0; k <= w->N; k++) {
        qp_stage *S = &w->st[k];
        for (int i = 0; i < NZ; i++) {
            double acc = S->g[i];
            for (int j = 0; j < NZ; j++) acc += S->H[i][j] * S->dz[j];
            S->q[i] = acc;
        }
        for (int c = 0; c < S->ni; c++) {
            double coef = KF ? S->lam[c] + (S->lam[c] * S->rin[c] - S->rc[c]) * (1.0 / S->t[c])
                             : S->lam[c] + (S->lam[c] * S->rin[c] - S->rc[c]) / S->t[c];
            for (int i = 0; i < NZ; i++) S->q[i] += S->D[c][i] * coef;
        }
    }
}

static void ineq_steps(qp_ws *w, double *dtv_unused) {
    (void)dtv_unused;
    for (int k = 0; k <= w->N; k++) {
        qp_stage *S = &w->st[k];
        for (int c = 0; c < S->ni; c++) {
            double acc = 0.0;
            for (int i = 0; i < NZ; i++) acc += S->D[c][i] * S->ddz[i];
            S->dt[c] = -S->rin[c] - acc;
            S->dl[c] = KF ? -(S->rc[c] + S->lam[c] * S->dt[c]) * (1.0 / S->t[c])
                          : -(S->rc[c] + S->lam[c] * S->dt[c]) / S->t[c];
        }
    }
}

static double max_step(qp_ws *w) {
    if (KK) {
        /* kernel forms: 1 / max over rows of -dt/t and -dl/l */
        double rmax = 0.0;
        for (int k = 0; k <= w->N; k++) {
            qp_stage *S = &w->st[k];
            for (int c = 0; c < S->ni; c++) {
                double a = -S->dt[c] * (1.0 / S->t[c]);
                if (a > rmax) rmax = a;
                if (S->dl[c] < 0.0) { a = -S->dl[c] * (1.0 / S->lam[c]); if (a > rmax) rmax = a; }
            }
        }
        return rmax > 0.0 ? 1.0 / rmax : 1e300;
    }
    double amax = 1e300;
    for (int k = 0; k <= w->N; k++) {
        qp_stage *S = &w->st[k];
        for (int c = 0; c < S->ni; c++) {
            if (S->dt[c] < 0.0) { double a = -S->t[c] / S->dt[c]; if (a < amax) amax = a; }
            if (S->dl[c] < 0.0) { double a = -S->lam[c] / S->dl[c]; if (a < amax) amax = a; }
        }
    }
    return amax;
}

/* linear residual of the Newton system for the step (ddz, pin - pi, dt, dl) against its
 * right-hand side (the iterate's rg, dynamics residual, rin, rc) -- HPIPM res_compute_lin --
 * into lg / lb / ld / lm; res[0..3] = inf-norms (stationarity on the free variables, dynamics,
 * rows, complementarity) */
static void lin_residuals(qp_ws *w, double res[4]) {
    int N = w->N;
    res[0] = res[1] = res[2] = res[3] = 0.0;
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w->st[k];
        double r[NZ];
        for (int i = 0; i < NZ; i++) {
            double acc = S->rg[i];
            for (int j = 0; j < NZ; j++) acc += S->H[i][j] * S->ddz[j];
            r[i] = acc;
        }
        for (int c = 0; c < S->ni; c++) {
            for (int i = 0; i < NZ; i++) r[i] += S->D[c][i] * S->dl[c];
            double dd = 0.0;
            for (int i = 0; i < NZ; i++) dd += S->D[c][i] * S->ddz[i];
            S->ld[c] = S->rin[c] + dd + S->dt[c];
            S->lm[c] = S->rc[c] + S->lam[c] * S->dt[c] + S->t[c] * S->dl[c];
            if (fabs(S->ld[c]) > res[2] || isnan(S->ld[c])) res[2] = fabs(S->ld[c]);
            if (fabs(S->lm[c]) > res[3] || isnan(S->lm[c])) res[3] = fabs(S->lm[c]);
        }
        if (k < N)
            for (int i = 0; i < NZ; i++)
                for (int m = 0; m < NX; m++)
                    r[i] += (i < NU ? S->B[m][i] : S->A[m][i - NU]) * (S->pin[m] - S->pi[m]);
        if (k > 0)
            for (int i = 0; i < NX; i++) r[NU + i] -= w->st[k - 1].pin[i] - w->st[k - 1].pi[i];
        int i0 = (k == N) ? NU : 0, i1 = (k == 0) ? NU : NZ;
        for (int i = 0; i < NZ; i++) S->lg[i] = (i >= i0 && i < i1) ? r[i] : 0.0;
        for (int i = i0; i < i1; i++)
            if (fabs(r[i]) > res[0] || isnan(r[i])) res[0] = fabs(r[i]);
        if (k < N) {
            qp_stage *S1 = &w->st[k + 1];
            double rb[NX];
            dyn_res(w, k, rb);
            for (int i = 0; i < NX; i++) {
                double acc = rb[i] - S1->ddz[NU + i];
                for (int j = 0; j < NX; j++) acc += S->A[i][j] * S->ddz[NU + j];
                for (int j = 0; j < NU; j++) acc += S->B[i][j] * S->ddz[j];
                S->lb[i] = acc;
                if (fabs(acc) > res[1] || isnan(acc)) res[1] = fabs(acc);
            }
        }
    }
}

static int qp_solve(const orc_problem *pr, qp_ws *w, int *iters, int warm, int *n_center, int *n_itref,
                    int *n_lq) {
    int N = w->N;
    w->force_lq = w->lq_fact == 2;  /* HPIPM lq_fact 2: LQ factorisations only */
    if (!warm) {
        /* cold start (HPIPM init_var, warm_start 0): ux = 0, pi = 0; then per row t = gap at
         * ux clipped below at thr0, lambda = mu0 / t.  With qp_init_move (HPIPM's own start), the
         * box rows come first: a variable whose lower (upper) gap is below thr0 is moved to
         * thr0 inside that bound, or to the midpoint of its bounds when both gaps are; the
         * general rows then take their gaps at the moved ux */
        const double thr0 = pr->qp_thr0;
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int i = 0; i < NZ; i++)
                if (!(k == 0 && i >= NU)) S->dz[i] = 0.0; /* x0 part stays fixed */
            for (int i = 0; i < NX; i++) S->pi[i] = 0.0;
            int c0 = 0;
            if (pr->qp_init_move) {
                /* box rows: pairs (lower, upper) of one variable, before the h rows (linearise) */
                for (; c0 + 1 < S->ni && S->hrow[c0] < 0; c0 += 2) {
                    int v = 0;
                    while (v < NZ && S->D[c0][v] == 0.0) v++;
                    double tl = S->d[c0] + S->dz[v], tu = S->d[c0 + 1] - S->dz[v]; /* -d_lb + ux, d_ub - ux */
                    if (tl < thr0) {
                        if (tu < thr0) {
                            S->dz[v] = 0.5 * (-S->d[c0] + S->d[c0 + 1]); /* 0.5 (d_lb + d_ub) */
                            tl = thr0;
                            tu = thr0;
                        } else {
                            tl = thr0;
                            S->dz[v] = -S->d[c0] + thr0; /* d_lb + thr0 */
                        }
                    } else if (tu < thr0) {
                        tu = thr0;
                        S->dz[v] = S->d[c0 + 1] - thr0; /* d_ub - thr0 */
                    }
                    S->t[c0] = tl;
                    S->t[c0 + 1] = tu;
                    S->lam[c0] = pr->qp_mu0 / tl;
                    S->lam[c0 + 1] = pr->qp_mu0 / tu;
                }
            }
            for (int c = c0; c < S->ni; c++) {
                double s;
                if (pr->qp_init_move) {
                    double dd = 0.0; /* t = -D ux + d (HPIPM's order) */
                    for (int i = 0; i < NZ; i++) dd += S->D[c][i] * S->dz[i];
                    s = -dd + S->d[c];
                } else {
                    s = S->d[c];
                    for (int i = 0; i < NZ; i++) s -= S->D[c][i] * S->dz[i];
                }
                S->t[c] = s > thr0 ? s : thr0;
                S->lam[c] = pr->qp_mu0 / S->t[c];
            }
        }
    } else {
        /* HPIPM warm_start 2 (d_ocp_qp_ipm init_var): the previous QP solution is the
         * initial point -- primal step, dynamics multipliers, inequality slacks and
         * multipliers -- with the slacks and multipliers clipped below at thr0; the
         * x0 part of the step is the fixed xinit - z_0 */
        const double thr = pr->qp_ws_thr;
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int c = 0; c < S->ni; c++) {
                if (S->t[c] < thr) S->t[c] = thr;
                if (S->lam[c] < thr) S->lam[c] = thr;
            }
        }
    }
    int status = AC_MAXITER;
    int it;
    /* the divergence test of the robust profile (qp_mu_max > 0); without it only a non-finite
     * mu ends the QP with the NaN status */
    const double mu_lim = pr->qp_mu_max > 0.0 ? pr->qp_mu_max : INFINITY;
    for (it = 0;; it++) {
        double rs, re, ri, mu, cmx;
        int m;
        qp_residuals(w, &rs, &re, &ri, &mu, &m, &cmx);
        /* non-finite or diverged (infeasible QP: duals blow up; qp_mu_max) -> NaN status */
        if (!(rs < 1e30) || !(re < 1e30) || !(ri < 1e30) || !(mu < mu_lim)) { status = AC_NAN; break; }
        /* HPIPM's exit order: the iteration cap first (qp_maxit_first) */
        if (pr->qp_maxit_first && it >= pr->qp_iter_max) { status = AC_MAXITER; break; }
        if (getenv("ORC_DEBUG")) fprintf(stderr, "  ipm it %d rs %.3e re %.3e ri %.3e mu %.3e\n", it, rs, re, ri, mu);
        if (getenv("ORC_DEBUG2")) {
            /* top complementarity contributors */
            for (int k = 0; k <= N; k++) {
                qp_stage *S = &w->st[k];
                for (int c = 0; c < S->ni; c++)
                    if (S->lam[c] * S->t[c] > 1e-2 * mu * 50)
                        fprintf(stderr, "     k %d row %d (h %d) t %.3e lam %.3e d %.3e\n", k, c, S->hrow[c], S->t[c], S->lam[c], S->d[c]);
            }
        }
        if (rs < pr->qp_tol && re < pr->qp_tol && ri < pr->qp_tol && mu < pr->qp_tol) { status = AC_SUCCESS; break; }
        if (it >= pr->qp_iter_max) { status = AC_MAXITER; break; }
        /* barrier-augmented Hessian */
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            memcpy(S->Hh, S->H, sizeof S->H);
            for (int c = 0; c < S->ni; c++) {
                double wc = KF ? S->lam[c] * (1.0 / S->t[c]) : S->lam[c] / S->t[c];
                for (int i = 0; i < NZ; i++) {
                    if (S->D[c][i] == 0.0) continue;
                    for (int j = 0; j < NZ; j++) S->Hh[i][j] += S->D[c][i] * wc * S->D[c][j];
                }
            }
        }
        if (riccati_factor(w)) { status = AC_NAN; break; }
        /* predictor */
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int c = 0; c < S->ni; c++) S->rc[c] = S->lam[c] * S->t[c];
        }
        build_q(w);
        riccati_solve(w);
        ineq_steps(w, NULL);
        if (w->lq_fact == 1 && !w->force_lq) {
            /* HPIPM lq_fact 1: the predictor direction's linear KKT residual; above 1e-5 in any component
             * (or NaN) the Cholesky factorisation was inaccurate, and this and every later factorisation of
             * the QP is an LQ one; the predictor is solved again with it */
            double lr[4];
            lin_residuals(w, lr);
            if (!(lr[0] <= 1e-5) || !(lr[1] <= 1e-5) || !(lr[2] <= 1e-5) || !(lr[3] <= 1e-5)) {
                w->force_lq = 1;
                ++*n_lq;
                riccati_factor(w);
                build_q(w);
                riccati_solve(w);
                ineq_steps(w, NULL);
            }
        }
        double aa = max_step(w);
        if (aa > 1.0) aa = 1.0;
        double comp_aff = 0.0;
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int c = 0; c < S->ni; c++) {
                comp_aff += (S->lam[c] + aa * S->dl[c]) * (S->t[c] + aa * S->dt[c]);
                S->dt_aff[c] = S->dt[c];
                S->dl_aff[c] = S->dl[c];
            }
        }
        double mu_aff = comp_aff / m;
        double sig = mu_aff / mu;
        if (pr->qp_sigma_clip && sig > 1.0) sig = 1.0;
        sig = sig * sig * sig;
        /* corrector */
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int c = 0; c < S->ni; c++)
                S->rc[c] = S->lam[c] * S->t[c] + S->dl_aff[c] * S->dt_aff[c] - sig * mu;
        }
        build_q(w);
        riccati_solve(w);
        ineq_steps(w, NULL);
        if (pr->qp_cond_pred_corr) {
            /* HPIPM cond_pred_corr: mu_aff of the corrected direction (its boundary step, at most
             * 1); above twice the predictor's, the direction is the centring one instead
             * (complementarity target sigma mu without the second-order term) */
            double ac = max_step(w);
            if (ac > 1.0) ac = 1.0;
            double cc = 0.0;
            if (KK) {
                /* kernel forms: sum l t + a (sum (l dt + t dl) + a sum dl dt) */
                double cb = 0.0, cq = 0.0;
                for (int k = 0; k <= N; k++) {
                    qp_stage *S = &w->st[k];
                    for (int c = 0; c < S->ni; c++) {
                        cb += S->lam[c] * S->dt[c] + S->t[c] * S->dl[c];
                        cq += S->dl[c] * S->dt[c];
                    }
                }
                cc = mu * m + ac * (cb + ac * cq);
            } else {
                for (int k = 0; k <= N; k++) {
                    qp_stage *S = &w->st[k];
                    for (int c = 0; c < S->ni; c++) cc += (S->lam[c] + ac * S->dl[c]) * (S->t[c] + ac * S->dt[c]);
                }
            }
            if (cc / m > 2.0 * mu_aff) {
                for (int k = 0; k <= N; k++) {
                    qp_stage *S = &w->st[k];
                    for (int c = 0; c < S->ni; c++) S->rc[c] = S->lam[c] * S->t[c] - sig * mu;
                }
                build_q(w);
                riccati_solve(w);
                ineq_steps(w, NULL);
                ++*n_center;
            }
        }
        /* HPIPM itref_corr_max: while the direction's linear KKT residual is not below
         * max(tol, 1e-3 x the iterate's residual) in every component, solve the Newton system
         * again for it (same factorisation) and add the correction; dt and dl then follow from
         * the refined step */
        for (int itr = 0; itr < pr->qp_itref_corr_max; itr++) {
            double lr[4];
            lin_residuals(w, lr);
            const double tol = pr->qp_tol;
            const int pass_ = (lr[0] < tol || lr[0] < 1e-3 * rs) && (lr[1] < tol || lr[1] < 1e-3 * re) &&
                (lr[2] < tol || lr[2] < 1e-3 * ri) && (lr[3] < tol || lr[3] < 1e-3 * cmx);
            if (getenv("ORC_ITREF_DIAG")) {
                double lmx = 0, itm = 0, dlm = 0, pmx = 0, dzm = 0;
                for (int k = 0; k <= N; k++) { qp_stage *S = &w->st[k];
                    for (int c = 0; c < S->ni; c++) { if (S->lam[c] > lmx) lmx = S->lam[c]; if (1.0/S->t[c] > itm) itm = 1.0/S->t[c]; if (fabs(S->dl[c]) > dlm) dlm = fabs(S->dl[c]); }
                    for (int i = 0; i < NX; i++) for (int j = 0; j < NX; j++) if (fabs(S->P[i][j]) > pmx) pmx = fabs(S->P[i][j]);
                    for (int i = 0; i < NZ; i++) if (fabs(S->ddz[i]) > dzm) dzm = fabs(S->ddz[i]); }
                fprintf(stderr, "ITREF %d itr %d lam %.2e it %.2e dl %.2e P %.2e dz %.2e | lr %.1e %.1e %.1e %.1e | r %.1e %.1e %.1e %.1e\n", pass_, itr, lmx, itm, dlm, pmx, dzm, lr[0], lr[1], lr[2], lr[3], rs, re, ri, cmx);
            }
            if (pass_) break;
            double rb[ORC_MAX_N][NX];
            for (int k = 0; k <= N; k++) {
                qp_stage *S = &w->st[k];
                memcpy(S->ddz0, S->ddz, sizeof S->ddz);
                memcpy(S->pin0, S->pin, sizeof S->pin);
                if (k < N) memcpy(rb[k], S->lb, sizeof S->lb);
                for (int i = 0; i < NZ; i++) S->q[i] = S->lg[i];
                for (int c = 0; c < S->ni; c++) {
                    const double coef = KF ? (S->lam[c] * S->ld[c] - S->lm[c]) * (1.0 / S->t[c])
                                           : (S->lam[c] * S->ld[c] - S->lm[c]) / S->t[c];
                    for (int i = 0; i < NZ; i++) S->q[i] += S->D[c][i] * coef;
                }
            }
            riccati_solve_r(w, rb);
            for (int k = 0; k <= N; k++) {
                qp_stage *S = &w->st[k];
                for (int i = 0; i < NZ; i++) S->ddz[i] = S->ddz0[i] + S->ddz[i];
                if (k < N)
                    for (int i = 0; i < NX; i++) S->pin[i] = S->pin0[i] + S->pin[i];
            }
            ineq_steps(w, NULL);
            ++*n_itref;
        }
        double alpha = 0.995 * max_step(w);
        if (alpha > 1.0) alpha = 1.0;
        if (alpha < 1e-12) { status = AC_MINSTEP; it++; break; }
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w->st[k];
            for (int i = 0; i < NZ; i++) S->dz[i] += alpha * S->ddz[i];
            if (k < N)
                for (int i = 0; i < NX; i++) S->pi[i] += alpha * (S->pin[i] - S->pi[i]);
            for (int c = 0; c < S->ni; c++) {
                /* the step, then the t / lambda floor qp_t_min */
                const double tn = S->t[c] + alpha * S->dt[c], ln = S->lam[c] + alpha * S->dl[c];
                S->t[c] = tn < pr->qp_t_min ? pr->qp_t_min : tn;
                S->lam[c] = ln < pr->qp_t_min ? pr->qp_t_min : ln;
            }
        }
    }
    *iters = it;
    return status;
}

/* ------------------------------------------------------------------ */
/* Solver::solve() (acados_solver_interface.cpp:86-119, 162-204)              */
/* ------------------------------------------------------------------ */
int orc_solve(const orc_problem *pr, const double *params, const double *warm, const double *xinit,
              double *xtraj, double *utraj, orc_info *info) {
    return orc_solve_ex(pr, params, warm, xinit, NULL, xtraj, utraj, NULL, info);
}

/* side of the single finite bound of h row r: 1 upper, 0 lower */
static int h_side(const double *uh, int r) { return uh[r] < BIGBOUND ? 1 : 0; }

/* NLP residuals at the linearisation point (acados ocp_nlp_res_compute) with the
 * multipliers the NLP holds: dynamics pi, row multipliers lr[k][c] */
static void nlp_residuals(qp_ws *w, double *const *lr, double *rstat, double *rineq, double *rcomp,
                          int *nonfinite) {
    int N = w->N;
    double s_max = 0.0, i_max = 0.0, c_max = 0.0;
    int bad = 0; /* a non-finite operand (the max tests below drop NaN) */
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w->st[k];
        double r[NZ];
        for (int i = 0; i < NZ; i++) r[i] = S->g[i];
        if (k < N)
            for (int i = 0; i < NZ; i++) {
                double acc = 0.0;
                for (int m = 0; m < NX; m++) acc += (i < NU ? S->B[m][i] : S->A[m][i - NU]) * S->pi[m];
                r[i] += acc;
            }
        if (k > 0)
            for (int i = 0; i < NX; i++) r[NU + i] -= w->st[k - 1].pi[i];
        for (int c = 0; c < S->ni; c++) {
            for (int i = 0; i < NZ; i++) r[i] += S->D[c][i] * lr[k][c];
            if (-S->d[c] > i_max) i_max = -S->d[c];
            if (fabs(lr[k][c] * S->d[c]) > c_max) c_max = fabs(lr[k][c] * S->d[c]);
            bad |= !isfinite(S->d[c]) || !isfinite(lr[k][c]);
        }
        int i0 = (k == N) ? NU : 0, i1 = (k == 0) ? NU : NZ;
        for (int i = i0; i < i1; i++)
            if (fabs(r[i]) > s_max) s_max = fabs(r[i]);
        for (int i = 0; i < NZ; i++) bad |= !isfinite(r[i]);
        if (k < N)
            for (int i = 0; i < NX; i++) bad |= !isfinite(S->b[i]);
    }
    *rstat = s_max; *rineq = i_max; *rcomp = c_max;
    *nonfinite = bad;
}

/* SQP preparation phase: the QP of the iterate z (cost gradient / exact Hessian with
 * MIRROR, shooting defects and sensitivities, bounds and linearised h rows with the
 * multiplier-weighted Hessians); returns the dynamics residual res_eq */
static double linearise(const orc_problem *pr, const double *params, double (*z)[NZ], double (*pi)[NX],
                        const double *lamh, const double *lh, const double *uh, qp_ws *ws, double *hh) {
    qp_ws w = *ws;
    int N = pr->N, npar = pr->npar, nh = orc_num_h(pr);
    double res_eq;
    double h[ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN], jac[(ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN) * NZ];
        res_eq = 0.0;
    for (int k = 0; k < N; k++) {
        qp_stage *S = &w.st[k];
        const double *p = params + (size_t)k * npar;
        double L, g[NZ], Hc[NZ * NZ], Hd[NZ * NZ], xn[NX], A[NX * NX], B[NX * NU];
        orc_stage_cost_k(pr, k, z[k], p, &L, g, Hc);
        orc_discrete(pr, z[k], p, xn, A, B, pi[k], Hd);
        for (int i = 0; i < NZ; i++) {
            S->g[i] = g[i];
            for (int j = 0; j < NZ; j++) S->H[i][j] = Hc[i * NZ + j] + Hd[i * NZ + j];
        }
        for (int i = 0; i < NX; i++) {
            S->b[i] = xn[i] - z[k + 1][NU + i];
            if (fabs(S->b[i]) > res_eq) res_eq = fabs(S->b[i]);
            for (int j = 0; j < NX; j++) S->A[i][j] = A[i * NX + j];
            for (int j = 0; j < NU; j++) S->B[i][j] = B[i * NU + j];
        }
        int ni = 0;
        /* input bounds (idxbu = all, :104-107) */
        for (int i = 0; i < NU; i++) {
            memset(S->D[ni], 0, sizeof(double) * NZ); S->D[ni][i] = -1.0;
            S->d[ni] = z[k][i] - pr->lbu[i]; S->hrow[ni] = -1; ni++;
            memset(S->D[ni], 0, sizeof(double) * NZ); S->D[ni][i] = 1.0;
            S->d[ni] = pr->ubu[i] - z[k][i]; S->hrow[ni] = -1; ni++;
        }
        if (k >= 1) {
            /* state bounds on stages 1..N-1 (idxbx = all, :100-102) */
            for (int i = 0; i < NX; i++) {
                memset(S->D[ni], 0, sizeof(double) * NZ); S->D[ni][NU + i] = -1.0;
                S->d[ni] = z[k][NU + i] - pr->lbx[i]; S->hrow[ni] = -1; ni++;
                memset(S->D[ni], 0, sizeof(double) * NZ); S->D[ni][NU + i] = 1.0;
                S->d[ni] = pr->ubx[i] - z[k][NU + i]; S->hrow[ni] = -1; ni++;
            }
            /* nonlinear constraints h, linearised; Hessian weighted by the
             * NLP multipliers (exact Hessian of the Lagrangian) */
            orc_stage_constraints(pr, z[k], p, h, jac, hh);
            for (int r = 0; r < nh; r++) {
                double wgt = lamh[(size_t)k * 2 * nh + 2 * r + 1] - lamh[(size_t)k * 2 * nh + 2 * r + 0];
                if (wgt != 0.0)
                    for (int i = 0; i < NZ; i++)
                        for (int j = 0; j < NZ; j++) S->H[i][j] += wgt * hh[(size_t)r * NZ * NZ + i * NZ + j];
                if (uh[r] < BIGBOUND) {
                    for (int i = 0; i < NZ; i++) S->D[ni][i] = jac[r * NZ + i];
                    S->d[ni] = uh[r] - h[r]; S->hrow[ni] = r; S->hsgn[ni] = 1; ni++;
                }
                if (lh[r] > -BIGBOUND) {
                    for (int i = 0; i < NZ; i++) S->D[ni][i] = -jac[r * NZ + i];
                    S->d[ni] = h[r] - lh[r]; S->hrow[ni] = r; S->hsgn[ni] = 0; ni++;
                }
            }
        }
        S->ni = ni;
        double Hf[NZ * NZ];
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NZ; j++) Hf[i * NZ + j] = S->H[i][j];
        orc_mirror(NZ, Hf, pr->reg_eps);
        for (int i = 0; i < NZ; i++)
            for (int j = 0; j < NZ; j++) S->H[i][j] = Hf[i * NZ + j];
    }
    /* terminal stage: no cost (cost_type_e default), no constraints,
     * zero Hessian mirrored to eps*I */
    {
        qp_stage *S = &w.st[N];
        memset(S->H, 0, sizeof S->H);
        memset(S->g, 0, sizeof S->g);
        double Hx[NX * NX] = {0};
        orc_mirror(NX, Hx, pr->reg_eps);
        for (int i = 0; i < NX; i++)
            for (int j = 0; j < NX; j++) S->H[NU + i][NU + j] = Hx[i * NX + j];
        S->ni = 0;
    }
    return res_eq;
}

int orc_qp_mem_size(const orc_problem *pr) {
    return (pr->N + 1) * (NZ + NX + 2 * (2 * NZ + 2 * orc_num_h(pr)));
}

int orc_solve_ex(const orc_problem *pr, const double *params, const double *warm, const double *xinit,
                 const double *lam_in, double *xtraj, double *utraj, double *lam_out, orc_info *info) {
    return orc_solve_full(pr, params, warm, xinit, lam_in, NULL, xtraj, utraj, lam_out, NULL, info);
}

int orc_solve_full(const orc_problem *pr, const double *params, const double *warm, const double *xinit,
                   const double *lam_in, const double *qp_in, double *xtraj, double *utraj, double *lam_out,
                   double *qp_out, orc_info *info) {
    int N = pr->N, npar = pr->npar;
    int nh = orc_num_h(pr);
    int maxi = 2 * NZ + 2 * nh;
    const int qstride = NZ + NX + 2 * maxi;  /* orc_qp_mem_size per stage */
    double lh[ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN], uh[ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN];
    orc_h_bounds(pr, lh, uh);

    qp_ws w;
    w.N = N;
    /* the square-root Riccati of HPIPM's profile in the kernel-agnostic builds (the kernel-forms build
     * mirrors the kernel, which runs the classical form) */
    w.ric_sqrt = pr->qp_ric_alg == 1 && !KK;
    w.pivot_zero = pr->qp_pivot_zero != 0;
    w.lq_fact = w.ric_sqrt ? pr->qp_lq_fact : 0;
    w.st = (qp_stage *)calloc(N + 1, sizeof(qp_stage));
    size_t nrow = (size_t)(N + 1) * maxi;
    double (*Dall)[NZ] = (double (*)[NZ])calloc(nrow, sizeof(double[NZ]));
    double *dbl = (double *)calloc(nrow * 11, sizeof(double));
    int *ibl = (int *)calloc(nrow * 2, sizeof(int));
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w.st[k];
        size_t o = (size_t)k * maxi;
        S->D = Dall + o;
        S->d = dbl + o; S->t = dbl + nrow + o; S->lam = dbl + 2 * nrow + o;
        S->dt = dbl + 3 * nrow + o; S->dl = dbl + 4 * nrow + o; S->dt_aff = dbl + 5 * nrow + o;
        S->dl_aff = dbl + 6 * nrow + o; S->rin = dbl + 7 * nrow + o; S->rc = dbl + 8 * nrow + o;
        S->ld = dbl + 9 * nrow + o; S->lm = dbl + 10 * nrow + o;
        S->hrow = ibl + o; S->hsgn = ibl + nrow + o;
    }
    /* NLP iterate: z_k = [u_k; x_k] from the warm start (loadWarmstart, acados_solver_interface.cpp:274-284);
     * NLP multipliers: those the capsule kept from the previous solve
     * (lam_in, [N][NX + nh]) or zero (fresh / reset capsule). */
    double (*z)[NZ] = (double (*)[NZ])calloc(N + 1, sizeof(double[NZ]));
    double (*pi)[NX] = (double (*)[NX])calloc(N + 1, sizeof(double[NX]));
    double *lamh = (double *)calloc((size_t)(N + 1) * 2 * nh, sizeof(double)); /* [k][2*i+side] */
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < NZ; i++) z[k][i] = warm[k * NZ + i];
    for (int i = 0; i < NU; i++) z[N][i] = 0.0;
    const int LS = NX + nh;
    if (lam_in) {
        for (int k = 0; k < N; k++) {
            for (int i = 0; i < NX; i++) pi[k][i] = lam_in[(size_t)k * LS + i];
            if (k >= 1)
                for (int r = 0; r < nh; r++)
                    lamh[(size_t)k * 2 * nh + 2 * r + h_side(uh, r)] = lam_in[(size_t)k * LS + NX + r];
        }
    }

    /* the capsule's QP memory (HPIPM's qp_sol: step, pi, slacks, multipliers of the last QP) */
    int have_qp = 0;
    if (qp_in && !isnan(qp_in[0])) {
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w.st[k];
            const double *q = qp_in + (size_t)k * qstride;
            memcpy(S->dz, q, sizeof(double) * NZ);
            memcpy(S->pi, q + NZ, sizeof(double) * NX);
            memcpy(S->t, q + NZ + NX, sizeof(double) * maxi);
            memcpy(S->lam, q + NZ + NX + maxi, sizeof(double) * maxi);
        }
        have_qp = 1;
    }
    double *lrow = (double *)calloc((size_t)(N + 1) * maxi, sizeof(double));
    double *lrp[ORC_MAX_N + 1];
    for (int k = 0; k <= N; k++) lrp[k] = lrow + (size_t)k * maxi;
    double res_stat = 0.0, res_ineq = 0.0, res_comp = 0.0;

    double *hh = (double *)malloc(sizeof(double) * nh * NZ * NZ);
    int acados_status = AC_SUCCESS, qp_status = AC_SUCCESS, sqp_iter = 0, qp_iter_total = 0, n_maxit = 0;
    int n_center = 0, n_itref = 0, n_lq = 0;
    double res_eq = 0.0;

    const int sqp_mode = pr->nlp_solver == 1;
    for (int it = 0; sqp_mode || it < pr->sqp_iters; it++) {
        res_eq = linearise(pr, params, z, pi, lamh, lh, uh, &w, hh);
        /* x0 elimination: lbx_0 = ubx_0 = xinit (acados_solver_interface.cpp:124-125) */
        for (int i = 0; i < NX; i++) w.st[0].dz[NU + i] = xinit[i] - z[0][NU + i];

        /* NLP residuals with the NLP's multipliers: the dynamics pi; per row the previous
         * QP's multiplier (FIXED_STEP: lam = lam_qp), else the carried h-row ones (box 0) */
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w.st[k];
            if (k < N && !have_qp) memcpy(S->pi, pi[k], sizeof(double) * NX);
            for (int c = 0; c < S->ni; c++)
                lrp[k][c] = have_qp ? S->lam[c]
                                    : (S->hrow[c] >= 0 ? lamh[(size_t)k * 2 * nh + 2 * S->hrow[c] + S->hsgn[c]] : 0.0);
        }
        int nonfinite = 0;
        nlp_residuals(&w, lrp, &res_stat, &res_ineq, &res_comp, &nonfinite);
        if (sqp_mode) {
            /* a non-finite NLP residual ends the call with the NaN status (the kernel's guard) */
            if (nonfinite) {
                acados_status = AC_NAN;
                break;
            }
            /* acados SQP termination at this linearisation point */
            if (res_stat < pr->nlp_tol && res_eq < pr->nlp_tol && res_ineq < pr->nlp_tol && res_comp < pr->nlp_tol) {
                acados_status = AC_SUCCESS;
                break;
            }
            if (it >= pr->nlp_max_iter) {
                acados_status = AC_MAXITER;
                break;
            }
        }

        /* ---- feedback phase: QP ---- (warm: every QP of an acados call after its first;
         * the first with warm_start_first_qp) */
        int qit = 0;
        const int warm = have_qp && pr->qp_warm_start == 2 && ((sqp_mode && it > 0) || pr->qp_warm_first);
        qp_status = qp_solve(pr, &w, &qit, warm, &n_center, &n_itref, &n_lq);
        have_qp = 1;
        qp_iter_total += qit;
        sqp_iter++;
        n_maxit += qp_status == AC_MAXITER;
        if (qp_status != AC_SUCCESS && qp_status != AC_MAXITER) {
            acados_status = AC_QP_FAILURE;
            break;
        }
        /* FIXED_STEP full step on primal and multipliers */
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w.st[k];
            for (int i = 0; i < NZ; i++) z[k][i] += S->dz[i];
            if (k < N) memcpy(pi[k], S->pi, sizeof(double) * NX);
            for (int r = 0; r < 2 * nh; r++) lamh[(size_t)k * 2 * nh + r] = 0.0;
            for (int c = 0; c < S->ni; c++)
                if (S->hrow[c] >= 0) lamh[(size_t)k * 2 * nh + 2 * S->hrow[c] + S->hsgn[c]] = S->lam[c];
        }
        for (int i = 0; i < NU; i++) z[N][i] = 0.0;
        acados_status = AC_SUCCESS;
        /* SQP-RTI, acados_solver_interface.cpp:105: break when the QP did not succeed (a full
         * SQP call continues after a max-iter QP) */
        if (!sqp_mode && qp_status != AC_SUCCESS) break;
    }

    double pobj = 0.0;
    for (int k = 0; k < N; k++) {
        double L;
        orc_stage_cost_k(pr, k, z[k], params + (size_t)k * npar, &L, NULL, NULL);
        pobj += L;
    }
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < NX; i++) xtraj[k * NX + i] = z[k][NU + i];
    for (int k = 0; k < N; k++)
        for (int i = 0; i < NU; i++) utraj[k * NU + i] = z[k][i];

    if (lam_out) {
        for (int k = 0; k < N; k++) {
            for (int i = 0; i < NX; i++) lam_out[(size_t)k * LS + i] = pi[k][i];
            for (int r = 0; r < nh; r++)
                lam_out[(size_t)k * LS + NX + r] = k >= 1 ? lamh[(size_t)k * 2 * nh + 2 * r + h_side(uh, r)] : 0.0;
        }
    }

    if (qp_out) {
        for (int k = 0; k <= N; k++) {
            qp_stage *S = &w.st[k];
            double *q = qp_out + (size_t)k * qstride;
            memcpy(q, S->dz, sizeof(double) * NZ);
            memcpy(q + NZ, S->pi, sizeof(double) * NX);
            memcpy(q + NZ + NX, S->t, sizeof(double) * maxi);
            memcpy(q + NZ + NX + maxi, S->lam, sizeof(double) * maxi);
        }
    }
    free(lrow);

    int exit_code = acados_status;
    if (res_eq > pr->res_eq_fail && exit_code == AC_SUCCESS) exit_code = AC_QP_FAILURE;
    if (exit_code == AC_SUCCESS) exit_code = 1;
    else if (exit_code == 1) exit_code = 0;
    if (info) {
        info->sqp_iter = sqp_iter;
        info->qp_iter_total = qp_iter_total;
        info->qp_status = qp_status;
        info->res_eq = res_eq;
        info->pobj = pobj;
        info->res_stat = res_stat;
        info->res_ineq = res_ineq;
        info->res_comp = res_comp;
        info->qp_maxiter = n_maxit;
        info->qp_center = n_center;
        info->qp_itref = n_itref;
        info->qp_lq = n_lq;
    }
    free(hh); free(lamh); free(pi); free(z);
    free(ibl); free(dbl); free(Dall); free(w.st);
    return exit_code;
}

void orc_solve_batch(const orc_problem *pr, int batch, const double *params, const double *warm,
                     const double *xinit, double *xtraj, double *utraj, double *pobj,
                     int *status, int *qp_iters, int nthreads) {
    int N = pr->N;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
#endif
    for (int b = 0; b < batch; b++) {
        orc_info info;
        status[b] = orc_solve(pr, params + (size_t)b * N * pr->npar, warm + (size_t)b * (N + 1) * NZ,
                              xinit + (size_t)b * NX, xtraj + (size_t)b * (N + 1) * NX,
                              utraj + (size_t)b * N * NU, &info);
        pobj[b] = info.pobj;
        if (qp_iters) qp_iters[b] = info.qp_iter_total;
    }
    (void)nthreads;
}

void orc_solve_batch_ex(const orc_problem *pr, int batch, const double *params, const double *warm,
                        const double *xinit, const double *lam_in, double *xtraj, double *utraj, double *pobj,
                        int *status, int *qp_iters, double *lam_out, int nthreads) {
    int N = pr->N;
    size_t LS = (size_t)N * (NX + orc_num_h(pr));
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
#endif
    for (int b = 0; b < batch; b++) {
        orc_info info;
        status[b] = orc_solve_ex(pr, params + (size_t)b * N * pr->npar, warm + (size_t)b * (N + 1) * NZ,
                                 xinit + (size_t)b * NX, lam_in ? lam_in + b * LS : NULL,
                                 xtraj + (size_t)b * (N + 1) * NX, utraj + (size_t)b * N * NU,
                                 lam_out ? lam_out + b * LS : NULL, &info);
        pobj[b] = info.pobj;
        if (qp_iters) qp_iters[b] = info.qp_iter_total;
    }
    (void)nthreads;
}

void orc_solve_batch_full(const orc_problem *pr, int batch, const double *params, const double *warm,
                          const double *xinit, const double *lam_in, const double *qp_in, double *xtraj,
                          double *utraj, int *status, double *lam_out, double *qp_out, orc_info *infos,
                          int nthreads) {
    int N = pr->N;
    size_t LS = (size_t)N * (NX + orc_num_h(pr)), QS = (size_t)orc_qp_mem_size(pr);
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
#endif
    for (int b = 0; b < batch; b++) {
        orc_info info;
        status[b] = orc_solve_full(pr, params + (size_t)b * N * pr->npar, warm + (size_t)b * (N + 1) * NZ,
                                   xinit + (size_t)b * NX, lam_in ? lam_in + b * LS : NULL,
                                   qp_in ? qp_in + b * QS : NULL, xtraj + (size_t)b * (N + 1) * NX,
                                   utraj + (size_t)b * N * NU, lam_out ? lam_out + b * LS : NULL,
                                   qp_out ? qp_out + b * QS : NULL, &info);
        if (infos) infos[b] = info;
    }
    (void)nthreads;
}

/* Diagnostics: the first QP of a solve (the linearisation at the warm start), for an
 * independent feasibility check (scripts/qp_feasibility.py, HiGHS LP).  A [N][NX][NX],
 * B [N][NX][NU], b [N][NX], D [(N+1)][maxi][NZ], d [(N+1)][maxi], ni [N+1], dx0 [NX];
 * rows are D_c dz <= d_c.  Returns maxi = 2 NZ + 2 nh. */
int orc_qp_data(const orc_problem *pr, const double *params, const double *warm, const double *xinit,
                const double *lam_in, double *A, double *B, double *b, double *D, double *d, int *ni,
                double *dx0) {
    int N = pr->N, nh = orc_num_h(pr), maxi = 2 * NZ + 2 * nh;
    double lh[ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN], uh[ORC_MAX_LIN + ORC_MAX_ELL + ORC_MAX_SCEN];
    orc_h_bounds(pr, lh, uh);
    qp_ws w;
    w.N = N;
    /* the square-root Riccati of HPIPM's profile in the kernel-agnostic builds (the kernel-forms build
     * mirrors the kernel, which runs the classical form) */
    w.ric_sqrt = pr->qp_ric_alg == 1 && !KK;
    w.pivot_zero = pr->qp_pivot_zero != 0;
    w.lq_fact = w.ric_sqrt ? pr->qp_lq_fact : 0;
    w.st = (qp_stage *)calloc(N + 1, sizeof(qp_stage));
    size_t nrow = (size_t)(N + 1) * maxi;
    double (*Dall)[NZ] = (double (*)[NZ])calloc(nrow, sizeof(double[NZ]));
    double *dbl = (double *)calloc(nrow * 11, sizeof(double));
    int *ibl = (int *)calloc(nrow * 2, sizeof(int));
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w.st[k];
        size_t o = (size_t)k * maxi;
        S->D = Dall + o;
        S->d = dbl + o; S->t = dbl + nrow + o; S->lam = dbl + 2 * nrow + o;
        S->dt = dbl + 3 * nrow + o; S->dl = dbl + 4 * nrow + o; S->dt_aff = dbl + 5 * nrow + o;
        S->dl_aff = dbl + 6 * nrow + o; S->rin = dbl + 7 * nrow + o; S->rc = dbl + 8 * nrow + o;
        S->ld = dbl + 9 * nrow + o; S->lm = dbl + 10 * nrow + o;
        S->hrow = ibl + o; S->hsgn = ibl + nrow + o;
    }
    double (*z)[NZ] = (double (*)[NZ])calloc(N + 1, sizeof(double[NZ]));
    double (*pi)[NX] = (double (*)[NX])calloc(N + 1, sizeof(double[NX]));
    double *lamh = (double *)calloc((size_t)(N + 1) * 2 * nh, sizeof(double));
    double *hh = (double *)malloc(sizeof(double) * (nh ? nh : 1) * NZ * NZ);
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < NZ; i++) z[k][i] = warm[k * NZ + i];
    for (int i = 0; i < NU; i++) z[N][i] = 0.0;
    const int LS = NX + nh;
    if (lam_in)
        for (int k = 0; k < N; k++) {
            for (int i = 0; i < NX; i++) pi[k][i] = lam_in[(size_t)k * LS + i];
            if (k >= 1)
                for (int r = 0; r < nh; r++)
                    lamh[(size_t)k * 2 * nh + 2 * r + h_side(uh, r)] = lam_in[(size_t)k * LS + NX + r];
        }
    linearise(pr, params, z, pi, lamh, lh, uh, &w, hh);
    for (int k = 0; k <= N; k++) {
        qp_stage *S = &w.st[k];
        if (k < N)
            for (int i = 0; i < NX; i++) {
                b[k * NX + i] = S->b[i];
                for (int j = 0; j < NX; j++) A[(k * NX + i) * NX + j] = S->A[i][j];
                for (int j = 0; j < NU; j++) B[(k * NX + i) * NU + j] = S->B[i][j];
            }
        ni[k] = S->ni;
        for (int c = 0; c < S->ni; c++) {
            d[(size_t)k * maxi + c] = S->d[c];
            for (int i = 0; i < NZ; i++) D[((size_t)k * maxi + c) * NZ + i] = S->D[c][i];
        }
    }
    for (int i = 0; i < NX; i++) dx0[i] = xinit[i] - z[0][NU + i];
    free(hh); free(lamh); free(pi); free(z);
    free(ibl); free(dbl); free(Dall); free(w.st);
    return maxi;
}
