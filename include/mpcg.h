/*
 * mpcg.h — C ABI of the MI355X-native T-MPC++ per-guess SQP backend.
 *
 * This is the drop-in boundary for the hot path of
 * Juleszwanen/oscar_mpc_planner_mr_modification: the OpenMP fan-out of
 * independent `MPCPlanner::Solver::solve()` calls inside
 * `GuidanceConstraints::optimize` (mpc_planner_modules/src/guidance_constraints.cpp:304-421)
 * and the acados SQP-RTI solve each of them runs
 * (mpc_planner_solver/src/acados_solver_interface.cpp:86-119, 162-204).
 *
 * Plain pointers and sizes only.  Buffers use the reference's own layouts:
 *   params  [batch][N][npar]      == AcadosParameters::all_parameters, horizon-major
 *                                    (mpc_planner_solver/include/mpc_planner_solver/acados_solver_interface.h:56)
 *   warm    [batch][N+1][nu+nx]   == AcadosParameters::x0 = [u0 x0 | u1 x1 | ...] (:54)
 *   xinit   [batch][nx]           == AcadosParameters::xinit (:53)
 *   xtraj   [batch][N+1][nx]      == AcadosOutput::xtraj (:129)
 *   utraj   [batch][N][nu]        == AcadosOutput::utraj (:130)
 *   pobj    [batch]               == AcadosInfo::pobj (:108)
 *   exit    [batch]               == return value of Solver::solve(): 1 success, 0 failure,
 *                                    2 max-iter, 3 min-step, 4 QP failure (acados_solver_interface.cpp:176-201)
 * Batch element b = scene * n_guesses + guess.
 */
#ifndef MPCG_H
#define MPCG_H

#ifdef __cplusplus
extern "C" {
#endif

/* ContouringSecondOrderUnicycleModel (solver_model.py:185-214): nx 5, nu 2.  The
 * SH-MPC model ContouringSecondOrderUnicycleModelWithSlack (:274-298) adds the
 * slack state last: nx 6.  BicycleModel2ndOrderCurvatureAware (:355-437, C3):
 * nu 3 (a, w, slack), nx 6 (x, y, psi, v, delta, spline).  Every buffer below is
 * sized by mpcg_problem.nx / nu. */
#define MPCG_NX 5
#define MPCG_MAX_NX 6
#define MPCG_NU 2            /* the unicycle models */
#define MPCG_MAX_NU 3
#define MPCG_NVAR 7
#define MPCG_ABI_VERSION 9
/* mpcg_problem.model */
#define MPCG_MODEL_UNICYCLE 0      /* contouring unicycle (+ slack state): MPCBase + Contouring (+ Consistency) */
#define MPCG_MODEL_BICYCLE_CA 1    /* curvature-aware bicycle: MPCBase(a, w, slack) + CurvatureAwareContouring */
/* mpcg_problem.nlp_solver: solver_settings.acados.solver_type (settings.yaml:19,
 * generate_acados_solver.py:153) */
#define MPCG_NLP_SQP_RTI 0         /* sqp_iters SQP-RTI iterations per solve (the reference's loop of
                                      Solver_acados_solve calls, acados_solver_interface.cpp:86-119) */
#define MPCG_NLP_SQP 1             /* one full acados SQP call (the reference sets _num_iterations = 1,
                                      :27-29): up to nlp_max_iter iterations, converged when the four NLP
                                      residuals are below nlp_tol */

/* Problem description: the generated solver's dimensions + the parameter
 * map (parameter_map.yaml written by solver_generator/generate_solver.py:34-46)
 * reduced to the base index of every parameter bundle the stage functions
 * read, and the acados options of generate_acados_solver.py:88-173.
 * -1 marks an absent module. */
typedef struct mpcg_problem {
    int N, npar;
    int n_lin, n_ell, n_seg;
    int i_w_acc, i_w_ang, i_w_vel, i_v_ref, i_w_contour, i_w_lag;
    int i_spline0;                 /* segment j at i_spline0 + 9 j: xa xb xc xd ya yb yc yd start */
    int i_cons_w, i_prev_x, i_prev_y;
    int i_lin0;                    /* halfspace i at i_lin0 + 3 i: a1 a2 b */
    int i_disc_r, i_disc_off;
    int i_ell0;                    /* obstacle j at i_ell0 + 7 j: x y psi major minor chi r */
    int n_scen, i_scen0;           /* scenario halfspace i at i_scen0 + 3 i: a1 a2 b
                                      (a1 xd + a2 yd - (b + slack) <= 0, scenario_constraints.py:64-94);
                                      the bicycle model: the decomp halfspaces, same row
                                      (disc_0_decomp_<i>_a1 ..., decomp_constraints.py:46-98) */
    int i_w_slack;                 /* MPCBase weight of the slack variable */
    int nx;                        /* 5, or 6 with the slack state / the bicycle */
    double dt;                     /* integrator_step; ERK4 over dt with rk_steps steps */
    int rk_steps;                  /* acados sim_method_num_steps 3; the bicycle (Forces RK4): 1 */
    double lbu[MPCG_MAX_NU], ubu[MPCG_MAX_NU], lbx[MPCG_MAX_NX], ubx[MPCG_MAX_NX];
    int sqp_iters;                 /* solver_settings.acados.iterations (timeout disabled) */
    double qp_tol;                 /* 1e-5 */
    int qp_iter_max;               /* 50 */
    double reg_eps;                /* MIRROR epsilon 1e-4 */
    double qp_mu0, qp_thr0;        /* interior-point cold start */
    double res_eq_fail;            /* 1e-2 */
    int nu;                        /* 2, or 3 for the bicycle */
    int model;                     /* MPCG_MODEL_* */
    int i_w_tangle, i_w_tcont;     /* terminal_angle / terminal_contouring: read by the bicycle model's
                                      CurvatureAwareContouring at stage N-1 (curvature_aware_contouring.py:94-103,
                                      Forces' per-stage objective, generate_forces_solver.py:50-59) */
    int qp_warm_start;             /* qp_solver_warm_start (generate_acados_solver.py:173, default 2): 2 = HPIPM
                                      primal + dual warm start from the previous QP's solution (the capsule's QP
                                      memory), slacks and multipliers clipped below at qp_ws_thr; 0 = cold start.
                                      Applies to every QP of an acados call after its first, and to the first
                                      one only with qp_warm_first (so every SQP-RTI QP starts cold by default) */
    double qp_ws_thr;              /* 0.1 */
    /* ABI 6 */
    int nlp_solver;                /* MPCG_NLP_SQP_RTI (default) or MPCG_NLP_SQP */
    int nlp_max_iter;              /* MPCG_NLP_SQP: acados nlp_solver_max_iter (acados_template default 100; the
                                      reference leaves it unset, generate_acados_solver.py:154) */
    double nlp_tol;                /* MPCG_NLP_SQP: solver_options.tol 1e-2 (generate_acados_solver.py:144) on the
                                      stationarity, dynamics, inequality and complementarity residuals */
    int qp_warm_first;             /* acados warm_start_first_qp (default 0): the first QP of a call also starts
                                      warm (from mpcg_io.qp_in, or in SQP-RTI from the previous iteration's QP) */
    /* ABI 7 */
    double qp_t_min;               /* floor of every inequality row's slack t and multiplier lambda after each
                                      interior-point step (HPIPM's t_min / lam_min safeguard; 1e-12 here, where
                                      the dual-degenerate SH-MPC QPs' exit decisions stop depending on rounding,
                                      DESIGN.md §2.2); 0 = no floor */
    double qp_mu_max;              /* divergence test: an interior point whose mean complementarity reaches this
                                      is diverging -- the QP is infeasible, its duals blow up -- and ends with the
                                      NaN status (robust profile: 1e8; <= 0: no such test, HPIPM's behaviour, where
                                      only a non-finite iterate ends a QP with that status) */
    /* ABI 8: the interior point's profile (mpcg_problem_set_qp_profile sets the group).
     * MPCG_QP_HPIPM (the default of mpcg_problem_from_map*): HPIPM's BALANCE mode as acados configures it,
     * which the reference leaves at acados' defaults but for four options (generate_acados_solver.py:162-173):
     * qp_mu0 10, qp_thr0 0.1, qp_t_min 1e-16, qp_mu_max 0 and 1 / 1 / 2 / 0 / 1 below (ABI 9: qp_pivot_zero 1).
     * MPCG_QP_ROBUST: the round-4 algorithm, qp_mu0 1, qp_thr0 1, qp_t_min 1e-12, qp_mu_max 1e8 and 0 / 0 / 0 /
     * 1 / 0 (qp_pivot_zero 0). */
    int qp_profile;                /* MPCG_QP_*: what mpcg_problem_set_qp_profile wrote (informative) */
    int qp_init_move;              /* HPIPM init_var at a cold start: a box row whose gap is below qp_thr0 moves
                                      the primal start inside its bounds (to the midpoint when both are) */
    int qp_cond_pred_corr;         /* conditional predictor-corrector: a centring direction when the corrected
                                      one's mu_aff exceeds twice the predictor's */
    int qp_itref_corr_max;         /* iterative refinement steps of the corrector direction (its linear KKT
                                      residual above max(qp_tol, 1e-3 x the iterate's residual)) */
    int qp_sigma_clip;             /* 1: sigma = min(mu_aff / mu, 1)^3; 0: (mu_aff / mu)^3 (HPIPM) */
    int qp_maxit_first;            /* 1: the iteration cap is tested before convergence (HPIPM's exit order) */
    /* ABI 9 */
    int qp_pivot_zero;             /* a non-positive Cholesky pivot of the Riccati recursion: 1 BLASFEO's dpotrf rule
                                      (zero diagonal and inverse, the column below multiplied by it, the QP goes on;
                                      MPCG_QP_HPIPM), 0 the QP ends with the NaN status (MPCG_QP_ROBUST) */
} mpcg_problem;

#define MPCG_QP_HPIPM 0
#define MPCG_QP_ROBUST 1
/* Set the interior point's profile fields of `pr` (above).  Returns 0, or -1 for an unknown profile. */
int mpcg_problem_set_qp_profile(mpcg_problem *pr, int profile);

/* per-solve diagnostics, int32 x 4: sqp iterations, total QP iterations,
 * last QP status (acados: 0 ok, 1 nan/diverged, 2 max-iter, 3 min-step), and the
 * number of QPs that stopped at max-iter (their unconverged steps were applied) */
#define MPCG_INFO_STRIDE 4
/* per-solve NLP residuals, double x 4, at the last linearisation point with the
 * multipliers the NLP holds there (acados ocp_nlp_res_compute; their max is what
 * acados_solver_interface.cpp:151,164 reads as nlp_res / kkt_norm_inf):
 * stationarity, dynamics (res_eq), inequality violation, complementarity */
#define MPCG_STATS_STRIDE 4

int mpcg_abi_version(void);
const char *mpcg_last_error(void);

/* Number of nonlinear-constraint rows per stage (n_lin + n_ell + n_scen). */
int mpcg_num_h(const mpcg_problem *pr);

/* Size in doubles of one solve's multiplier block: N * (nx + nh). */
int mpcg_lam_size(const mpcg_problem *pr);

/* Size in doubles of one solve's QP memory (mpcg_io.qp_in / qp_out): the last QP's
 * step, dynamics multipliers and every inequality row's slack and multiplier, in the
 * kernel's own order (opaque: hand back what a previous solve of the same problem
 * wrote).  -1 without a compiled instance. */
int mpcg_qp_mem_size(const mpcg_problem *pr);

/* Fill `pr` from a parameter map (the name -> index pairs of
 * parameter_map.yaml) and the solver settings: the module bundles are found
 * by the names the reference's generator gives them (mpc_base.py, contouring.py,
 * consistency_module.py, guidance_constraints.py:333-338,
 * ellipsoid_constraints.py:406-419, scenario_constraints.py:41-50); n_lin /
 * n_ell / n_scen / n_seg are counted from `lin_constraint_<i>_a1`,
 * `ellipsoid_obst_<j>_x`, `disc_0_scenario_constraint_<i>_a1`, `spline<i>_start`.
 * nx: 5, or 6 for the model with the slack state (its weight is "slack").
 * lb/ub: nu + nx bounds in z order [u x] (model_map.yaml columns 3, 4).
 * Options take the defaults listed in mpcg_problem.  Returns 0, or -1 with
 * mpcg_last_error() naming the missing entry. */
int mpcg_problem_from_map(mpcg_problem *pr, int N, int nx, int npar, int n_entries, const char *const *names,
                          const int *indices, const double *lb, const double *ub, double dt,
                          int sqp_iters);

/* Same for a given model (MPCG_MODEL_*): the bicycle (nx 6, nu 3) finds its
 * decomp halfspaces by `disc_0_decomp_<i>_a1`, the terminal weights by
 * "terminal_angle" / "terminal_contouring", and integrates with one RK4 step
 * (rk_steps 1); lb/ub hold nu + nx bounds. */
int mpcg_problem_from_map_model(mpcg_problem *pr, int model, int N, int nx, int npar, int n_entries,
                                const char *const *names, const int *indices, const double *lb, const double *ub,
                                double dt, int sqp_iters);

/* Input/output buffers of one batched solve (all device pointers for
 * mpcg_solve, all host pointers for mpcg_context_solve).
 *   lam_in / lam_out  [batch][N][nx + nh]: NLP multipliers that persist in the
 *     acados capsule between Solver::solve() calls (ocp_nlp_out pi and lam;
 *     acados_solver_interface.cpp:86-119, reset to zero by Solver_acados_reset
 *     on failure, :186-190): per stage k < N the dynamics multipliers pi_k
 *     (x_{k+1} = phi(z_k)) then, for each h row, the multiplier of its finite
 *     side (>= 0; stage 0 rows are not part of the QP and stay 0).
 *     lam_in NULL = zero multipliers (a fresh or reset solver).  lam_out may be
 *     NULL; on a QP failure it holds the multipliers of the last accepted step. */
typedef struct mpcg_io {
    const double *params, *warm, *xinit;
    const double *lam_in;
    double *xtraj, *utraj, *pobj;
    int *exit_code, *info;
    double *lam_out;
    /* ABI 5: the capsule's QP memory [batch][mpcg_qp_mem_size] in / out (HPIPM's qp_sol,
     * kept between Solver::solve() calls: the first QP's initial point with
     * qp_warm_start 2, and the bound multipliers of the NLP residuals; NULL qp_in = a
     * fresh or reset capsule: ocp_nlp_solver_reset_qp_memory, acados_solver_interface.cpp:189),
     * and the NLP residuals [batch][MPCG_STATS_STRIDE]; each may be NULL.  A solve whose
     * qp_in block starts with a NaN has no QP memory (mixed batches of fresh and carried
     * solvers) */
    const double *qp_in;
    double *qp_out;
    double *stats;
} mpcg_io;

/* Batched solve on device buffers, enqueued on `stream` (hipStream_t, NULL =
 * default stream).  Returns 0 on a successful launch.  Instances whose stage blocks live
 * in global memory (N 30 with 12 obstacles, the bicycle) use a device workspace that
 * libmpcg keeps per stream on the stream's device (reused by later calls on the stream,
 * released by mpcg_release_stream_workspace); contexts own theirs. */
int mpcg_solve(const mpcg_problem *pr, int batch, const mpcg_io *io, void *stream);

/* Frees the workspace mpcg_solve keeps for `stream` (after the stream's work).  Returns 0. */
int mpcg_release_stream_workspace(void *stream);

/* A persistent solve context: device buffers and pinned staging for up to
 * `max_batch` solves plus a private stream, so that one Solver::solve()
 * (batch 1) or one GuidanceConstraints::optimize fan-out (batch = guesses)
 * costs two copies and one launch.  Not thread-safe per context; contexts are
 * independent (one per planner thread, like the reference's one capsule per
 * Solver). */
typedef struct mpcg_context mpcg_context;
mpcg_context *mpcg_context_create(const mpcg_problem *pr, int max_batch);
void mpcg_context_destroy(mpcg_context *ctx);
/* host pointers; synchronous.  Returns 0, or < 0 with mpcg_last_error(). */
int mpcg_context_solve(mpcg_context *ctx, int batch, const mpcg_io *io);
/* SQP-RTI iterations of the next mpcg_context_solve calls (1 = one
 * solveOneIteration(), acados_solver_interface.cpp:145-160).  Returns 0. */
int mpcg_context_set_iterations(mpcg_context *ctx, int sqp_iters);

/* Scene-level inputs of one control step (GuidanceConstraints::optimize) for
 * S scenes x G planners, device pointers.  Semantics and the reference lines
 * each step restates: oscar_mpc_planner_mr_modification_amd/producers.py.
 *   stage_params   [S][npar]         parameters the other modules write identically on every
 *                                    stage (weights, spline segments, disc radius / offset)
 *   state          [S][nx]           ego state (xinit)
 *   obst           [S][n_ell][N][5]  mode-0 prediction j of each obstacle: x y angle major minor
 *                                    (list padded to max_obstacles with the planner's dummies)
 *   obst_meta      [S][n_ell][2]     radius, chi
 *   guidance       [S][G][N+1][4]    guidance trajectory at t = k dt: x y vx vy
 *   guided         [S][G]            1 guided planner, 0 the non-guided T-MPC++ planner
 *   main_warm      [S][N+1][nvar]    the main solver's warm start, or NULL = braking plan
 *   prev_traj      [S][N][2]         stored previous plan, or NULL
 *   prev_elapsed   [S]               seconds since it was stored (NaN: none)
 *   consistency_on [S][G]            planners with the consistency cost, or NULL
 * ABI 6, t-mpc.warmstart_with_mpc_solution (settings.yaml:71; guidance_constraints.cpp:335-338):
 *   planner_xtraj  [S*G][N+1][nx]    each planner's own previous output (its Solver's _output)
 *   planner_utraj  [S*G][N][nu]
 *   existing_guidance [S][G]         the planner's guidance existed in the previous step
 *   warmstart_with_mpc_solution      1: guided planners with existing guidance start from
 *                                    initializeWarmstart(state, shift_forward) of their own
 *                                    previous output instead of the guidance trajectory
 *   shift_forward                    shift_previous_solution_forward && enable_output */
typedef struct mpcg_scene_io {
    const double *stage_params, *state, *obst, *obst_meta, *guidance;
    const unsigned char *guided;
    const double *main_warm, *prev_traj, *prev_elapsed;
    const unsigned char *consistency_on;
    double robot_radius, w_consistency, deceleration;
    const double *planner_xtraj, *planner_utraj;
    const unsigned char *existing_guidance;
    int warmstart_with_mpc_solution, shift_forward;
} mpcg_scene_io;

/* Per-planner solver inputs of one control step on the device: params
 * [S*G][N][npar], warm [S*G][N+1][nvar], xinit [S*G][nx] (the mpcg_io inputs),
 * prev_interp [S][N][2] (the consistency reference, may be NULL) and
 * consistency_active [S*G] (may be NULL), enqueued on `stream`.  Requires
 * nx 5 (the T-MPC problem), N <= 32 and min(n_lin, n_ell) <= 24.  Returns 0 on a successful launch. */
int mpcg_prepare(const mpcg_problem *pr, int n_scenes, int n_guesses, const mpcg_scene_io *in,
                 double *params, double *warm, double *xinit, double *prev_interp,
                 unsigned char *consistency_active, void *stream);

/* SH-MPC inputs of one control step (ScenarioConstraints::optimize,
 * scenario_constraints.cpp:58-84) for S scenes x P parallel solvers, device
 * pointers.  Semantics: oscar_mpc_planner_mr_modification_amd/scenario.py.
 *   stage_params [S][npar]           parameters written identically on every stage
 *                                    (weights incl. "slack", spline segments, disc offset)
 *   state        [S][nx]             ego state (xinit)
 *   main_warm    [S][N+1][nu+nx]     the main solver's warm start, or NULL = braking plan
 *   samples      [S*P][N][M][2]      obstacle prediction samples of every parallel solver at
 *                                    every stage (M = obstacles x samples per obstacle)
 * Each solver's scenario rows at stage k >= 1 are the halfspaces of its
 * n_scen samples closest to the warm-start position p_k (ties: lower sample
 * index): n = (q - p_k) / max(|q - p_k|, 1e-9), b = n . q - radius; stage 0
 * rows are inactive (0, 0, 100).  This reduction restates the external
 * scenario_module (parity unpinned). */
typedef struct mpcg_scenario_io {
    const double *stage_params, *state, *main_warm, *samples;
    int n_samples;                 /* M, at most 2048 */
    double radius;                 /* robot radius + obstacle radius */
    double deceleration;           /* deceleration_at_infeasible (braking plan) */
} mpcg_scenario_io;

/* Outputs params [S*P][N][npar], warm [S*P][N+1][nu+nx], xinit [S*P][nx]
 * (solve = scene * P + solver), enqueued on `stream`.  Requires n_scen in
 * 1..32 and N <= 32.  Returns 0 on a successful launch. */
int mpcg_prepare_scenario(const mpcg_problem *pr, int n_scenes, int n_solvers, const mpcg_scenario_io *in,
                          double *params, double *warm, double *xinit, void *stream);

/* ScenarioConstraints::optimize's pick (scenario_constraints.cpp:86-103): per
 * scene the parallel solver with exit 1 and the lowest pobj below 1e9 (first
 * index on ties), -1 when none.  pobj / exit_code [S*P], best [S], device. */
int mpcg_select_lowest_cost_device(int n_scenes, int n_solvers, const double *pobj, const int *exit_code,
                                   int *best, void *stream);

/* Bookkeeping between two control steps of every scene: the state the
 * reference keeps in Planner / GuidanceConstraints / each LocalPlanner's
 * solver (device pointers; semantics restated in producers.advance_host).
 * Inputs (step t):
 *   best [S]                        FindBestPlanner result, -1 = no feasible planner
 *   exit_code [S*G], xtraj, utraj   the solves of step t
 *   warm [S*G][N+1][nvar]           the warm start each planner used (its x0)
 *   lam_out [S*G][N][nx+nh]         multipliers after the solves, or NULL
 *   state_next [S][nx]              ego state at step t+1
 *   guided [S][G]                   planner kinds (the non-guided one is the "original planner")
 *   topology, topology_next [S][G]  topology class of every planner at t and t+1, or NULL = planner index
 *   previously_selected [S][G]      selection flags at t (kept when no planner was feasible), or NULL
 * Outputs (step t+1):
 *   main_warm_next [S][N+1][nvar]   Planner::solveMPC: initializeWarmstart(state, shift) of the
 *                                   winner's output (x0[N] from the winner's parameters) when step t
 *                                   was feasible, else the braking plan (planner.cpp:129-137)
 *   prev_traj_next [S][N][2], prev_elapsed_next [S]  storePreviousTrajectoryFromSolver (NaN: none)
 *   consistency_on_next [S][G]      shouldEnableConsistencyForPlanner (guidance_constraints.cpp:951-984)
 *   previously_selected_next [S][G] OverrideSelectedTrajectory (:500-513)
 *   lam_next [S*G][N][nx+nh]        each planner's carried multipliers, zeroed after a failed solve */
typedef struct mpcg_step_io {
    const int *best, *exit_code;
    const double *xtraj, *utraj, *warm, *lam_out, *state_next;
    const unsigned char *guided;
    const int *topology, *topology_next;
    const unsigned char *previously_selected;
    int shift_forward;              /* shift_previous_solution_forward && enable_output */
    int consistency_on_non_guided;  /* JULES.consistency_on_non_guided_planner */
    double elapsed;                 /* seconds from step t to step t+1 */
    double deceleration;            /* deceleration_at_infeasible */
} mpcg_step_io;

int mpcg_advance(const mpcg_problem *pr, int n_scenes, int n_guesses, const mpcg_step_io *io,
                 double *main_warm_next, double *prev_traj_next, double *prev_elapsed_next,
                 unsigned char *consistency_on_next, unsigned char *previously_selected_next, double *lam_next,
                 void *stream);

/* 0 if (model, N, nx, n_lin, n_ell, n_scen) has a compiled kernel instance, else -1 */
int mpcg_supported(const mpcg_problem *pr);

/* The compiled instance's storage choices as "key=value ..." text (lane parts per stage,
 * row slots, stored 1/t, LEAN / GFH storage, constant [B A] rows, paired chains, LDS
 * bytes) into buf[len]: 0, or -1 without an instance. */
int mpcg_instance_traits(const mpcg_problem *pr, char *buf, int len);

/* Batched solve, every pointer in device memory, enqueued on `stream`
 * (a hipStream_t, NULL = default stream).  Returns 0 on successful launch. */
int mpcg_solve_batch_device(const mpcg_problem *pr, int batch,
                            const double *params, const double *warm, const double *xinit,
                            double *xtraj, double *utraj, double *pobj, int *exit_code,
                            int *info, void *stream);

/* Same with host buffers: copies in, solves, copies out, synchronises.
 * This is what one `Solver::solve()` call maps to (batch = 1). */
int mpcg_solve_batch_host(const mpcg_problem *pr, int batch,
                          const double *params, const double *warm, const double *xinit,
                          double *xtraj, double *utraj, double *pobj, int *exit_code, int *info);

/* Planner selection per scene == the objective bookkeeping of
 * GuidanceConstraints::optimize (guidance_constraints.cpp:372-420) followed
 * by FindBestPlanner (:572-590):
 *   obj_g = pobj_g - [consistency_g] * w_cons * sum_{k=1}^{N-2} |xy_k - prev_k|^2
 *   obj_g *= selection_weight            if previously_selected_g
 *   best  = argmin obj_g over !disabled && exit == 1, -1 if none (first index wins ties)
 * prev_traj: [n_scenes][N][2] or NULL; flags: [n_scenes][G] bytes, may be NULL.
 * best: [n_scenes], objective out: [n_scenes][G] (may be NULL).  Device pointers. */
int mpcg_select_best_device(int n_scenes, int n_guesses, int N,
                            const double *xtraj, const double *pobj, const int *exit_code,
                            const double *prev_traj, double w_cons,
                            const unsigned char *consistency_enabled,
                            const unsigned char *previously_selected, double selection_weight,
                            const unsigned char *disabled,
                            int *best, double *objective, void *stream);

/* Per-scene record of the selected planner for the winner all-gather (the device form of
 * distributed.winner_records; the reference hands the winner's trajectory to the module,
 * guidance_constraints.cpp:429-442): out[n_scenes][(N+1)*nx + N*nu + 2] =
 * xtraj | utraj | pobj | best of planner max(best, 0) (best == -1: planner 0, index -1 kept).
 * xtraj [n_scenes*G][N+1][nx], utraj [..][N][nu], pobj [..], best [n_scenes].  Device pointers. */
int mpcg_winner_records_device(int n_scenes, int n_guesses, int N, int nx, int nu,
                               const double *xtraj, const double *utraj, const double *pobj,
                               const int *best, double *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCG_H */
