// mpcg_kernels.hip — the C ABI of the MI355X (gfx950) batched T-MPC++ SQP solve
// (include/mpcg.h): problem description from a parameter map, dispatch to the compiled
// kernel instances (mpcg_instance.h; the built-in ones live in mpcg_inst_*.hip), the
// persistent host-buffer context, and the per-scene selection kernels.
//
// The solve kernel itself is sqp_kernel<Cfg<...>> in mpcg_sqp.h: one wavefront (64
// lanes, one workgroup) solves one (scene, guess) pair -- the body of one
// `Solver::solve()` call of the OpenMP fan-out in GuidanceConstraints::optimize
// (guidance_constraints.cpp:304-421), i.e. `sqp_iters` acados SQP-RTI iterations
// (acados_solver_interface.cpp:86-119).  Its lanes are stage x part (stage algebra,
// inequality rows), element lanes of the Riccati block, and vector chains carried in
// SGPRs; inequality-row state lives in registers, stage blocks in LDS; reductions are
// DPP trees read back from lane 63 (see the header of mpcg_sqp.h and DESIGN.md §3).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mpcg.h"
#include "mpcg_device.h"
#include "mpcg_instance.h"

namespace mpcg {

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
                const double dx = xtraj[((size_t)s * (N + 1) + k) * MPCG_NX + 0] - prev[((size_t)sc * N + k) * 2 + 0];
                const double dy = xtraj[((size_t)s * (N + 1) + k) * MPCG_NX + 1] - prev[((size_t)sc * N + k) * 2 + 1];
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

// ---- per-scene record of the selected planner: xtraj | utraj | pobj | index (best -1 records
// planner 0, whose exit code the reference returns then, guidance_constraints.cpp:429-442); one
// wave per scene, coalesced copies
__global__ void winner_records_kernel(int G, int N, int nx, int nu, const double* __restrict__ xtraj,
                                      const double* __restrict__ utraj, const double* __restrict__ pobj,
                                      const int* __restrict__ best, double* __restrict__ out) {
    const int sc = blockIdx.x;
    const int nxt = (N + 1) * nx, nut = N * nu, w = nxt + nut + 2;
    const int b = best[sc];
    const size_t s = (size_t)sc * G + (b < 0 ? 0 : b);
    double* o = out + (size_t)sc * w;
    for (int e = threadIdx.x; e < w; e += blockDim.x) {
        double v;
        if (e < nxt) v = xtraj[s * nxt + e];
        else if (e < nxt + nut) v = utraj[s * nut + (e - nxt)];
        else if (e == nxt + nut) v = pobj[s];
        else v = (double)b;
        o[e] = v;
    }
}

// ---- ScenarioConstraints::optimize's pick (scenario_constraints.cpp:86-103)
__global__ void select_lowest_cost_kernel(int n_scenes, int P, const double* __restrict__ pobj,
                                          const int* __restrict__ exit_code, int* __restrict__ best) {
    const int sc = blockIdx.x * blockDim.x + threadIdx.x;
    if (sc >= n_scenes) return;
    double lowest = 1e9;
    int b = -1;
    for (int s = 0; s < P; ++s) {
        const int i = sc * P + s;
        if (exit_code[i] == 1 && pobj[i] < lowest) {
            lowest = pobj[i];
            b = s;
        }
    }
    best[sc] = b;
}

// ---- dispatch over compiled instances ------------------------------------
thread_local std::string g_err;  // also set by mpcg_prepare.hip
static unsigned long long* g_stamps = nullptr;  // diagnostic stamp buffer (MPCG_STAMPS builds only)

// the instance table (mpcg_instance.h): built-in instances register from mpcg_inst_*.hip,
// generated solvers from the drop-in library codegen.py writes
struct Inst {
    int model = 0, N = 0, nl = 0, ne = 0, ns = 0, nx = 0;
    mpcg_instance_launch fn = nullptr;
    int qpm = 0;         // doubles of one solve's QP memory (Cfg::QPM)
    long long ws = 0;    // workspace bytes of one solve (GFH stage blocks; 0: none)
    const char* traits = "";
};
static std::mutex& registry_mutex() {
    static std::mutex m;
    return m;
}
static std::vector<Inst>& registry() {
    static std::vector<Inst> r;
    return r;
}

static Inst find_instance(const mpcg_problem& pr) {
    if (pr.rk_steps < 1 || pr.n_seg < 1 || pr.n_seg > 16) return {};
    if (pr.nu != (pr.model == MPCG_MODEL_BICYCLE_CA ? 3 : 2)) return {};
    std::lock_guard<std::mutex> l(registry_mutex());
    for (const Inst& in : registry())
        if (in.model == pr.model && in.N == pr.N && in.nl == pr.n_lin && in.ne == pr.n_ell && in.ns == pr.n_scen &&
            in.nx == pr.nx)
            return in;
    return {};
}

static int launch(const Inst& in, const mpcg_problem& pr, int batch, const mpcg_io& io, hipStream_t stream,
                  void* ws) {
    const int e = in.fn(&pr, batch, &io, (void*)stream, g_stamps, ws);
    if (e != (int)hipSuccess) {
        g_err = std::string("sqp_kernel launch: ") + hipGetErrorString((hipError_t)e);
        return -1;
    }
    return 0;
}

// Workspaces of the raw mpcg_solve path, one per (device, stream) on the STREAM's device:
// kernels enqueued on one stream run in order, so one buffer serves every call on it.  The
// lock is held until the launch is enqueued, so a larger request from another thread (which
// synchronises the stream before it replaces the buffer) cannot free it under a launch.
struct StreamWs {
    int dev;
    void* stream;
    void* ptr;
    size_t size;
};
static std::mutex g_ws_mutex;
static std::vector<StreamWs> g_ws;

static int stream_device(hipStream_t stream, int* dev) {
    if (stream) return hipStreamGetDevice(stream, dev) == hipSuccess ? 0 : -1;
    return hipGetDevice(dev) == hipSuccess ? 0 : -1;
}

static int launch_on_stream(const Inst& in, const mpcg_problem& pr, int batch, const mpcg_io& io,
                            hipStream_t stream) {
    // the work-queue words (mpcg_instance.h) then the stage blocks of GFH instances
    const size_t bytes = MPCG_QUEUE_BYTES + (size_t)batch * (size_t)(in.ws > 0 ? in.ws : 0);
    int dev = 0;
    if (stream_device(stream, &dev)) { g_err = "mpcg_solve: no device for the stream"; return -1; }
    std::lock_guard<std::mutex> l(g_ws_mutex);
    StreamWs* w = nullptr;
    for (StreamWs& e : g_ws)
        if (e.dev == dev && e.stream == (void*)stream) w = &e;
    if (!w) {
        g_ws.push_back(StreamWs{dev, (void*)stream, nullptr, 0});
        w = &g_ws.back();
    }
    if (w->size < bytes) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) cur = dev;
        bool ok = hipSetDevice(dev) == hipSuccess;
        if (ok && w->ptr) {
            ok = hipStreamSynchronize(stream) == hipSuccess;
            (void)hipFree(w->ptr);
            w->ptr = nullptr;
            w->size = 0;
        }
        if (ok && hipMalloc(&w->ptr, bytes) != hipSuccess) { w->ptr = nullptr; ok = false; }
        if (ok && hipMemsetAsync(w->ptr, 0, MPCG_QUEUE_BYTES, stream) != hipSuccess) {
            (void)hipFree(w->ptr);
            w->ptr = nullptr;
            ok = false;
        }
        (void)hipSetDevice(cur);
        if (!ok) { g_err = "mpcg_solve: workspace allocation failed"; return -1; }
        w->size = bytes;
    }
    return launch(in, pr, batch, io, stream, w->ptr);
}

static int check_problem(const mpcg_problem* pr, int batch, Inst* inst) {
    if (!pr || batch < 0) { g_err = "invalid arguments"; return -1; }
    if (pr->nlp_solver != MPCG_NLP_SQP_RTI && pr->nlp_solver != MPCG_NLP_SQP) {
        g_err = "nlp_solver must be MPCG_NLP_SQP_RTI or MPCG_NLP_SQP";
        return -1;
    }
    if (pr->nlp_solver == MPCG_NLP_SQP && (pr->nlp_max_iter < 0 || !(pr->nlp_tol > 0.0))) {
        g_err = "MPCG_NLP_SQP needs nlp_max_iter >= 0 and nlp_tol > 0";
        return -1;
    }
    *inst = find_instance(*pr);
    if (!inst->fn) {
        g_err = "no compiled instance for model=" + std::to_string(pr->model) + " N=" + std::to_string(pr->N) +
                " nx=" + std::to_string(pr->nx) + " nu=" + std::to_string(pr->nu) +
                " n_lin=" + std::to_string(pr->n_lin) + " n_ell=" + std::to_string(pr->n_ell) +
                " n_scen=" + std::to_string(pr->n_scen);
        return -2;
    }
    return 0;
}

}  // namespace mpcg

static std::atomic<int> g_rejected_instances{0};

extern "C" int mpcg_rejected_instances(void) { return g_rejected_instances.load(); }

extern "C" int mpcg_register_instance(int abi_version, int model, int N, int n_lin, int n_ell, int n_scen, int nx,
                                      mpcg_instance_launch fn, int qp_mem_size, long long workspace_bytes_per_solve,
                                      const char* traits) {
    if (abi_version != MPCG_ABI_VERSION) {
        // a stale instance library: its kernels read another mpcg_problem / workspace layout
        ++g_rejected_instances;
        std::fprintf(stderr, "mpcg: instance library compiled against ABI %d, libmpcg.so is ABI %d: rebuild it\n",
                     abi_version, MPCG_ABI_VERSION);
        return -3;
    }
    if (!fn) return -1;
    std::lock_guard<std::mutex> l(mpcg::registry_mutex());
    for (const mpcg::Inst& in : mpcg::registry())
        if (in.model == model && in.N == N && in.nl == n_lin && in.ne == n_ell && in.ns == n_scen && in.nx == nx)
            return 0;
    mpcg::Inst in;
    in.model = model; in.N = N; in.nl = n_lin; in.ne = n_ell; in.ns = n_scen; in.nx = nx;
    in.fn = fn;
    in.qpm = qp_mem_size;
    in.ws = workspace_bytes_per_solve;
    in.traits = traits ? traits : "";
    mpcg::registry().push_back(in);
    return 0;
}

// Persistent context (include/mpcg.h): one device allocation for every
// buffer of `max_batch` solves, one pinned staging block, a private stream.
struct mpcg_context {
    mpcg_problem pr;
    mpcg::Inst inst;
    int max_batch = 0;
    hipStream_t stream = nullptr;
    void* ws = nullptr;      // work-queue words + the instance's workspace for max_batch solves (context's device)
    double* dev = nullptr;   // params | warm | xinit | lam_in | qp_in | xtraj | utraj | pobj | lam_out | qp_out | stats
    double* host = nullptr;  // pinned mirror of the same layout
    int* idev = nullptr;     // exit | info
    int* ihost = nullptr;
    size_t n_par, n_warm, n_xi, n_lam, n_qpm, n_xt, n_ut, n_st, n_dbl, n_int;
};

extern "C" {

int mpcg_abi_version(void) { return MPCG_ABI_VERSION; }

/* tests only (tests/test_queue.py): write `value` into the work-queue counter of the workspace that
 * mpcg_solve keeps for `stream`, as a launch that died mid-way would leave it.  Returns 0, or -1
 * when the stream has no workspace yet. */
int mpcg_debug_set_queue(void* stream, unsigned value) {
    std::lock_guard<std::mutex> l(mpcg::g_ws_mutex);
    for (const mpcg::StreamWs& w : mpcg::g_ws)
        if (w.stream == stream && w.ptr) {
            static unsigned v;
            v = value;
            if (hipMemcpyAsync(w.ptr, &v, sizeof v, hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess) return -1;
            return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : -1;
        }
    return -1;
}

/* diagnostic builds only: device buffer of batch x 20 u64 phase-cycle sums */
void mpcg_debug_set_stamp_buffer(unsigned long long* dev_ptr) { mpcg::g_stamps = dev_ptr; }

const char* mpcg_last_error(void) { return mpcg::g_err.c_str(); }

int mpcg_supported(const mpcg_problem* pr) { return (pr && mpcg::find_instance(*pr).fn) ? 0 : -1; }

int mpcg_instance_traits(const mpcg_problem* pr, char* buf, int len) {
    if (!pr || !buf || len < 1) return -1;
    const mpcg::Inst in = mpcg::find_instance(*pr);
    if (!in.fn) return -1;
    std::snprintf(buf, (size_t)len, "%s", in.traits);
    return 0;
}

int mpcg_qp_mem_size(const mpcg_problem* pr) {
    if (!pr) return -1;
    const mpcg::Inst in = mpcg::find_instance(*pr);
    return in.fn ? in.qpm : -1;
}

int mpcg_num_h(const mpcg_problem* pr) { return pr ? pr->n_lin + pr->n_ell + pr->n_scen : 0; }

int mpcg_lam_size(const mpcg_problem* pr) { return pr ? pr->N * (pr->nx + mpcg_num_h(pr)) : 0; }

int mpcg_problem_from_map(mpcg_problem* pr, int N, int nx, int npar, int n_entries, const char* const* names,
                          const int* indices, const double* lb, const double* ub, double dt, int sqp_iters) {
    return mpcg_problem_from_map_model(pr, MPCG_MODEL_UNICYCLE, N, nx, npar, n_entries, names, indices, lb, ub, dt,
                                       sqp_iters);
}

int mpcg_problem_from_map_model(mpcg_problem* pr, int model, int N, int nx, int npar, int n_entries,
                                const char* const* names, const int* indices, const double* lb, const double* ub,
                                double dt, int sqp_iters) {
    const bool bike = model == MPCG_MODEL_BICYCLE_CA;
    if (!pr || !names || !indices || !lb || !ub || N < 1 || npar < 1 || n_entries < 0 || nx < 5 ||
        nx > MPCG_MAX_NX || (model != MPCG_MODEL_UNICYCLE && !bike) || (bike && nx != 6)) {
        mpcg::g_err = "invalid arguments";
        return -1;
    }
    auto find = [&](const std::string& nm) {
        for (int i = 0; i < n_entries; ++i)
            if (names[i] && nm == names[i]) return indices[i];
        return -1;
    };
    std::memset(pr, 0, sizeof(*pr));
    pr->N = N;
    pr->nx = nx;
    pr->nu = bike ? 3 : MPCG_NU;
    pr->model = model;
    pr->npar = npar;
    // MPCBase weights (mpc_base.py:47-60), contouring (contouring.py:114-138)
    pr->i_w_acc = find("acceleration");
    pr->i_w_ang = find("angular_velocity");
    pr->i_w_vel = find("velocity");
    pr->i_v_ref = find("reference_velocity");
    pr->i_w_contour = find("contour");
    pr->i_w_lag = find("lag");
    pr->i_spline0 = find("spline_x0_a");
    // consistency (consistency_module.py:220-227): optional
    pr->i_cons_w = find("consistency_weight");
    pr->i_prev_x = find("prev_traj_x");
    pr->i_prev_y = find("prev_traj_y");
    // disc + obstacles (ellipsoid_constraints.py:406-419), topology halfspaces (guidance_constraints.py:333-338)
    pr->i_disc_r = find("ego_disc_radius");
    pr->i_disc_off = find("ego_disc_0_offset");
    pr->i_lin0 = find("lin_constraint_0_a1");
    pr->i_ell0 = find("ellipsoid_obst_0_x");
    // scenario halfspaces (scenario_constraints.py:41-50) or, bicycle, the decomp
    // halfspaces (decomp_constraints.py:46-54), and the slack weight
    const std::string rows = bike ? "disc_0_decomp_" : "disc_0_scenario_constraint_";
    pr->i_scen0 = find(rows + "0_a1");
    pr->i_w_slack = find("slack");
    pr->i_w_tangle = find("terminal_angle");
    pr->i_w_tcont = find("terminal_contouring");
    const char* required[] = {"acceleration", "angular_velocity", "velocity", "reference_velocity", "contour",
                              "lag", "spline_x0_a", "ego_disc_0_offset"};
    for (const char* r : required)
        if (find(r) < 0) { mpcg::g_err = std::string("parameter map has no '") + r + "'"; return -1; }
    if ((nx > 5 || bike) && pr->i_w_slack < 0) { mpcg::g_err = "parameter map has no 'slack'"; return -1; }
    if (bike && (pr->i_w_tangle < 0 || pr->i_w_tcont < 0)) {
        mpcg::g_err = "parameter map has no 'terminal_angle' / 'terminal_contouring'";
        return -1;
    }
    while (find("spline" + std::to_string(pr->n_seg) + "_start") >= 0) ++pr->n_seg;
    while (find("lin_constraint_" + std::to_string(pr->n_lin) + "_a1") >= 0) ++pr->n_lin;
    while (find("ellipsoid_obst_" + std::to_string(pr->n_ell) + "_x") >= 0) ++pr->n_ell;
    while (find(rows + std::to_string(pr->n_scen) + "_a1") >= 0) ++pr->n_scen;
    if (pr->n_ell > 0 && pr->i_disc_r < 0) { mpcg::g_err = "parameter map has no 'ego_disc_radius'"; return -1; }
    // the kernels read bundles at fixed strides from their base index: check them
    for (int j = 0; j < pr->n_seg; ++j)
        if (find("spline_y" + std::to_string(j) + "_d") != pr->i_spline0 + 9 * j + 7 ||
            find("spline" + std::to_string(j) + "_start") != pr->i_spline0 + 9 * j + 8) {
            mpcg::g_err = "spline segment " + std::to_string(j) + " is not contiguous";
            return -1;
        }
    for (int i = 0; i < pr->n_lin; ++i)
        if (find("lin_constraint_" + std::to_string(i) + "_b") != pr->i_lin0 + 3 * i + 2) {
            mpcg::g_err = "halfspace " + std::to_string(i) + " is not contiguous";
            return -1;
        }
    for (int j = 0; j < pr->n_ell; ++j)
        if (find("ellipsoid_obst_" + std::to_string(j) + "_r") != pr->i_ell0 + 7 * j + 6) {
            mpcg::g_err = "obstacle " + std::to_string(j) + " is not contiguous";
            return -1;
        }
    for (int i = 0; i < pr->n_scen; ++i)
        if (find(rows + std::to_string(i) + "_b") != pr->i_scen0 + 3 * i + 2) {
            mpcg::g_err = "scenario halfspace " + std::to_string(i) + " is not contiguous";
            return -1;
        }
    pr->dt = dt;
    // sim_method_num_steps (generate_acados_solver.py:148-150); the bicycle: one
    // Forces RK4 step of integrator_step (solver_model.py:11-36)
    pr->rk_steps = bike ? 1 : 3;
    const int nu = pr->nu;
    for (int i = 0; i < nu; ++i) { pr->lbu[i] = lb[i]; pr->ubu[i] = ub[i]; }
    for (int i = 0; i < nx; ++i) { pr->lbx[i] = lb[nu + i]; pr->ubx[i] = ub[nu + i]; }
    pr->sqp_iters = sqp_iters;
    pr->qp_tol = 1e-5;
    pr->qp_iter_max = 50;
    pr->reg_eps = 1e-4;
    pr->res_eq_fail = 1e-2;
    // QP start as the reference configures it: qp_solver_warm_start = 2 (generate_acados_solver.py:173)
    // with acados' warm_start_first_qp off, so the first QP of each acados call starts cold -- every
    // QP of the SQP-RTI loop (DESIGN.md §2 "QP start"), the first of a full SQP call
    pr->qp_warm_start = 2;
    pr->qp_ws_thr = 0.1;
    pr->qp_warm_first = 0;
    // solver_type SQP_RTI (settings.yaml:19); SQP: tol 1e-2 (generate_acados_solver.py:144) and
    // acados_template's default nlp_solver_max_iter
    pr->nlp_solver = MPCG_NLP_SQP_RTI;
    pr->nlp_max_iter = 100;
    pr->nlp_tol = 1e-2;
    // the interior point as acados configures HPIPM
    mpcg_problem_set_qp_profile(pr, MPCG_QP_HPIPM);
    return 0;
}

int mpcg_problem_set_qp_profile(mpcg_problem* pr, int profile) {
    if (!pr || (profile != MPCG_QP_HPIPM && profile != MPCG_QP_ROBUST)) {
        mpcg::g_err = "unknown QP profile";
        return -1;
    }
    const bool h = profile == MPCG_QP_HPIPM;
    pr->qp_profile = profile;
    // HPIPM BALANCE (d_ocp_qp_ipm_arg_set_default, applied by acados before the reference's qp_tol /
    // qp_solver_iter_max / qp_solver_warm_start): mu0 1e1, init_var's thr0 1e-1 with the primal box
    // move, t_min = lam_min 1e-16, cond_pred_corr 1, itref_corr_max 2, sigma (mu_aff / mu)^3, the
    // iteration cap before convergence, no divergence test.  Robust: the round-4 constants
    pr->qp_mu0 = h ? 10.0 : 1.0;
    pr->qp_thr0 = h ? 0.1 : 1.0;
    pr->qp_t_min = h ? 1e-16 : 1e-12;
    pr->qp_mu_max = h ? 0.0 : 1e8;
    pr->qp_init_move = h;
    pr->qp_cond_pred_corr = h;
    pr->qp_itref_corr_max = h ? 2 : 0;
    pr->qp_sigma_clip = !h;
    pr->qp_maxit_first = h;
    // BLASFEO's dpotrf continues past a non-positive pivot with a zero inverse (ABI 9)
    pr->qp_pivot_zero = h;
    return 0;
}

static int check_io(const mpcg_io* io) {
    if (!io || !io->params || !io->warm || !io->xinit || !io->xtraj || !io->utraj || !io->pobj || !io->exit_code) {
        mpcg::g_err = "missing buffer";
        return -1;
    }
    return 0;
}

int mpcg_solve(const mpcg_problem* pr, int batch, const mpcg_io* io, void* stream) {
    mpcg::Inst in;
    int rc = mpcg::check_problem(pr, batch, &in);
    if (rc) return rc;
    if (batch == 0) return 0;  // nothing to do: buffers may be NULL
    if (check_io(io)) return -1;
    return mpcg::launch_on_stream(in, *pr, batch, *io, (hipStream_t)stream);
}

int mpcg_release_stream_workspace(void* stream) {
    std::lock_guard<std::mutex> l(mpcg::g_ws_mutex);
    for (size_t i = 0; i < mpcg::g_ws.size();) {
        mpcg::StreamWs& w = mpcg::g_ws[i];
        if (w.stream == stream) {
            int cur = 0;
            if (hipGetDevice(&cur) != hipSuccess) cur = w.dev;
            if (hipSetDevice(w.dev) == hipSuccess) {
                (void)hipStreamSynchronize((hipStream_t)stream);
                if (w.ptr) (void)hipFree(w.ptr);
            }
            (void)hipSetDevice(cur);
            mpcg::g_ws.erase(mpcg::g_ws.begin() + i);
        } else {
            ++i;
        }
    }
    return 0;
}

int mpcg_solve_batch_device(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                            const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                            int* info, void* stream) {
    mpcg_io io{params, warm, xinit, nullptr, xtraj, utraj, pobj, exit_code, info, nullptr};
    return mpcg_solve(pr, batch, &io, stream);
}

mpcg_context* mpcg_context_create(const mpcg_problem* pr, int max_batch) {
    mpcg::Inst in;
    if (mpcg::check_problem(pr, max_batch, &in)) return nullptr;
    if (max_batch < 1) { mpcg::g_err = "max_batch must be >= 1"; return nullptr; }
    auto* c = new mpcg_context();
    c->pr = *pr;
    c->inst = in;
    c->max_batch = max_batch;
    const size_t B = max_batch, N = pr->N;
    c->n_par = B * N * pr->npar;
    const size_t nx = pr->nx;
    c->n_warm = B * (N + 1) * (pr->nu + nx);
    c->n_xi = B * nx;
    c->n_lam = B * (size_t)mpcg_lam_size(pr);
    c->n_qpm = B * (size_t)mpcg_qp_mem_size(pr);
    c->n_xt = B * (N + 1) * nx;
    c->n_ut = B * N * pr->nu;
    c->n_st = B * MPCG_STATS_STRIDE;
    c->n_dbl = c->n_par + c->n_warm + c->n_xi + 2 * c->n_lam + 2 * c->n_qpm + c->n_xt + c->n_ut + B + c->n_st;
    c->n_int = B * (1 + MPCG_INFO_STRIDE);
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&c->dev, c->n_dbl * sizeof(double)) == hipSuccess &&
              hipHostMalloc(&c->host, c->n_dbl * sizeof(double), hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&c->idev, c->n_int * sizeof(int)) == hipSuccess &&
              hipHostMalloc(&c->ihost, c->n_int * sizeof(int), hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&c->ws, MPCG_QUEUE_BYTES + (size_t)max_batch * (size_t)(in.ws > 0 ? in.ws : 0)) ==
                  hipSuccess &&
              hipMemset(c->ws, 0, MPCG_QUEUE_BYTES) == hipSuccess;
    if (!ok) {
        mpcg::g_err = "mpcg_context_create: device allocation failed";
        mpcg_context_destroy(c);
        return nullptr;
    }
    return c;
}

void mpcg_context_destroy(mpcg_context* c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ws) (void)hipFree(c->ws);
    if (c->dev) (void)hipFree(c->dev);
    if (c->idev) (void)hipFree(c->idev);
    if (c->host) (void)hipHostFree(c->host);
    if (c->ihost) (void)hipHostFree(c->ihost);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mpcg_context_set_iterations(mpcg_context* c, int sqp_iters) {
    /* (MPCG_NLP_SQP ignores it: one SQP call per solve) */
    if (!c || sqp_iters < 1) { mpcg::g_err = "invalid arguments"; return -1; }
    c->pr.sqp_iters = sqp_iters;
    return 0;
}

int mpcg_context_solve(mpcg_context* c, int batch, const mpcg_io* io) {
    if (!c || !io || batch < 0 || batch > c->max_batch) {
        mpcg::g_err = "mpcg_context_solve: invalid arguments or batch > max_batch";
        return -1;
    }
    if (batch == 0) return 0;  // nothing to do: buffers may be NULL
    if (!io->params || !io->warm || !io->xinit || !io->xtraj || !io->utraj || !io->pobj || !io->exit_code) {
        mpcg::g_err = "missing buffer";
        return -1;
    }
    const mpcg_problem& pr = c->pr;
    const size_t B = batch, N = pr.N, L = (size_t)mpcg_lam_size(&pr), Q = (size_t)mpcg_qp_mem_size(&pr);
    const size_t nx = pr.nx;
    const size_t nu = pr.nu;
    const size_t s_par = B * N * pr.npar, s_warm = B * (N + 1) * (nu + nx), s_xi = B * nx, s_lam = B * L;
    const size_t s_qpm = B * Q, s_xt = B * (N + 1) * nx, s_ut = B * N * nu, s_st = B * MPCG_STATS_STRIDE;
    // inputs are packed contiguously (params | warm | xinit | lam_in | qp_in) so one copy moves them
    double* h = c->host;
    std::memcpy(h, io->params, s_par * sizeof(double));
    std::memcpy(h + s_par, io->warm, s_warm * sizeof(double));
    std::memcpy(h + s_par + s_warm, io->xinit, s_xi * sizeof(double));
    size_t n_in = s_par + s_warm + s_xi;
    double* d = c->dev;
    const double* d_lam = nullptr;
    const double* d_qpi = nullptr;
    if (io->lam_in) {
        std::memcpy(h + n_in, io->lam_in, s_lam * sizeof(double));
        d_lam = d + n_in;
        n_in += s_lam;
    }
    if (io->qp_in) {
        std::memcpy(h + n_in, io->qp_in, s_qpm * sizeof(double));
        d_qpi = d + n_in;
        n_in += s_qpm;
    }
    // outputs: xtraj | utraj | pobj | lam_out | qp_out | stats, packed from the first output slot
    const size_t o0 = c->n_par + c->n_warm + c->n_xi + c->n_lam + c->n_qpm;
    double* d_out = d + o0;
    double* h_out = c->host + o0;
    size_t n_out = s_xt + s_ut + B;
    double* d_lo = nullptr;
    double* d_qo = nullptr;
    double* d_st = nullptr;
    size_t o_lo = 0, o_qo = 0, o_st = 0;
    if (io->lam_out) { o_lo = n_out; d_lo = d_out + n_out; n_out += s_lam; }
    if (io->qp_out) { o_qo = n_out; d_qo = d_out + n_out; n_out += s_qpm; }
    if (io->stats) { o_st = n_out; d_st = d_out + n_out; n_out += s_st; }
    mpcg_io dio{d, d + s_par, d + s_par + s_warm, d_lam, d_out, d_out + s_xt, d_out + s_xt + s_ut, c->idev,
                c->idev + B, d_lo, d_qpi, d_qo, d_st};
    bool ok = hipMemcpyAsync(d, h, n_in * sizeof(double), hipMemcpyHostToDevice, c->stream) == hipSuccess;
    int rc = ok ? mpcg::launch(c->inst, pr, batch, dio, c->stream, c->ws) : -5;
    if (rc == 0)
        ok = hipMemcpyAsync(h_out, d_out, n_out * sizeof(double), hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
             hipMemcpyAsync(c->ihost, c->idev, B * (1 + MPCG_INFO_STRIDE) * sizeof(int), hipMemcpyDeviceToHost,
                            c->stream) == hipSuccess;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (!ok || e != hipSuccess) {
        mpcg::g_err = std::string("mpcg_context_solve: ") + hipGetErrorString(e != hipSuccess ? e : hipGetLastError());
        return rc ? rc : -4;
    }
    if (rc) return rc;
    std::memcpy(io->xtraj, h_out, s_xt * sizeof(double));
    std::memcpy(io->utraj, h_out + s_xt, s_ut * sizeof(double));
    std::memcpy(io->pobj, h_out + s_xt + s_ut, B * sizeof(double));
    if (io->lam_out) std::memcpy(io->lam_out, h_out + o_lo, s_lam * sizeof(double));
    if (io->qp_out) std::memcpy(io->qp_out, h_out + o_qo, s_qpm * sizeof(double));
    if (io->stats) std::memcpy(io->stats, h_out + o_st, s_st * sizeof(double));
    std::memcpy(io->exit_code, c->ihost, B * sizeof(int));
    if (io->info) std::memcpy(io->info, c->ihost + B, B * MPCG_INFO_STRIDE * sizeof(int));
    return 0;
}

int mpcg_solve_batch_host(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                          const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                          int* info) {
    if (batch == 0) return pr ? 0 : -1;
    mpcg_context* c = mpcg_context_create(pr, batch);
    if (!c) return -3;
    mpcg_io io{params, warm, xinit, nullptr, xtraj, utraj, pobj, exit_code, info, nullptr};
    int rc = mpcg_context_solve(c, batch, &io);
    mpcg_context_destroy(c);
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

int mpcg_winner_records_device(int n_scenes, int n_guesses, int N, int nx, int nu, const double* xtraj,
                               const double* utraj, const double* pobj, const int* best, double* out, void* stream) {
    if (n_scenes < 0 || n_guesses < 1 || N < 1 || nx < 1 || nu < 1 ||
        (n_scenes > 0 && (!xtraj || !utraj || !pobj || !best || !out))) {
        mpcg::g_err = "mpcg_winner_records_device: invalid arguments";
        return -1;
    }
    if (n_scenes == 0) return 0;
    hipLaunchKernelGGL(mpcg::winner_records_kernel, dim3(n_scenes), dim3(64), 0, (hipStream_t)stream, n_guesses, N, nx,
                       nu, xtraj, utraj, pobj, best, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("winner_records launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

int mpcg_select_lowest_cost_device(int n_scenes, int n_solvers, const double* pobj, const int* exit_code, int* best,
                                   void* stream) {
    if (n_scenes < 0 || n_solvers < 1 || (n_scenes > 0 && (!pobj || !exit_code || !best))) {
        mpcg::g_err = "mpcg_select_lowest_cost_device: invalid arguments";
        return -1;
    }
    if (n_scenes == 0) return 0;
    const int T = 64;
    hipLaunchKernelGGL(mpcg::select_lowest_cost_kernel, dim3((n_scenes + T - 1) / T), dim3(T), 0, (hipStream_t)stream,
                       n_scenes, n_solvers, pobj, exit_code, best);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("select_lowest_cost launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // extern "C"
