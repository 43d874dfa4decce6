// mpcg_solver_interface.h — drop-in `MPCPlanner::Solver` over the MI355X backend.
//
// Same public surface as the reference's acados Solver
// (mpc_planner_solver/include/mpc_planner_solver/acados_solver_interface.h:51-222):
// the per-solver buffers (AcadosParameters / AcadosInfo / AcadosOutput with
// the reference's member names and layouts), the dimensions, the YAML maps,
// and every method the planner and the modules call.  A solve runs the
// batched HIP SQP kernel (libmpcg.so, include/mpcg.h) on batch 1, or on all
// guesses at once through SolverBatch (the replacement of the OpenMP fan-out
// in GuidanceConstraints::optimize, guidance_constraints.cpp:304-421; see
// INTEGRATION.md).
//
// Compile-time dimensions come from the generated mpcg_solver_dims.h
// (SOLVER_N, SOLVER_NP, SOLVER_NX, SOLVER_NU), as the reference takes them
// from the generated acados_solver_Solver.h.
#pragma once

#include <string>
#include <vector>

#include "mpc_planner_solver/mpcg_config.h"
#include "mpc_planner_solver/mpcg_solver_dims.h"
#include "mpc_planner_solver/state.h"
#include "mpcg.h"

// The reference header's short dimension names (acados_solver_interface.h:20-47), over the generated
// SOLVER_* values, for code compiled against that header.  MPCG_NO_DIM_MACROS leaves them out where a
// translation unit has its own NX / NU / ... identifiers.
#ifndef MPCG_NO_DIM_MACROS
#define NX SOLVER_NX
#define NZ SOLVER_NZ
#define NU SOLVER_NU
#define NBX SOLVER_NBX
#define NBX0 SOLVER_NBX0
#define NBU SOLVER_NBU
#define NSBX SOLVER_NSBX
#define NSBU SOLVER_NSBU
#define NSH SOLVER_NSH
#define NSG SOLVER_NSG
#define NSPHI SOLVER_NSPHI
#define NSHN SOLVER_NSHN
#define NSGN SOLVER_NSGN
#define NSPHIN SOLVER_NSPHIN
#define NSBXN SOLVER_NSBXN
#define NS SOLVER_NS
#define NSN SOLVER_NSN
#define NG SOLVER_NG
#define NBXN SOLVER_NBXN
#define NGN SOLVER_NGN
#define NY0 SOLVER_NY0
#define NY SOLVER_NY
#define NYN SOLVER_NYN
#define NH SOLVER_NH
#define NPHI SOLVER_NPHI
#define NHN SOLVER_NHN
#define NPHIN SOLVER_NPHIN
#define NR SOLVER_NR
#endif

namespace MPCPlanner {

// Input block of one solve (acados_solver_interface.h:51-90).
struct AcadosParameters {
    double xinit[SOLVER_NX];                                   // initial state
    double x0[(SOLVER_NU + SOLVER_NX) * (SOLVER_N + 1)];       // warm start [u0 x0 | u1 x1 | ... | uN xN]
    double all_parameters[SOLVER_NP * SOLVER_N];               // horizon-major: [k * SOLVER_NP + index]
    double solver_timeout{0.};                                 // accepted, not used (fixed iteration count)

    double* getU0() { return x0; }

    AcadosParameters();
    void printParameters(const YamlNode& parameter_map) const;
};

class Solver {
public:
    // acados_solver_interface.h:96-124
    // Filled as the reference fills it (acados_solver_interface.cpp:137, 151-153, 164, 193-194):
    //   qp_status     the acados QP status of the last RTI iteration, unchanged (0 ok, 1 nan,
    //                 2 max-iter, 3 min-step), as ocp_nlp_get("qp_status") returns it
    //   nlp_res       max of the NLP residuals (stationarity, dynamics, inequalities,
    //   kkt_norm_inf  complementarity) at the last linearisation point (acados computes them
    //                 in the feedback step; the kernel returns them in mpcg_io.stats)
    //   sqp_iter      RTI iterations executed since initializeOneIteration
    //   elapsed_time  host wall time of the last kernel call per RTI iteration (time_tot of one
    //                 Solver_acados_solve), solvetime = their sum, min_time = their minimum
    struct AcadosInfo {
        double min_time = 1e12;
        double kkt_norm_inf = 0.;
        double elapsed_time = 0.;
        int sqp_iter = 0;
        double nlp_res = 0.;
        double solvetime = 0.;
        int qp_status = 0;
        double pobj{0.};
        int qp_iter = 0;          // total interior-point iterations of the last solve (extra)
        double res_stat = 0., res_eq = 0., res_ineq = 0., res_comp = 0.;  // the four residuals (extra)
        void print() const;
    };

    // acados_solver_interface.h:126-148
    struct AcadosOutput {
        double xtraj[SOLVER_NX * (SOLVER_N + 1)];
        double utraj[SOLVER_NU * SOLVER_N];
        AcadosOutput();
        void print() const;
    };

    int _solver_id;

    AcadosParameters _params;
    AcadosInfo _info;
    AcadosOutput _output;

    int N;
    unsigned int nu;
    unsigned int nx;
    unsigned int nvar;
    unsigned int npar;
    double dt;

    YamlNode _config, _parameter_map, _model_map;

    int _num_iterations;

    explicit Solver(int solver_id = 0);
    ~Solver();
    Solver(const Solver&) = delete;

    // Copies the parameters only (acados_solver_interface.cpp:67-77): the
    // multipliers this solver kept from its own previous solve stay.
    Solver& operator=(const Solver& rhs);

    void reset();

    int solve();

    // One iteration at a time (acados_solver_interface.cpp:121-204)
    void initializeOneIteration();
    int solveOneIteration();
    int completeOneIteration();

    // PARAMETERS
    bool hasParameter(std::string&& parameter);
    void setParameter(int k, std::string&& parameter, double value);
    void setParameter(int k, std::string& parameter, double value);
    double getParameter(int k, std::string&& parameter);

    // XINIT
    void setXinit(std::string&& state_name, double value);
    void setXinit(const State& state);

    // WARMSTART
    void setEgoPrediction(unsigned int k, std::string&& var_name, double value);
    double getEgoPrediction(unsigned int k, std::string&& var_name);
    void setEgoPredictionPosition(unsigned int k, const Vec2& value);
    Vec2 getEgoPredictionPosition(unsigned int k);

    void loadWarmstart();
    void initializeWarmstart(const State& state, bool shift_previous_solution_forward);
    void initializeWithState(const State& initial_state);
    void initializeWithBraking(const State& initial_state);

    // OUTPUT
    double getOutput(int k, std::string&& state_name) const;

    // DEBUG
    std::string explainExitFlag(int exitflag) const;
    void printIfBoundLimited() const;

    // ---- backend access (not in the reference surface)
    const mpcg_problem& problem() const { return _problem; }
    // NLP multipliers carried between solves, [N][nx + nh] (include/mpcg.h, mpcg_io)
    std::vector<double>& multipliers() { return _lam; }
    // the capsule's QP memory (HPIPM warm start of the next QP), empty after a reset
    const std::vector<double>& qpMemory() const { return _qp; }

private:
    friend class SolverBatch;
    mpcg_problem _problem;
    mpcg_context* _ctx = nullptr;   // created on the first solve (no GPU needed before)
    std::vector<double> _iterate;   // NLP iterate [u x] per stage, what loadWarmstart loads (ocp_nlp_out x/u)
    std::vector<double> _lam;       // ocp_nlp_out multipliers
    std::vector<double> _qp;        // QP memory (mpcg_io.qp_out of the last call); empty = fresh / reset
    int _exit_code_one_iter = -1;
    int _raw_status = 0;            // kernel exit code of the last call (already mapped to the 1/0/2/3/4 convention)

    int run(int iterations);
    void absorb(const double* xtraj, const double* utraj, double pobj, int exit_code, const int* info,
                const double* lam, const double* qp, const double* stats, double seconds);
    int model_index(const std::string& name) const;
    bool is_state(const std::string& name) const;
};

// All guesses of one GuidanceConstraints::optimize call in one launch.
// solve() is equivalent to calling Solver::solve() on each solver in turn
// (same results, same side effects on each solver's outputs, info and
// multipliers) and returns their exit codes.
class SolverBatch {
public:
    SolverBatch(const Solver& prototype, int max_batch);
    ~SolverBatch();
    SolverBatch(const SolverBatch&) = delete;
    SolverBatch& operator=(const SolverBatch&) = delete;

    std::vector<int> solve(const std::vector<Solver*>& solvers);

private:
    mpcg_problem _problem;
    int _max_batch;
    mpcg_context* _ctx = nullptr;
    std::vector<double> _params, _warm, _xinit, _lam_in, _xtraj, _utraj, _pobj, _lam_out, _qp_in, _qp_out, _stats;
    std::vector<int> _exit, _info;
};

}  // namespace MPCPlanner
