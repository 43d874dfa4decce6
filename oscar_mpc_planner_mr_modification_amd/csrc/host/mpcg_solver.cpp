// mpcg_solver.cpp — drop-in MPCPlanner::Solver / State / SolverBatch over the
// C ABI of libmpcg.so.  Behaviour follows the reference's acados Solver
// (mpc_planner_solver/src/acados_solver_interface.cpp) method by method; the
// acados capsule's persistent state (NLP iterate and multipliers, ocp_nlp_out)
// is held here as `_iterate` / `_lam` and handed to the kernel on every solve.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <mutex>

#include "mpc_planner_solver/mpcg_solver_interface.h"

namespace MPCPlanner {

// ------------------------------------------------------------ configuration
namespace {
std::mutex g_cfg_mutex;
std::string g_solver_dir, g_settings_file;
bool g_settings_loaded = false;
YamlNode g_settings;

std::string env_or(const char* name, const std::string& fallback) {
    const char* v = std::getenv(name);
    return v ? std::string(v) : fallback;
}

[[noreturn]] void fatal(const std::string& msg) {
    // the reference exits when the solver cannot be created (acados_solver_interface.cpp:35-39)
    std::cerr << "[mpcg] " << msg << std::endl;
    std::exit(1);
}
}  // namespace

void SolverConfig::setSolverDirectory(const std::string& dir) {
    std::lock_guard<std::mutex> l(g_cfg_mutex);
    g_solver_dir = dir;
}

void SolverConfig::setSettingsFile(const std::string& settings_yaml) {
    std::lock_guard<std::mutex> l(g_cfg_mutex);
    g_settings_file = settings_yaml;
    g_settings_loaded = false;
}

std::string SolverConfig::solverDirectory() {
    std::lock_guard<std::mutex> l(g_cfg_mutex);
    return g_solver_dir.empty() ? env_or("MPCG_SOLVER_DIR", ".") : g_solver_dir;
}

std::string SolverConfig::solverFile(const std::string& name) { return solverDirectory() + "/" + name + ".yaml"; }

const YamlNode& SolverConfig::settings() {
    std::lock_guard<std::mutex> l(g_cfg_mutex);
    if (!g_settings_loaded) {
        std::string f = g_settings_file.empty() ? env_or("MPCG_SETTINGS", "") : g_settings_file;
        if (f.empty()) fatal("no planner settings: SolverConfig::setSettingsFile() or MPCG_SETTINGS");
        g_settings = load_yaml_file(f);
        g_settings_loaded = true;
    }
    return g_settings;
}

void SolverConfig::reload() {
    std::lock_guard<std::mutex> l(g_cfg_mutex);
    g_settings_loaded = false;
}

// -------------------------------------------------------------------- State
State::State() {
    _config = load_yaml_file(SolverConfig::solverFile("solver_settings"));
    _model_map = load_yaml_file(SolverConfig::solverFile("model_map"));
    initialize();
}

void State::initialize() {
    _state.assign(_config["nx"].as<int>(), 0.0);
    _nu = _config["nu"].as<int>();
}

int State::index(const std::string& var_name) const {
    const YamlNode& e = _model_map[var_name];
    if (!e.IsDefined()) throw std::runtime_error("State: no variable '" + var_name + "' in model_map.yaml");
    return e[1].as<int>() - _nu;  // states come after the inputs
}

double State::get(std::string&& var_name) const { return _state[index(var_name)]; }

Vec2 State::getPos() const { return Vec2(get("x"), get("y")); }

void State::set(std::string&& var_name, double value) { _state[index(var_name)] = value; }

void State::print() const {
    for (auto it = _model_map.begin(); it != _model_map.end(); ++it)
        if (it->second[0].as<std::string>() == "x")
            std::cout << it->first.as<std::string>() << ": " << get(it->first.as<std::string>()) << "\n";
}

bool State::validData() const {
    const double x = get("x"), y = get("y"), psi = get("psi"), v = get("v");
    if (!std::isfinite(x) || !std::isfinite(y) || !std::isfinite(psi) || !std::isfinite(v)) return false;
    return !(x == 0.0 && y == 0.0 && psi == 0.0 && v == 0.0);
}

// --------------------------------------------------------- solver buffers
AcadosParameters::AcadosParameters() {
    for (double& v : xinit) v = 0.;
    for (double& v : x0) v = 0.;
    for (double& v : all_parameters) v = 0.;
}

void AcadosParameters::printParameters(const YamlNode& parameter_map) const {
    for (int k = 0; k < SOLVER_N; ++k) {
        std::cout << "--- stage " << k << " ---\n";
        for (auto it = parameter_map.begin(); it != parameter_map.end(); ++it) {
            const std::string name = it->first.as<std::string>();
            if (name == "num parameters") continue;
            std::cout << name << ": " << all_parameters[k * SOLVER_NP + it->second.as<int>()] << "\n";
        }
    }
}

void Solver::AcadosInfo::print() const {
    // acados_solver_interface.h:111-122
    std::cout << "SQP iterations: " << sqp_iter << "\nMinimum time for solve [ms]: " << min_time * 1000
              << "\nKKT: " << kkt_norm_inf << "\nSolve Time [ms]: " << solvetime * 1000. << "\nNLP Residuals: " << nlp_res
              << "\nQP iterations: " << qp_iter << "\nQP status: " << qp_status << "\npobj: " << pobj << "\n";
}

Solver::AcadosOutput::AcadosOutput() {
    for (double& v : xtraj) v = 0.;
    for (double& v : utraj) v = 0.;
}

void Solver::AcadosOutput::print() const {
    std::cout << "--- xtraj ---\n";
    for (int k = 0; k <= SOLVER_N; ++k) {
        for (int i = 0; i < SOLVER_NX; ++i) std::cout << xtraj[k * SOLVER_NX + i] << " ";
        std::cout << "\n";
    }
    std::cout << "--- utraj ---\n";
    for (int k = 0; k < SOLVER_N; ++k) {
        for (int i = 0; i < SOLVER_NU; ++i) std::cout << utraj[k * SOLVER_NU + i] << " ";
        std::cout << "\n";
    }
}

// ------------------------------------------------------------------- Solver
Solver::Solver(int solver_id) : _solver_id(solver_id) {
    _config = load_yaml_file(SolverConfig::solverFile("solver_settings"));
    _parameter_map = load_yaml_file(SolverConfig::solverFile("parameter_map"));
    _model_map = load_yaml_file(SolverConfig::solverFile("model_map"));

    N = _config["N"].as<int>();
    nu = _config["nu"].as<unsigned int>();
    nx = _config["nx"].as<unsigned int>();
    nvar = _config["nvar"].as<unsigned int>();
    npar = _config["npar"].as<unsigned int>();
    if (N != SOLVER_N || (int)npar != SOLVER_NP || (int)nx != SOLVER_NX || (int)nu != SOLVER_NU)
        fatal("solver_settings.yaml (N=" + std::to_string(N) + ", npar=" + std::to_string(npar) +
              ") does not match the compiled dimensions in mpcg_solver_dims.h");
    if (SOLVER_MODEL == MPCG_MODEL_BICYCLE_CA ? (nx != 6 || nu != 3) : ((nx != 5 && nx != 6) || nu != MPCG_NU))
        fatal("the MI355X backend implements the contouring unicycle model (nx 5, or 6 with the slack state) and "
              "the curvature-aware bicycle (nx 6, nu 3)");

    const YamlNode& cfg = SolverConfig::settings();
    dt = cfg["integrator_step"].as<double>();
    _num_iterations = cfg["solver_settings"]["acados"]["iterations"].as<int>();
    const std::string solver_type = cfg["solver_settings"]["acados"]["solver_type"].as<std::string>();
    if (solver_type != "SQP" && solver_type != "SQP_RTI")
        fatal("solver_settings.acados.solver_type must be SQP_RTI or SQP, not '" + solver_type + "'");
    if (solver_type == "SQP") _num_iterations = 1;

    // the kernel's problem description from the generator's maps
    std::vector<std::string> names;
    std::vector<int> idx;
    for (auto it = _parameter_map.begin(); it != _parameter_map.end(); ++it) {
        std::string name = it->first.as<std::string>();
        if (name == "num parameters") continue;
        names.push_back(name);
        idx.push_back(it->second.as<int>());
    }
    std::vector<const char*> cnames;
    for (auto& s : names) cnames.push_back(s.c_str());
    std::vector<double> lb(nvar, -1e15), ub(nvar, 1e15);
    for (auto it = _model_map.begin(); it != _model_map.end(); ++it) {
        const int i = it->second[1].as<int>();
        if (i < 0 || i >= (int)nvar) fatal("model_map.yaml: index out of range");
        lb[i] = it->second[2].as<double>();
        ub[i] = it->second[3].as<double>();
    }
    if (mpcg_problem_from_map_model(&_problem, SOLVER_MODEL, N, (int)nx, npar, (int)names.size(), cnames.data(),
                                    idx.data(), lb.data(), ub.data(), dt, _num_iterations) != 0)
        fatal(std::string("parameter map: ") + mpcg_last_error());
    // solver_type SQP: each Solver_acados_solve is a full acados SQP call (nlp_solver_type,
    // generate_acados_solver.py:153; tol 1e-2, :144), run to its own termination by the kernel
    if (solver_type == "SQP") _problem.nlp_solver = MPCG_NLP_SQP;
    if (mpcg_supported(&_problem) != 0)
        fatal("no compiled kernel instance for N=" + std::to_string(N) + ", nx=" + std::to_string(nx) + " with " +
              std::to_string(_problem.n_lin) + " halfspaces, " + std::to_string(_problem.n_ell) + " obstacles and " +
              std::to_string(_problem.n_scen) + " scenario halfspaces");
    _iterate.assign((size_t)(N + 1) * nvar, 0.0);
    _lam.assign((size_t)mpcg_lam_size(&_problem), 0.0);
    reset();
}

Solver::~Solver() {
    if (_ctx) mpcg_context_destroy(_ctx);
}

Solver& Solver::operator=(const Solver& rhs) {
    _params = rhs._params;
    return *this;
}

void Solver::reset() {
    _params = AcadosParameters();
    _info = AcadosInfo();
    _output = AcadosOutput();
}

int Solver::solve() {
    initializeOneIteration();
    // all iterations in one launch: the kernel breaks where the reference's
    // loop breaks (qp_status != 0, acados_solver_interface.cpp:105); the
    // wall-clock timeout (:110-116) is not applied
    run(_num_iterations);
    return completeOneIteration();
}

void Solver::initializeOneIteration() {
    // parameters and xinit are read from _params at launch time
    _info = AcadosInfo();
    _raw_status = 1;
}

int Solver::solveOneIteration() {
    int code = run(1);
    // raw acados status (0 success, 1 nan, 2 max-iter, 3 min-step, 4 qp failure)
    return code == 1 ? 0 : (code == 0 ? 1 : code);
}

int Solver::run(int iterations) {
    if (!_ctx) {
        _ctx = mpcg_context_create(&_problem, 1);
        if (!_ctx) fatal(std::string("cannot create the GPU solve context: ") + mpcg_last_error());
    }
    mpcg_context_set_iterations(_ctx, iterations);
    std::vector<double> xt((size_t)nx * (N + 1)), ut((size_t)nu * N), lam_out(_lam.size());
    std::vector<double> qp_out((size_t)mpcg_qp_mem_size(&_problem));
    double pobj = 0., stats[MPCG_STATS_STRIDE] = {0., 0., 0., 0.};
    int exit_code = 0, info[MPCG_INFO_STRIDE] = {0, 0, 0, 0};
    mpcg_io io{_params.all_parameters, _iterate.data(), _params.xinit, _lam.data(),
               xt.data(), ut.data(), &pobj, &exit_code, info, lam_out.data(),
               _qp.empty() ? nullptr : _qp.data(), qp_out.data(), stats};
    const auto t0 = std::chrono::steady_clock::now();
    if (mpcg_context_solve(_ctx, 1, &io) != 0) {
        std::cerr << "[mpcg] solve failed: " << mpcg_last_error() << std::endl;
        _raw_status = 0;
        return 0;
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    absorb(xt.data(), ut.data(), pobj, exit_code, info, lam_out.data(), qp_out.data(), stats, sec);
    return exit_code;
}

void Solver::absorb(const double* xtraj, const double* utraj, double pobj, int exit_code, const int* info,
                    const double* lam, const double* qp, const double* stats, double seconds) {
    for (int k = 0; k <= N; ++k) {
        for (unsigned i = 0; i < nu; ++i) _iterate[k * nvar + i] = k < N ? utraj[k * nu + i] : 0.0;
        for (unsigned i = 0; i < nx; ++i) _iterate[k * nvar + nu + i] = xtraj[k * nx + i];
    }
    for (size_t i = 0; i < _lam.size(); ++i) _lam[i] = lam[i];
    _qp.assign(qp, qp + mpcg_qp_mem_size(&_problem));
    _info.pobj = pobj;
    _info.sqp_iter += info[0];
    _info.qp_iter += info[1];
    _info.qp_status = info[2];  // the acados QP status, as ocp_nlp_get("qp_status") stores it (:157)
    _info.res_stat = stats[0];
    _info.res_eq = stats[1];
    _info.res_ineq = stats[2];
    _info.res_comp = stats[3];
    _info.nlp_res = std::max(std::max(stats[0], stats[1]), std::max(stats[2], stats[3]));
    _info.kkt_norm_inf = _info.nlp_res;
    const double per_iter = seconds / std::max(1, info[0]);
    _info.elapsed_time = per_iter;
    _info.solvetime += seconds;
    _info.min_time = std::min(_info.min_time, per_iter);
    _raw_status = exit_code;
}

int Solver::completeOneIteration() {
    for (int k = 0; k <= N; ++k)
        for (unsigned i = 0; i < nx; ++i) _output.xtraj[k * nx + i] = _iterate[k * nvar + nu + i];
    for (int k = 0; k < N; ++k)
        for (unsigned i = 0; i < nu; ++i) _output.utraj[k * nu + i] = _iterate[k * nvar + i];
    _exit_code_one_iter = _raw_status;  // res_eq rule and the 0 <-> 1 swap were applied by the kernel
    if (_exit_code_one_iter != 1) {
        // Solver_acados_reset(capsule, 1): the capsule's iterate and multipliers go back to zero, and
        // ocp_nlp_solver_reset_qp_memory drops the QP warm start (:186-190)
        std::fill(_iterate.begin(), _iterate.end(), 0.0);
        std::fill(_lam.begin(), _lam.end(), 0.0);
        _qp.clear();
    }
    return _exit_code_one_iter;
}

int Solver::model_index(const std::string& name) const {
    const YamlNode& e = _model_map[name];
    if (!e.IsDefined()) throw std::runtime_error("Solver: no variable '" + name + "' in model_map.yaml");
    return e[1].as<int>();
}

bool Solver::is_state(const std::string& name) const { return _model_map[name][0].as<std::string>() == "x"; }

bool Solver::hasParameter(std::string&& parameter) { return _parameter_map[parameter].IsDefined(); }

void Solver::setParameter(int k, std::string&& parameter, double value) {
    _params.all_parameters[k * npar + _parameter_map[parameter].as<int>()] = value;
}

void Solver::setParameter(int k, std::string& parameter, double value) {
    _params.all_parameters[k * npar + _parameter_map[parameter].as<int>()] = value;
}

double Solver::getParameter(int k, std::string&& parameter) {
    return _params.all_parameters[k * npar + _parameter_map[parameter].as<int>()];
}

void Solver::setXinit(std::string&& state_name, double value) { _params.xinit[model_index(state_name) - nu] = value; }

void Solver::setXinit(const State& state) {
    for (auto it = _model_map.begin(); it != _model_map.end(); ++it)
        if (it->second[0].as<std::string>() == "x") {
            std::string name = it->first.as<std::string>();
            setXinit(std::string(name), state.get(std::string(name)));
        }
}

void Solver::setEgoPrediction(unsigned int k, std::string&& var_name, double value) {
    _params.x0[k * nvar + model_index(var_name)] = value;
}

double Solver::getEgoPrediction(unsigned int k, std::string&& var_name) {
    return _params.x0[k * nvar + model_index(var_name)];
}

void Solver::setEgoPredictionPosition(unsigned int k, const Vec2& value) {
    setEgoPrediction(k, "x", value(0));
    setEgoPrediction(k, "y", value(1));
}

Vec2 Solver::getEgoPredictionPosition(unsigned int k) { return Vec2(getEgoPrediction(k, "x"), getEgoPrediction(k, "y")); }

void Solver::loadWarmstart() {
    // x0 -> the capsule's iterate: u and x for k < N, x only at N (:274-284)
    for (int k = 0; k < N; ++k)
        for (unsigned i = 0; i < nvar; ++i) _iterate[k * nvar + i] = _params.x0[k * nvar + i];
    for (unsigned i = 0; i < nx; ++i) _iterate[N * nvar + nu + i] = _params.x0[N * nvar + nu + i];
}

void Solver::initializeWithState(const State& initial_state) {
    for (int k = 0; k <= N; ++k)
        for (auto it = _model_map.begin(); it != _model_map.end(); ++it) {
            std::string name = it->first.as<std::string>();
            double v = it->second[0].as<std::string>() == "x" ? initial_state.get(std::string(name)) : 0.;
            setEgoPrediction(k, std::move(name), v);
        }
}

void Solver::initializeWithBraking(const State& initial_state) {
    initializeWithState(initial_state);
    const double decel = std::abs(SolverConfig::settings()["deceleration_at_infeasible"].as<double>());
    double x = initial_state.get("x"), y = initial_state.get("y"), psi = initial_state.get("psi");
    double v = initial_state.get("v"), spline = initial_state.get("spline");
    const double a = -decel;
    auto put = [&](int k) {
        setEgoPrediction(k, "x", x);
        setEgoPrediction(k, "y", y);
        setEgoPrediction(k, "psi", psi);
        setEgoPrediction(k, "v", v);
        setEgoPrediction(k, "spline", spline);
        setEgoPrediction(k, "a", a);
        setEgoPrediction(k, "w", 0.);
    };
    put(0);
    for (int k = 1; k <= N; ++k) {  // :320-341
        x += v * dt * std::cos(psi);
        y += v * dt * std::sin(psi);
        spline += v * dt;
        v += a * dt;
        v = std::max(v, 0.);
        put(k);
    }
}

void Solver::initializeWarmstart(const State& initial_state, bool shift_previous_solution_forward) {
    for (auto it = _model_map.begin(); it != _model_map.end(); ++it) {
        const std::string name = it->first.as<std::string>();
        if (shift_previous_solution_forward) {
            // [initial_state, x_2, ..., x_{N-1}, x_{N-1}, x_{N-1}] (:346-368)
            for (int k = 0; k <= N; ++k) {
                double v;
                if (k == 0) v = initial_state.get(std::string(name));
                else if (k >= N - 1) v = getOutput(N - 1, std::string(name));
                else v = getOutput(k + 1, std::string(name));
                setEgoPrediction(k, std::string(name), v);
            }
        } else {
            for (int k = 0; k < N; ++k) setEgoPrediction(k, std::string(name), getOutput(k, std::string(name)));
        }
    }
}

double Solver::getOutput(int k, std::string&& state_name) const {
    const int i = model_index(state_name);
    if (is_state(state_name)) return _output.xtraj[k * nx + i - nu];
    return _output.utraj[k * nu + i];
}

std::string Solver::explainExitFlag(int exitflag) const {
    switch (exitflag) {
        case 1: return "Success";
        case 0: return "Failure (no more information)";
        case 2: return "Failure (maximum number of iterations reached)";
        case 3: return "Failure (minimum step size reached)";
        case 4: break;
        default: return "Unknown exit code; code: " + std::to_string(exitflag);
    }
    switch (_info.qp_status) {
        case 1: return "QP Failure: No more information on QP failure";
        case 2: return "QP Failure: Max Iterations";
        case 3: return "QP Failure: Minimal Step Reached";
        case 4: return "QP Failure: NAN in solution";
        case 5: return "QP Failure: Inconsistent Equality Constraints";
        default: return "QP Failure: UNKNOWN";
    }
}

void Solver::printIfBoundLimited() const {
    for (int k = 0; k < N; ++k)
        for (auto it = _model_map.begin(); it != _model_map.end(); ++it) {
            const std::string name = it->first.as<std::string>();
            if (k == 0 && it->second[0].as<std::string>() == "x") continue;
            const double v = getOutput(k, std::string(name));
            if (std::abs(v - it->second[2].as<double>()) < 1e-2) std::cerr << name << " limited by lower bound\n";
            if (std::abs(v - it->second[3].as<double>()) < 1e-2) std::cerr << name << " limited by upper bound\n";
        }
}

// --------------------------------------------------------------- SolverBatch
SolverBatch::SolverBatch(const Solver& prototype, int max_batch) : _problem(prototype._problem), _max_batch(max_batch) {
    if (max_batch < 1) fatal("SolverBatch: max_batch must be >= 1");
}

SolverBatch::~SolverBatch() {
    if (_ctx) mpcg_context_destroy(_ctx);
}

std::vector<int> SolverBatch::solve(const std::vector<Solver*>& solvers) {
    const int B = (int)solvers.size();
    std::vector<int> codes(B, 0);
    if (B == 0) return codes;
    if (B > _max_batch) fatal("SolverBatch: more solvers than max_batch");
    if (!_ctx) {
        _ctx = mpcg_context_create(&_problem, _max_batch);
        if (!_ctx) fatal(std::string("cannot create the GPU solve context: ") + mpcg_last_error());
    }
    const Solver& s0 = *solvers[0];
    const size_t P = (size_t)s0.N * s0.npar, W = (size_t)(s0.N + 1) * s0.nvar, X = s0.nx, L = s0._lam.size();
    const size_t XT = (size_t)(s0.N + 1) * s0.nx, UT = (size_t)s0.N * s0.nu;
    _params.resize(B * P);
    _warm.resize(B * W);
    _xinit.resize(B * X);
    _lam_in.resize(B * L);
    const size_t Q = (size_t)mpcg_qp_mem_size(&_problem);
    _xtraj.resize(B * XT);
    _utraj.resize(B * UT);
    _pobj.resize(B);
    _lam_out.resize(B * L);
    _qp_in.resize(B * Q);
    _qp_out.resize(B * Q);
    _stats.resize((size_t)B * MPCG_STATS_STRIDE);
    _exit.resize(B);
    _info.resize((size_t)B * MPCG_INFO_STRIDE);
    // the QP memory goes in as one block; a solver without one (fresh or reset) gets a block
    // whose first value is NaN, which the kernel treats as absent (its first QP starts cold)
    bool any_qp = false;
    for (Solver* s : solvers) any_qp = any_qp || !s->_qp.empty();
    for (int b = 0; b < B; ++b) {
        Solver& s = *solvers[b];
        if (s.N != s0.N || s.npar != s0.npar || s._num_iterations != s0._num_iterations)
            fatal("SolverBatch: solvers of different problems in one batch");
        s.initializeOneIteration();
        std::copy(s._params.all_parameters, s._params.all_parameters + P, _params.begin() + b * P);
        std::copy(s._iterate.begin(), s._iterate.end(), _warm.begin() + b * W);
        std::copy(s._params.xinit, s._params.xinit + X, _xinit.begin() + b * X);
        std::copy(s._lam.begin(), s._lam.end(), _lam_in.begin() + b * L);
        if (!s._qp.empty()) std::copy(s._qp.begin(), s._qp.end(), _qp_in.begin() + b * Q);
        else if (Q) _qp_in[b * Q] = std::nan("");
    }
    mpcg_context_set_iterations(_ctx, s0._num_iterations);
    mpcg_io io{_params.data(), _warm.data(), _xinit.data(), _lam_in.data(), _xtraj.data(), _utraj.data(),
               _pobj.data(), _exit.data(), _info.data(), _lam_out.data(), any_qp ? _qp_in.data() : nullptr,
               _qp_out.data(), _stats.data()};
    const auto t0 = std::chrono::steady_clock::now();
    if (mpcg_context_solve(_ctx, B, &io) != 0) {
        std::cerr << "[mpcg] batched solve failed: " << mpcg_last_error() << std::endl;
        for (int b = 0; b < B; ++b) {
            solvers[b]->_raw_status = 0;
            codes[b] = solvers[b]->completeOneIteration();
        }
        return codes;
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int b = 0; b < B; ++b) {
        Solver& s = *solvers[b];
        s.absorb(&_xtraj[b * XT], &_utraj[b * UT], _pobj[b], _exit[b], &_info[(size_t)b * MPCG_INFO_STRIDE],
                 &_lam_out[b * L], &_qp_out[b * Q], &_stats[(size_t)b * MPCG_STATS_STRIDE], sec);
        codes[b] = s.completeOneIteration();
    }
    return codes;
}

}  // namespace MPCPlanner
