// Tests of the drop-in MPCPlanner::Solver surface (TEST INFRASTRUCTURE).
//
//   test_solver plumbing                  CPU only: maps, parameters, xinit,
//                                          warm start, outputs, generated setters,
//                                          YAML reader (the reference's
//                                          mpc_planner_solver/test/test_solver.cpp
//                                          checks the same plumbing)
//   test_solver solve <in.bin> <out.bin>  GPU: Solver::solve() per planner,
//                                          SolverBatch over all planners and the
//                                          one-iteration interface on the same inputs
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "mpc_planner_solver/mpc_planner_parameters.h"
#include "mpc_planner_solver/solver_interface.h"

using namespace MPCPlanner;

// the reference header's short dimension names (acados_solver_interface.h:20-47) over the generated values
static_assert(NX == SOLVER_NX && NU == SOLVER_NU && NH == SOLVER_NH && NZ == 0, "dimension macros");
static_assert(NBX == NX && NBX0 == NX && NBU == NU, "box bounds on every state and input");
static_assert(NS == 0 && NSN == 0 && NG == 0 && NY == 0 && NHN == 0 && NBXN == 0 && NR == 0, "no soft / LS / terminal");
static_assert(sizeof(AcadosParameters::x0) == sizeof(double) * (NU + NX) * (SOLVER_N + 1), "x0 layout");

static int g_fail = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            std::cerr << "CHECK failed: " #c " (" << __FILE__ << ":" << __LINE__ << ")\n"; \
            ++g_fail;                                                              \
        }                                                                          \
    } while (0)

static void test_yaml() {
    const char* doc =
        "# planner\nname: \"jackal\" # quoted\nN: 30\nintegrator_step: 0.2\nsolver_settings:\n"
        "  solver: \"acados\"\n  acados:\n    iterations: 10\n    solver_type: SQP_RTI # comment\n"
        "weights: [1, 2.5, 3]\nflag: true\nempty:\nm:\n- x\n- 2\n- -2000.0\n- 2000.0\n";
    mpcg::YamlNode n = mpcg::yaml_parse(doc);
    CHECK(n["name"].as<std::string>() == "jackal");
    CHECK(n["N"].as<int>() == 30);
    CHECK(std::abs(n["integrator_step"].as<double>() - 0.2) < 1e-15);
    CHECK(n["solver_settings"]["acados"]["iterations"].as<int>() == 10);
    CHECK(n["solver_settings"]["acados"]["solver_type"].as<std::string>() == "SQP_RTI");
    CHECK(n["weights"].size() == 3 && n["weights"][1].as<double>() == 2.5);
    CHECK(n["flag"].as<bool>());
    CHECK(n["empty"].IsDefined() && n["empty"].IsNull());
    CHECK(!n["missing"].IsDefined() && !n["missing"]["deeper"].IsDefined());
    CHECK(n["m"].IsSequence() && n["m"][0].as<std::string>() == "x" && n["m"][1].as<int>() == 2);
    CHECK(n["m"][2].as<double>() == -2000.0);
    bool threw = false;
    try {
        (void)n["name"].as<int>();
    } catch (const std::exception&) {
        threw = true;
    }
    CHECK(threw);
}

static void test_plumbing() {
    test_yaml();

    State state;
    state.set("x", 1.5);
    state.set("y", 3.5);
    CHECK(state.get("y") == 3.5);
    CHECK(state.get("x") == 1.5);
    CHECK(state.getPos()(0) == 1.5 && state.getPos()(1) == 3.5);
    CHECK(state.validData());
    CHECK(!State().validData());

    Solver solver;
    CHECK(solver.nu + solver.nx == solver.nvar);
    CHECK(solver.npar > 0 && (int)solver.npar == SOLVER_NP);
    CHECK(solver.dt > 0.);
    CHECK(solver.N == SOLVER_N);
    CHECK(solver._num_iterations == 10);
    CHECK(solver.problem().n_lin + solver.problem().n_ell + solver.problem().n_scen == SOLVER_NH);
    CHECK(solver.problem().nx == SOLVER_NX);
    CHECK((int)solver.multipliers().size() == SOLVER_N * (SOLVER_NX + SOLVER_NH));

    for (int k = 0; k < solver.N; k++) solver.setParameter(k, "reference_velocity", 1.);
    for (int k = 0; k < solver.N; k++) CHECK(solver.getParameter(k, "reference_velocity") == 1.);
    std::string name = "contour";
    solver.setParameter(3, name, 0.25);
    CHECK(solver.getParameter(3, "contour") == 0.25);
    CHECK(solver.hasParameter("lag"));
    CHECK(!solver.hasParameter("no_such_parameter"));

    // generated setters (generate_cpp_files.py:235-254 semantics)
    setSolverParameterAcceleration(2, solver._params, 0.34);
    CHECK(solver.getParameter(2, "acceleration") == 0.34);
    setSolverParameterSplineXA(4, solver._params, 7.0, 2);
    CHECK(solver.getParameter(4, "spline_x2_a") == 7.0);
#if SOLVER_N_ELL > 1
    setSolverParameterEllipsoidObstPsi(5, solver._params, 0.5, 1);
    CHECK(solver.getParameter(5, "ellipsoid_obst_1_psi") == 0.5);
#endif
#if SOLVER_N_LIN > 3
    setSolverParameterLinConstraintB(6, solver._params, -1.25, 3);
    CHECK(solver.getParameter(6, "lin_constraint_3_b") == -1.25);
#endif
#if SOLVER_MODEL == 1 && SOLVER_N_SCEN > 3
    // decomp_constraints.py:46-54: bundles decomp_a1 / decomp_a2 / decomp_b over the constraint index
    setSolverParameterDecompB(6, solver._params, -1.25, 3);
    CHECK(solver.getParameter(6, "disc_0_decomp_3_b") == -1.25);
    setSolverParameterSlack(1, solver._params, 10000.);
    CHECK(solver.getParameter(1, "slack") == 10000.);
#elif SOLVER_N_SCEN > 3
    // scenario_constraints.py:41-50: one bundle per scalar
    setSolverParameterDisc0ScenarioConstraint3B(6, solver._params, -1.25);
    CHECK(solver.getParameter(6, "disc_0_scenario_constraint_3_b") == -1.25);
    setSolverParameterSlack(1, solver._params, 10000.);
    CHECK(solver.getParameter(1, "slack") == 10000.);
#endif

    solver.setXinit("x", 5.4);
    solver.setXinit("y", 1.4);
    double sum = 0.;
    for (unsigned i = 0; i < solver.nx; i++) sum += solver._params.xinit[i];
    CHECK(std::abs(sum - 6.8) < 1e-12);
    State s2;
    s2.set("x", 4.4);
    s2.set("y", 1.2);
    solver.setXinit(s2);
    sum = 0.;
    for (unsigned i = 0; i < solver.nx; i++) sum += solver._params.xinit[i];
    CHECK(std::abs(sum - 5.6) < 1e-12);

    for (int k = 0; k < solver.N; k++) {
        solver.setEgoPrediction(k, "x", k * 1.);
        solver.setEgoPrediction(k, "y", 0.);
    }
    for (int k = 0; k < solver.N; k++) CHECK(solver.getEgoPrediction(k, "x") == k * 1.);
    solver.setEgoPredictionPosition(3, Vec2(9.0, -2.0));
    CHECK(solver.getEgoPredictionPosition(3)(0) == 9.0 && solver.getEgoPredictionPosition(3)(1) == -2.0);
    CHECK(solver._params.x0[3 * solver.nvar + solver._model_map["x"][1].as<int>()] == 9.0);

    // outputs: xtraj[k * nx + (index - nu)], utraj[k * nu + index]
    for (int k = 0; k <= solver.N; k++)
        for (unsigned i = 0; i < solver.nx; i++) solver._output.xtraj[k * solver.nx + i] = 100. * k + i;
    for (int k = 0; k < solver.N; k++)
        for (unsigned i = 0; i < solver.nu; i++) solver._output.utraj[k * solver.nu + i] = -100. * k - i;
    CHECK(solver.getOutput(4, "psi") == 402.);
    CHECK(solver.getOutput(4, "w") == -401.);

    // warm start keeping / shifting the previous output (acados_solver_interface.cpp:344-376)
    State s3;
    s3.set("x", -1.0);
    solver.initializeWarmstart(s3, false);
    CHECK(solver.getEgoPrediction(5, "y") == 501. && solver.getEgoPrediction(5, "a") == -500.);
    solver.initializeWarmstart(s3, true);
    CHECK(solver.getEgoPrediction(0, "x") == -1.0);
    CHECK(solver.getEgoPrediction(5, "y") == 601.);
    CHECK(solver.getEgoPrediction(solver.N - 1, "y") == 100. * (solver.N - 1) + 1);
    CHECK(solver.getEgoPrediction(solver.N, "v") == 100. * (solver.N - 1) + 3);

    // braking plan (acados_solver_interface.cpp:303-342)
    State s4;
    s4.set("x", 1.0);
    s4.set("y", 2.0);
    s4.set("psi", 0.3);
    s4.set("v", 1.0);
    s4.set("spline", 4.0);
    solver.initializeWithBraking(s4);
    double x = 1.0, v = 1.0, sp = 4.0;
    for (int k = 1; k <= solver.N; k++) {
        x += v * solver.dt * std::cos(0.3);
        sp += v * solver.dt;
        v = std::max(v - 3.0 * solver.dt, 0.);
        CHECK(std::abs(solver.getEgoPrediction(k, "x") - x) < 1e-12);
        CHECK(std::abs(solver.getEgoPrediction(k, "v") - v) < 1e-12);
        CHECK(std::abs(solver.getEgoPrediction(k, "spline") - sp) < 1e-12);
        CHECK(solver.getEgoPrediction(k, "a") == -3.0 && solver.getEgoPrediction(k, "w") == 0.);
    }

    // copy assignment copies the parameters only
    Solver other(1);
    other.setParameter(0, "lag", 42.);
    solver._output.xtraj[0] = -7.;
    other._output.xtraj[0] = 3.;
    solver = other;
    CHECK(solver.getParameter(0, "lag") == 42.);
    CHECK(solver._output.xtraj[0] == -7.);
    CHECK(solver._solver_id == 0);

    CHECK(solver.explainExitFlag(1) == "Success");
    CHECK(solver.explainExitFlag(3) == "Failure (minimum step size reached)");
    solver.reset();
    CHECK(solver.getParameter(0, "lag") == 0.);
}

// ------------------------------------------------------------------ GPU mode
struct Batch {
    int B = 0, N = 0, npar = 0, iters = 0;
    std::vector<double> params, warm, xinit;
};

static Batch read_batch(const char* path) {
    Batch b;
    std::ifstream f(path, std::ios::binary);
    int32_t h[4];
    f.read(reinterpret_cast<char*>(h), sizeof h);
    b.B = h[0];
    b.N = h[1];
    b.npar = h[2];
    b.iters = h[3];
    b.params.resize((size_t)b.B * b.N * b.npar);
    b.warm.resize((size_t)b.B * (b.N + 1) * (SOLVER_NU + SOLVER_NX));
    b.xinit.resize((size_t)b.B * SOLVER_NX);
    f.read(reinterpret_cast<char*>(b.params.data()), b.params.size() * 8);
    f.read(reinterpret_cast<char*>(b.warm.data()), b.warm.size() * 8);
    f.read(reinterpret_cast<char*>(b.xinit.data()), b.xinit.size() * 8);
    if (!f) throw std::runtime_error("short input file");
    return b;
}

static void load(Solver& s, const Batch& b, int i) {
    std::memcpy(s._params.all_parameters, &b.params[(size_t)i * b.N * b.npar], sizeof(double) * b.N * b.npar);
    const size_t nv = SOLVER_NU + SOLVER_NX;
    std::memcpy(s._params.x0, &b.warm[(size_t)i * (b.N + 1) * nv], sizeof(double) * (b.N + 1) * nv);
    std::memcpy(s._params.xinit, &b.xinit[(size_t)i * SOLVER_NX], sizeof(double) * SOLVER_NX);
    s.loadWarmstart();
}

static void dump(std::ofstream& o, const Solver& s, int code) {
    o.write(reinterpret_cast<const char*>(s._output.xtraj), sizeof(s._output.xtraj));
    o.write(reinterpret_cast<const char*>(s._output.utraj), sizeof(s._output.utraj));
    // AcadosInfo as the reference fills it (acados_solver_interface.cpp:151-164, 193-194)
    double extra[9] = {s._info.pobj, (double)code, (double)s._info.sqp_iter, (double)s._info.qp_status,
                       s._info.nlp_res, s._info.kkt_norm_inf, s._info.elapsed_time, s._info.solvetime,
                       s._info.min_time};
    o.write(reinterpret_cast<const char*>(extra), sizeof extra);
}

static int run_solve(const char* in, const char* out) {
    Batch b = read_batch(in);
    if (b.N != SOLVER_N || b.npar != SOLVER_NP) {
        std::cerr << "input dims do not match the compiled solver\n";
        return 2;
    }
    std::ofstream o(out, std::ios::binary);
    // (1) one Solver::solve() per planner, one solver per planner (like LocalPlanner)
    std::vector<std::unique_ptr<Solver>> solvers;
    for (int i = 0; i < b.B; i++) solvers.emplace_back(new Solver(i + 1));
    for (int i = 0; i < b.B; i++) {
        load(*solvers[i], b, i);
        int code = solvers[i]->solve();
        dump(o, *solvers[i], code);
    }
    // (2) the second control step on the same solvers: carried multipliers
    std::vector<std::unique_ptr<Solver>> again;
    for (int i = 0; i < b.B; i++) {
        load(*solvers[i], b, i);
        int code = solvers[i]->solve();
        dump(o, *solvers[i], code);
    }
    // (3) SolverBatch over fresh solvers, two steps
    std::vector<std::unique_ptr<Solver>> fresh;
    std::vector<Solver*> ptrs;
    for (int i = 0; i < b.B; i++) {
        fresh.emplace_back(new Solver(100 + i));
        ptrs.push_back(fresh.back().get());
    }
    SolverBatch batch(*fresh[0], b.B);
    for (int step = 0; step < 2; step++) {
        for (int i = 0; i < b.B; i++) load(*fresh[i], b, i);
        std::vector<int> codes = batch.solve(ptrs);
        for (int i = 0; i < b.B; i++) dump(o, *fresh[i], codes[i]);
    }
    // (4) one-iteration interface on fresh solvers (acados_solver_interface.cpp:121-204)
    for (int i = 0; i < b.B; i++) {
        Solver s(500 + i);
        load(s, b, i);
        s.initializeOneIteration();
        for (int it = 0; it < s._num_iterations; it++) {
            s.solveOneIteration();
            if (s._info.qp_status != 0) break;
        }
        int code = s.completeOneIteration();
        dump(o, s, code);
    }
    return o ? 0 : 3;
}

int main(int argc, char** argv) {
    std::string mode = argc > 1 ? argv[1] : "plumbing";
    try {
        if (mode == "plumbing") {
            test_plumbing();
        } else if (mode == "solve" && argc == 4) {
            int rc = run_solve(argv[2], argv[3]);
            if (rc) return rc;
        } else {
            std::cerr << "usage: test_solver plumbing | solve <in.bin> <out.bin>\n";
            return 2;
        }
    } catch (const std::exception& e) {
        std::cerr << "exception: " << e.what() << "\n";
        return 1;
    }
    if (g_fail) {
        std::cerr << g_fail << " check(s) failed\n";
        return 1;
    }
    std::cout << "OK " << mode << "\n";
    return 0;
}
