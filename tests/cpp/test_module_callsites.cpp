// test_module_callsites.cpp — boundary test: the call shapes the reference's
// controller modules use on `MPCPlanner::Solver` compile against the drop-in
// headers (include/mpc_planner_solver/ + the generated mpc_planner_parameters.h)
// and land in the slots the generated parameter map names.
//
// The reference's module translation units themselves cannot be compiled here
// (they need ROS, ros_tools, Eigen and yaml-cpp, none of which is in the image),
// so each block below restates one module's setParameters / glue with the same
// calls and argument kinds as the cited reference lines:
//   MPCBase::setParameters              mpc_base.cpp:26-35
//   Contouring::setParameters / setSplineParameters   contouring.cpp:70-125
//   LinearizedConstraints::setParameters             linearized_constraints.cpp:150-185
//   EllipsoidConstraints::setParameters              ellipsoid_constraints.cpp:36-86
//   GuidanceConstraints glue (warm start from a guidance trajectory, solve
//   bookkeeping, best-solver copy)      guidance_constraints.cpp:274, 336-375, 520-522, 546-570, 623-633
// CPU only: no solve is issued (solver directory from MPCG_SOLVER_DIR / MPCG_SETTINGS;
// driven by tests/test_cpp_solver.py::test_module_call_sites_compile_and_land).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "mpc_planner_solver/mpc_planner_parameters.h"
#include "mpc_planner_solver/solver_interface.h"

using namespace MPCPlanner;

static int g_fail = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                            \
        }                                                                        \
    } while (0)

static bool near(double a, double b) { return std::fabs(a - b) <= 1e-15 * (1.0 + std::fabs(b)); }

// one obstacle prediction step (the fields EllipsoidConstraints reads)
struct PredictionStep {
    Vec2 position;
    double angle, major_radius, minor_radius;
};

int main() {
    auto _solver = std::make_shared<Solver>(0);
    const int n_obs = 8, n_discs = 1, n_segments = 5;

    for (int k = 0; k < _solver->N; k++) {
        // MPCBase: weights by name (mpc_base.cpp:33)
        for (std::string weight : {"acceleration", "angular_velocity"}) _solver->setParameter(k, weight, 0.1 + k);

        // Contouring: weights and the spline window (contouring.cpp:80-89, 113-124)
        setSolverParameterContour(k, _solver->_params, 0.05);
        setSolverParameterLag(k, _solver->_params, 0.75);
        setSolverParameterTerminalAngle(k, _solver->_params, 1.0);
        setSolverParameterTerminalContouring(k, _solver->_params, 10.0);
        setSolverParameterVelocity(k, _solver->_params, 0.55);
        setSolverParameterReferenceVelocity(k, _solver->_params, 1.5);
        for (int i = 0; i < n_segments; i++) {
            setSolverParameterSplineXA(k, _solver->_params, 1.0 * i, i);
            setSolverParameterSplineXB(k, _solver->_params, 2.0 * i, i);
            setSolverParameterSplineXC(k, _solver->_params, 3.0 * i, i);
            setSolverParameterSplineXD(k, _solver->_params, 4.0 * i, i);
            setSolverParameterSplineYA(k, _solver->_params, -1.0 * i, i);
            setSolverParameterSplineYB(k, _solver->_params, -2.0 * i, i);
            setSolverParameterSplineYC(k, _solver->_params, -3.0 * i, i);
            setSolverParameterSplineYD(k, _solver->_params, -4.0 * i, i);
            setSolverParameterSplineStart(k, _solver->_params, 10.0 * i, i);
        }

        // LinearizedConstraints: dummies at k = 0, one halfspace per obstacle and disc after
        // (linearized_constraints.cpp:156-183)
        int constraint_counter = 0;
        if (k == 0) {
            for (int i = 0; i < n_obs; i++, constraint_counter++) {
                setSolverParameterLinConstraintA1(0, _solver->_params, 1.0, constraint_counter);
                setSolverParameterLinConstraintA2(0, _solver->_params, 0.0, constraint_counter);
                setSolverParameterLinConstraintB(0, _solver->_params, 100.0, constraint_counter);
            }
        } else {
            for (int d = 0; d < n_discs; d++) {
                setSolverParameterEgoDiscOffset(k, _solver->_params, 0.0, d);
                for (int i = 0; i < n_obs; i++, constraint_counter++) {
                    setSolverParameterLinConstraintA1(k, _solver->_params, std::cos(0.1 * i), constraint_counter);
                    setSolverParameterLinConstraintA2(k, _solver->_params, std::sin(0.1 * i), constraint_counter);
                    setSolverParameterLinConstraintB(k, _solver->_params, 3.0 + k, constraint_counter);
                }
            }
        }

        // EllipsoidConstraints (ellipsoid_constraints.cpp:38-84): disc radius/offset, far dummies
        // at k = 0, the k-1 prediction step of every obstacle after
        setSolverParameterEgoDiscRadius(k, _solver->_params, 0.325);
        for (int d = 0; d < n_discs; d++) setSolverParameterEgoDiscOffset(k, _solver->_params, 0.0, d);
        for (int i = 0; i < n_obs; i++) {
            if (k == 0) {
                setSolverParameterEllipsoidObstX(0, _solver->_params, 50., i);
                setSolverParameterEllipsoidObstY(0, _solver->_params, 50., i);
                setSolverParameterEllipsoidObstPsi(0, _solver->_params, 0., i);
                setSolverParameterEllipsoidObstR(0, _solver->_params, 0.1, i);
                setSolverParameterEllipsoidObstMajor(0, _solver->_params, 0., i);
                setSolverParameterEllipsoidObstMinor(0, _solver->_params, 0., i);
                setSolverParameterEllipsoidObstChi(0, _solver->_params, 1., i);
                continue;
            }
            const PredictionStep step{Vec2(2.0 * i + 0.1 * (k - 1), -1.0 * i), 0.01 * i, 0.0, 0.0};
            setSolverParameterEllipsoidObstX(k, _solver->_params, step.position(0), i);
            setSolverParameterEllipsoidObstY(k, _solver->_params, step.position(1), i);
            setSolverParameterEllipsoidObstPsi(k, _solver->_params, step.angle, i);
            setSolverParameterEllipsoidObstR(k, _solver->_params, 0.4, i);
            setSolverParameterEllipsoidObstMajor(k, _solver->_params, step.major_radius, i);
            setSolverParameterEllipsoidObstMinor(k, _solver->_params, step.minor_radius, i);
            setSolverParameterEllipsoidObstChi(k, _solver->_params, 1., i);
        }

        // consistency module parameters (set by the guidance module per planner)
        setSolverParameterConsistencyWeight(k, _solver->_params, 0.0);
        setSolverParameterPrevTrajX(k, _solver->_params, 0.5 * k);
        setSolverParameterPrevTrajY(k, _solver->_params, -0.5 * k);
    }

    // the same slots by name (the generated map), as the reference's setParameter resolves them
    CHECK(near(_solver->getParameter(3, "acceleration"), 3.1));
    CHECK(near(_solver->getParameter(2, "contour"), 0.05));
    CHECK(near(_solver->getParameter(7, "spline_y2_a"), -2.0));
    CHECK(near(_solver->getParameter(7, "spline4_start"), 40.0));
    CHECK(near(_solver->getParameter(0, "lin_constraint_5_b"), 100.0));
    CHECK(near(_solver->getParameter(4, "lin_constraint_5_b"), 7.0));
    CHECK(near(_solver->getParameter(4, "lin_constraint_3_a2"), std::sin(0.3)));
    CHECK(near(_solver->getParameter(0, "ellipsoid_obst_6_x"), 50.0));
    CHECK(near(_solver->getParameter(5, "ellipsoid_obst_6_x"), 12.4));
    CHECK(near(_solver->getParameter(5, "ellipsoid_obst_6_r"), 0.4));
    CHECK(near(_solver->getParameter(9, "prev_traj_y"), -4.5));
    CHECK(near(_solver->_params.all_parameters[5 * _solver->npar + 82], 2.0 * 0 + 0.1 * 4));  // obst 0 x at k 5
    CHECK(_solver->hasParameter("ellipsoid_obst_7_chi"));
    CHECK(!_solver->hasParameter("ellipsoid_obst_8_chi"));

    // GuidanceConstraints glue: per-planner copies of the main solver (*solver = *_solver,
    // guidance_constraints.cpp:331), a warm start from a guidance trajectory (:557-568), the
    // timeout field (:274, :363), the solve bookkeeping fields (:369-375) and the best-solver
    // copy back into the main solver (:520-522)
    std::vector<std::unique_ptr<Solver>> local;
    for (int p = 0; p < 3; p++) {
        local.emplace_back(new Solver(p + 1));
        *local.back() = *_solver;
        Solver* solver = local.back().get();
        solver->_params.solver_timeout = 0.02;
        for (int k = 1; k < solver->N; k++) {
            solver->setEgoPrediction(k, "x", 0.3 * k);
            solver->setEgoPrediction(k, "y", 0.1 * p);
            solver->setEgoPrediction(k, "psi", std::atan2(0.0, 1.0));
            solver->setEgoPrediction(k, "v", 1.5);
        }
        CHECK(near(solver->getParameter(5, "ellipsoid_obst_6_x"), 12.4));
        CHECK(near(solver->getEgoPrediction(4, "x"), 1.2));
        CHECK(near(solver->getEgoPredictionPosition(4)(1), 0.1 * p));
        CHECK(solver->_solver_id == p + 1);
    }
    Solver* best_solver = local[2].get();
    double objective = best_solver->_info.pobj;
    (void)objective;
    _solver->_output = best_solver->_output;
    _solver->_info = best_solver->_info;
    _solver->_params = best_solver->_params;
    CHECK(near(_solver->getEgoPrediction(4, "y"), 0.2));
    CHECK(!_solver->explainExitFlag(1).empty());

    if (g_fail) {
        std::fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK module call sites\n");
    return 0;
}
