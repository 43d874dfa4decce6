// mpcg_config.h — where the drop-in solver finds its configuration.
//
// The reference's Solver reads solver_settings.yaml / parameter_map.yaml /
// model_map.yaml from SYSTEM_CONFIG_PATH(__FILE__, ...) and the planner
// settings through the global CONFIG (acados_solver_interface.cpp:9-31,
// 303-342).  Here both locations are explicit: a solver directory (the
// generator's output, see oscar_mpc_planner_mr_modification_amd/codegen.py)
// and the planner's settings.yaml.  Defaults come from the environment
// variables MPCG_SOLVER_DIR and MPCG_SETTINGS.
#pragma once

#include <string>

#include "mpc_planner_solver/mpcg_yaml.h"

namespace MPCPlanner {

#if __has_include(<Eigen/Dense>)
}  // namespace MPCPlanner
#include <Eigen/Dense>
namespace MPCPlanner {
using Vec2 = Eigen::Vector2d;
#else
// 2-vector with Eigen's element access, for builds without Eigen.
struct Vec2 {
    double v[2];
    Vec2(double x = 0.0, double y = 0.0) : v{x, y} {}
    double operator()(int i) const { return v[i]; }
    double& operator()(int i) { return v[i]; }
};
#endif

struct SolverConfig {
    static void setSolverDirectory(const std::string& dir);
    static void setSettingsFile(const std::string& settings_yaml);
    static std::string solverDirectory();
    // <solver dir>/<name>.yaml
    static std::string solverFile(const std::string& name);
    // the planner settings (the reference's CONFIG), loaded once
    static const YamlNode& settings();
    static void reload();
};

}  // namespace MPCPlanner
