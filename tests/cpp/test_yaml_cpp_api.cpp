// The drop-in's YAML members through yaml-cpp's API (tests/test_cpp_yaml_api.py): with
// <yaml-cpp/yaml.h> on the include path, MPCPlanner::YamlNode is YAML::Node, so reference code that
// walks Solver::_parameter_map / _model_map with YAML::const_iterator
// (acados_solver_interface.cpp:236-246 style) compiles unchanged.  Built against the yaml-cpp API
// stand-in of tests/cpp/yaml_cpp_api (yaml-cpp is not installed here).
#include <cstdio>
#include <string>

#include "mpc_planner_solver/mpcg_solver_interface.h"

static_assert(MPCG_YAML_CPP == 1, "the yaml-cpp branch of mpcg_yaml.h");

// what a reference module does with a Solver's public members (compiled, not called: a Solver
// needs the GPU)
int count_states(const MPCPlanner::Solver& s) {
    int n = 0;
    for (YAML::const_iterator it = s._model_map.begin(); it != s._model_map.end(); ++it)
        if (it->second[0].as<std::string>() == "x") ++n;
    return n + (s._parameter_map["contour"].IsDefined() ? 0 : 1000);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const YAML::Node pmap = MPCPlanner::load_yaml_file(argv[1]);
    const YAML::Node mmap = MPCPlanner::load_yaml_file(argv[2]);
    int np = 0, nx = 0;
    for (YAML::const_iterator it = pmap.begin(); it != pmap.end(); ++it) np += it->second.as<int>() >= 0;
    for (YAML::const_iterator it = mmap.begin(); it != mmap.end(); ++it) nx += it->second[0].as<std::string>() == "x";
    std::printf("%d %d %d\n", np, nx, (int)pmap["contour"].as<int>());
    return 0;
}
