// state.h — MPCPlanner::State of the drop-in solver surface.
// Same interface and semantics as the reference's State
// (mpc_planner_solver/include/mpc_planner_solver/state.h:10-31,
// src/state.cpp:7-74): the robot state vector in model_map.yaml order,
// accessed by variable name.
#pragma once

#include <string>
#include <vector>

#include "mpc_planner_solver/mpcg_config.h"

namespace MPCPlanner {

struct State {
    State();

    void initialize();

    double get(std::string&& var_name) const;
    Vec2 getPos() const;

    void set(std::string&& var_name, double value);
    void print() const;

    // finite and not the all-zero default (state.cpp:45-74)
    bool validData() const;

private:
    std::vector<double> _state;
    YamlNode _config, _model_map;
    int _nu = 0;
    int index(const std::string& var_name) const;
};

}  // namespace MPCPlanner
