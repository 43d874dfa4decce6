// solver_interface.h — the include the planner and its modules use for the
// solver (reference: mpc_planner_solver/include/mpc_planner_solver/solver_interface.h).
// There is one backend here: the MI355X batched SQP (mpcg_solver_interface.h).
#pragma once
#include "mpc_planner_solver/mpcg_solver_interface.h"
