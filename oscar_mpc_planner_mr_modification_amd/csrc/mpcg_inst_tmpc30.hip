// Built-in instances: T-MPC++ unicycle, N = 30 -- C4 and the reference's shipped robot
// configurations (configuration_tmpc_consistency_cost):
//   mpc_planner_jackalsimulator/config/settings.yaml:3,37 (N 30, max_obstacles 4)
//   mpc_planner_jackal/config/settings.yaml:3,38 and mpc_planner_dingo (N 30, max_obstacles 5)
#include "mpcg_instance.h"

MPCG_DEFINE_INSTANCE(30, 12, 12, 0, 5, 0)  // C4
MPCG_DEFINE_INSTANCE(30, 4, 4, 0, 5, 0)    // jackalsimulator as shipped
MPCG_DEFINE_INSTANCE(30, 5, 5, 0, 5, 0)    // jackal / dingo as shipped
