// Built-in instances: SH-MPC on the slack model (C5) and its N = 10 test shape.
#include "mpcg_instance.h"

MPCG_DEFINE_INSTANCE(20, 0, 0, 24, 6, 0)   // C5
MPCG_DEFINE_INSTANCE(10, 0, 0, 4, 6, 0)
