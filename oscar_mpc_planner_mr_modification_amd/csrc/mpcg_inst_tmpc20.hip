// Built-in instances: T-MPC++ unicycle, N = 20 (C1, C2) and the N = 10 test shape.
#include "mpcg_instance.h"

MPCG_DEFINE_INSTANCE(20, 4, 4, 0, 5, 0)    // C1
MPCG_DEFINE_INSTANCE(20, 8, 8, 0, 5, 0)    // C2 (north star)
MPCG_DEFINE_INSTANCE(10, 2, 2, 0, 5, 0)    // small test shape
