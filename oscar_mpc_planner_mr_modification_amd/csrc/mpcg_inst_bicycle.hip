// Built-in instances: curvature-aware bicycle with decomp halfspaces (C3) and its test shape.
#include "mpcg_instance.h"

MPCG_DEFINE_INSTANCE(30, 0, 0, 12, 6, 1)   // C3
MPCG_DEFINE_INSTANCE(10, 0, 0, 4, 6, 1)
