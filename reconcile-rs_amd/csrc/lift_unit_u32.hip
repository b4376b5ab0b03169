// Lift kernels for the unit_u32 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME unit_u32
#define RH_KK 0
#define RH_KL 0
#define RH_VK 1
#define RH_VL 4
#include "lift_inst_body.inc"
