// Lift kernels for the b16_unit record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME b16_unit
#define RH_KK 3
#define RH_KL 16
#define RH_VK 0
#define RH_VL 0
#include "lift_inst_body.inc"
