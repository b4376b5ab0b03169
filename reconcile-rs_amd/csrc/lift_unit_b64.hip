// Lift kernels for the unit_b64 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME unit_b64
#define RH_KK 0
#define RH_KL 0
#define RH_VK 3
#define RH_VL 64
#include "lift_inst_body.inc"
