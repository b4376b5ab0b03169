// Lift kernels for the u64_unit record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME u64_unit
#define RH_KK 2
#define RH_KL 8
#define RH_VK 0
#define RH_VL 0
#include "lift_inst_body.inc"
