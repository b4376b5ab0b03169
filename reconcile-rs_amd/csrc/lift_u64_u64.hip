// Lift kernels for the u64_u64 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME u64_u64
#define RH_KK 2
#define RH_KL 8
#define RH_VK 2
#define RH_VL 8
#include "lift_inst_body.inc"
