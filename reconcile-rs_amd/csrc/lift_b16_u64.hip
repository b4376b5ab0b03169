// Lift kernels for the b16_u64 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME b16_u64
#define RH_KK 3
#define RH_KL 16
#define RH_VK 2
#define RH_VL 8
#include "lift_inst_body.inc"
