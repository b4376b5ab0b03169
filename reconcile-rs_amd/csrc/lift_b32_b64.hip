// Lift kernels for the b32_b64 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME b32_b64
#define RH_KK 3
#define RH_KL 32
#define RH_VK 3
#define RH_VL 64
#include "lift_inst_body.inc"
