// Lift kernels for the b16_b1024 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME b16_b1024
#define RH_KK 3
#define RH_KL 16
#define RH_VK 3
#define RH_VL 1024
#include "lift_inst_body.inc"
