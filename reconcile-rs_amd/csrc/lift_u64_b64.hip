// Lift kernels for the u64_b64 record shape (see schemas.def, lift_inst_body.inc).
#define RH_NAME u64_b64
#define RH_KK 2
#define RH_KL 8
#define RH_VK 3
#define RH_VL 64
#include "lift_inst_body.inc"
