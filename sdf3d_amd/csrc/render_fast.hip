// Fast-precision build of the render kernel (compiled -ffp-contract=fast).
#define SDF_EXACT 0
#include "render_kernel.inc"
