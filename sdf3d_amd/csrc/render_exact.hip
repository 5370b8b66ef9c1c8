// Exact-precision build of the render kernel (compiled -ffp-contract=off).
#define SDF_EXACT 1
#include "render_kernel.inc"
