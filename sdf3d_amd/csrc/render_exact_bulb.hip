// Exact-precision build of the Mandelbulb scene's render kernels (its own unit
// so that it gets its own scheduler, sdf3d_amd/build.py).
#define SDF_EXACT 1
#define SDF_TU_BULB 1
#include "render_kernel.inc"
