// vr_spec_c4.hip -- the path kernels of scene specialisation C4 (HDRI + MERL BRDF sphere):
// production and instrumented (F_COUNT_EXEC) instantiations of vr_kernel.hpp.
// One translation unit per specialisation, so the build compiles them in parallel.
#define VR_DK_HOISTED 1      // sphere-only kernels: the hoistable constant form (vr_math.hpp dk)
#include "vr_kernel.hpp"

namespace vr {

void launch_spec_c4(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    if (mode == 1) launch_spec<kFeatHdriBrdfSphere | F_EXACT | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
    else launch_spec<kFeatHdriBrdfSphere | F_EXACT>(p, n_tiles, stack_depth, s, mode == 2);
}

} // namespace vr
