// vr_cls_sphere.hip -- the sphere-scene kernels of the feature classes
// "Cornell box, spheres only" and "HDRI environment, spheres only" (the
// example sphere, its texture maps and the BRDF view tested against the
// launch's flags): every sphere scene other than C1's and C4's exact feature
// sets.  Production and instrumented (F_COUNT_EXEC) instantiations.
#define VR_DK_HOISTED 1      // sphere-only kernels: the hoistable constant form (vr_math.hpp dk)
#include "vr_kernel.hpp"

namespace vr {

void launch_cls_sphere(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    const bool cornell = (p.flags & F_CORNELL) != 0u;
    if (mode == 1) {
        if (cornell) launch_spec<kClassCornellSphere | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
        else launch_spec<kClassHdriSphere | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
    } else {
        if (cornell) launch_spec<kClassCornellSphere>(p, n_tiles, stack_depth, s);
        else launch_spec<kClassHdriSphere>(p, n_tiles, stack_depth, s);
    }
}

} // namespace vr
