// vr_cls_cornell_mesh.hip -- the path kernels of feature class "Cornell box +
// mesh, any material features" (kClassCornellMesh: texture maps and the BRDF
// view tested against the launch's flags): every Cornell-box mesh scene the
// Qt UI can produce other than C2's exact feature set.  Production and
// instrumented (F_COUNT_EXEC) instantiations of vr_kernel.hpp.
#include "vr_kernel.hpp"

namespace vr {

void launch_cls_cornell_mesh(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    if (mode == 1) launch_spec<kClassCornellMesh | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
    else launch_spec<kClassCornellMesh>(p, n_tiles, stack_depth, s, mode == 2);
}

} // namespace vr
