// vr_cls_hdri_mesh.hip -- the path kernels of feature class "HDRI environment
// + mesh, any material features" (kClassHdriMesh): every HDRI mesh scene the
// Qt UI can produce other than C3's and C5's exact feature sets (e.g. a mesh
// with only a diffuse map, or a BRDF-shaded mesh).  Production and
// instrumented (F_COUNT_EXEC) instantiations of vr_kernel.hpp.
#include "vr_kernel.hpp"

namespace vr {

void launch_cls_hdri_mesh(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    if (mode == 1) launch_spec<kClassHdriMesh | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
    else launch_spec<kClassHdriMesh>(p, n_tiles, stack_depth, s, mode == 2);
}

} // namespace vr
