// vr_spec_generic.hip -- the path kernels of scene specialisation every other flag combination (generic kernel):
// production and instrumented (F_COUNT_EXEC) instantiations of vr_kernel.hpp.
// One translation unit per specialisation, so the build compiles them in parallel.
#include "vr_kernel.hpp"

namespace vr {

void launch_spec_generic(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    if (mode == 1) launch_spec<kFeatAll | F_COUNT_EXEC>(p, n_tiles, stack_depth, s);
    else launch_spec<kFeatAll>(p, n_tiles, stack_depth, s, mode == 2);
}

void launch_spec_deep(const RenderParams& p, uint32_t n_tiles, hipStream_t s, bool exec)
{
    if (exec) launch_wave<64, kFeatAll | F_COUNT_EXEC>(p, n_tiles, s);
    else launch_wave<64, kFeatAll>(p, n_tiles, s);
}

void launch_counting(const RenderParams& p, uint32_t blocks, int stack_depth, hipStream_t s)
{
    if (stack_depth <= 32) hipLaunchKernelGGL((render_kernel<32, true, kFeatAll>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
    else hipLaunchKernelGGL((render_kernel<64, true, kFeatAll>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
}

} // namespace vr
