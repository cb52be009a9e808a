// vr_kernel.hip -- finish, order and helper kernels of the gfx950 path
// tracer, and the launch dispatch over the scene specialisations (the path
// kernels themselves: vr_kernel.hpp, instantiated in vr_spec_*.hip).
#include "vr_kernel.hpp"

namespace vr {

// Split launches: sums each pixel's path results in path order (the same
// float4 operations, in the same order, as the unsplit kernel), then writes
// the accumulation, colour and depth.
// Path results loaded per batch ahead of the finish passes' in-order adds:
// with one load in flight per thread, a shard's session finish (a few blocks
// per CU) was latency-bound -- 8-rank rehearsal C2 0.917 -> 0.927, C3 0.686
// -> 0.715 of linear (profiles/r06zl); whole frames unchanged
#ifndef VR_SVC_FINISH_BATCH
#define VR_SVC_FINISH_BATCH 8
#endif
// The completion flag of a synchronous one-frame call (RenderParams::
// sync_flag): every wave waits for its stores to complete, the block's
// arrival is counted, and the last block to arrive stores the call's number
// to host-coherent memory at system scope -- the host sees the frame done
// without waiting for the stream's completion signal (vrhip_api.cpp one_sync).
// The results are then complete in the L2s; the end of the kernel writes them
// back before any later work on the stream starts, and the library arms the
// flag only on a stream no other party queues work on (vrhip_api.cpp).  (An
// agent-scope release per wave -- an L2 write-back each -- cost 360 us per
// 1280x720 finish pass, r06zr.)
__device__ __forceinline__ void finish_arrive(const RenderParams& p)
{
    __builtin_amdgcn_s_waitcnt(0);      // this wave's stores have reached the L2
    __syncthreads();
    // two-level count (blocks by blockIdx mod kSyncGroups, then the groups):
    // the arrivals spread over kSyncGroups words instead of serialising on one
    // (one word: +25 us per 1280x720 pass, r06zr)
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x, g = blockIdx.x & (kSyncGroups - 1u);
        const uint32_t in_group = (G - g + kSyncGroups - 1u) / kSyncGroups, groups = G < kSyncGroups ? G : kSyncGroups;
        uint32_t* sub = p.sync_ctr + 64u * g;                     // one word per 256 B
        uint32_t* top = p.sync_ctr + 64u * kSyncGroups;
        if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1u) {
            __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1u) {
                __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(p.sync_flag, p.sync_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

__device__ __forceinline__ void finish_body(const RenderParams& p, const float* T);
#ifndef VR_FINISH_LDS_TONE
#define VR_FINISH_LDS_TONE 1
#endif
__global__ void __launch_bounds__(kBlockThreads) finish_kernel(const RenderParams p)
{
#if VR_FINISH_LDS_TONE
    // the tonemap's 256 thresholds in LDS: the dependent table reads of each
    // colour byte (tone_byte) then wait on LDS instead of the L1
    static_assert(kBlockThreads == 256, "one threshold per thread");
    __shared__ float T[256];
    T[threadIdx.x] = p.tone_t ? p.tone_t[threadIdx.x] : 0.f;
    __syncthreads();
    finish_body(p, p.tone_t ? T : nullptr);
#else
    finish_body(p, p.tone_t);
#endif
    if (p.sync_flag) finish_arrive(p);
}

__device__ __forceinline__ void finish_body(const RenderParams& p, const float* T)
{
    const uint32_t tile = blockIdx.x, tid = threadIdx.x;
    // the path kernel's queue heads, for the next launch on this scratch
    if (tile == 0 && tid <= VR_MAX_QUEUES && p.chunk_ctr) p.chunk_ctr[tid * kQueueStride] = 0u;
    if (tile == 0 && tid == VR_MAX_QUEUES && p.chunk_ctr) {
        p.chunk_ctr[tid * kQueueStride + 1u] = 0u;      // drained-queue mask
        *sparse_count_of(p.chunk_ctr) = 0u;            // an F_SPARSE launch's pixel list
    }
    const int wave = (int)tid >> 6, lane = (int)tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;      // tiles dealt round-robin to ranks
    const uint32_t tile_y = tile_row(gtile, p.tiles_x);
    const uint32_t tile_x = tile_col(gtile, p.tiles_x, p.nranks);
    const uint32_t x = tile_x * 16u + (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t y = tile_y * 16u + (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    if (x >= p.wr || y >= p.hr) return;
    const uint32_t ind = x + y * p.W;
    vr4 io = p.first_frame != 1u ? p.accum[ind] : mk4(0.f, 0.f, 0.f, 0.f);
    const uint32_t n_paths = 2u * p.n_frames;
    const uint32_t slot = tile * kBlockThreads + tid;
    const vr3* src = p.paths + slot;
    const float depth = p.path_w[slot];
    const bool cornell = (p.flags & F_CORNELL) != 0u;
    float last_w = 0.f;
    if (depth == kSharedMissW) {
        // a split sphere launch's escaped pixel: one result for all its paths
        // (their depth term is 1, the miss at bounce 0), added path by path
        const vr3 r = src[0];
        const vr4 h = mul4s(mk4(r.x, r.y, r.z, 1.f), 1.f / 2.f);
        for (uint32_t q = 0; q < n_paths; ++q) io = add4(io, h);
        last_w = 1.f;
    } else {
        // loads batched ahead of the in-order adds, as in svc_finish_kernel
        for (uint32_t q0 = 0; q0 < n_paths; q0 += VR_SVC_FINISH_BATCH) {
            vr3 r[VR_SVC_FINISH_BATCH];
#pragma unroll
            for (int j = 0; j < VR_SVC_FINISH_BATCH; ++j)
                if (q0 + j < n_paths) r[j] = src[(size_t)(q0 + j) * p.path_stride];
#pragma unroll
            for (int j = 0; j < VR_SVC_FINISH_BATCH; ++j) {
                if (q0 + j < n_paths) {
                    last_w = (cornell && escaped(r[j].x)) ? 0.f : depth;
                    io = add4(io, mul4s(mk4(r[j].x, r[j].y, r[j].z, last_w), 1.f / 2.f));
                }
            }
        }
    }
    const unsigned char db = f2u8((1.f - last_w) * 255);
    u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
    p.depth[ind] = dv;
    p.rgba[ind] = tonemap(io, p.first_frame + p.n_frames - 1u, T);
    p.accum[ind] = io;
    if (p.path_cost) {
        // the sub-tile's cost for the next launch's order: its paths' costs,
        // summed per pixel, then over the wave (one wave = one 8x8 sub-tile)
        uint32_t c = 0;
        for (uint32_t q = 0; q < n_paths; ++q) c += p.path_cost[(size_t)q * p.path_stride + slot];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
        if (lane == 0) p.sub_cost[tile * 4u + (uint32_t)wave] = c;
    }
}

// Longest-first order of a launch's sub-tiles for the next launch on the
// same scratch (RenderParams::sub_order): block x sorts the sub-tiles XCD x's
// queues serve (bands of VR_XCD_BANDS, dealt round-robin to the 8 XCDs) by
// the cost this launch measured (sub_cost, written by finish_kernel: node
// visits of all their paths), most expensive first, by a counting sort over
// half-octave cost classes.  Scheduling only: any permutation renders the
// same image (finish_kernel sums each pixel's paths in path order).
constexpr int kCostClasses = 64;
__device__ __forceinline__ uint32_t cost_class(uint32_t c)
{
    if (c < 2u) return c;
    const uint32_t msb = 31u - (uint32_t)__builtin_clz(c);
    return 2u * msb + ((c >> (msb - 1u)) & 1u);          // 0..63
}
// 256-thread blocks: a 1,024-thread block needs a whole CU's wave slots, which
// the next launch's path kernels hold; behind overlapped launches one waited
// 341 us for them (and every later finish pass behind it on the stream)
__global__ void __launch_bounds__(256) order_kernel(const uint32_t* __restrict__ cost, uint32_t* __restrict__ order,
                                                      uint32_t n_sub, uint32_t cap)
{
    __shared__ uint32_t hist[kCostClasses];
    const uint32_t x = blockIdx.x, tid = threadIdx.x;
    constexpr uint32_t B = (uint32_t)VR_XCD_BANDS;
    auto sub_of = [&](uint32_t k) { return ((k / B) * 8u + x) * B + (k % B); };
    // this XCD's sub-tiles: k < n_x  <=>  sub_of(k) < n_sub
    const uint32_t full = n_sub / (8u * B), rem = n_sub - full * 8u * B;
    const uint32_t n_x = full * B + (rem > x * B ? (rem - x * B < B ? rem - x * B : B) : 0u);
    if (tid < (uint32_t)kCostClasses) hist[tid] = 0u;
    __syncthreads();
    for (uint32_t k = tid; k < n_x; k += blockDim.x) atomicAdd(&hist[cost_class(cost[sub_of(k)])], 1u);
    __syncthreads();
    if (tid == 0) {                                      // start of each class, most expensive first
        uint32_t acc = 0;
        for (int c = kCostClasses - 1; c >= 0; --c) { const uint32_t h = hist[c]; hist[c] = acc; acc += h; }
    }
    __syncthreads();
    for (uint32_t k = tid; k < n_x; k += blockDim.x) {
        const uint32_t sb = sub_of(k);
        const uint32_t pos = atomicAdd(&hist[cost_class(cost[sb])], 1u);
        order[x * cap + pos] = sb;
    }
}

int launch_order(uint32_t* cost, uint32_t* order, uint32_t n_sub, uint32_t cap, void* stream)
{
    if (n_sub == 0) return 0;
    hipLaunchKernelGGL(order_kernel, dim3(8), dim3(256), 0, (hipStream_t)stream, cost, order, n_sub, cap);
    return (int)hipGetLastError();
}

__global__ void half_to_float_kernel(const uint16_t* __restrict__ src, vr4* __restrict__ dst, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint16_t* s = src + 4 * i;
    dst[i] = mk4(__half2float(__ushort_as_half(s[0])), __half2float(__ushort_as_half(s[1])),
                 __half2float(__ushort_as_half(s[2])), __half2float(__ushort_as_half(s[3])));
}

// Copies this rank's tiles between the full image and a packed buffer: owned
// tile j (global tile rank + j*nranks) occupies packed pixels [256j, 256j+256)
// in row-major order within the tile.
__global__ void pack_tiles_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t wpp,
                                  uint32_t W, uint32_t tiles_x, uint32_t rank, uint32_t nranks, int unpack)
{
    const uint32_t j = blockIdx.x;
    const uint32_t gt = rank + j * nranks;
    const uint32_t ty = tile_row(gt, tiles_x), tx = tile_col(gt, tiles_x, nranks);
    for (uint32_t w = threadIdx.x; w < 256u * wpp; w += blockDim.x) {
        const uint32_t px = w / wpp, word = w - px * wpp;
        const size_t full = ((size_t)(ty * 16u + px / 16u) * W + tx * 16u + px % 16u) * wpp + word;
        const size_t packed = ((size_t)j * 256u + px) * wpp + word;
        if (unpack) dst[full] = src[packed];
        else dst[packed] = src[full];
    }
}

// The gathering rank's scatter of several ranks' packed buffers in ONE
// launch (rank r0 + blockIdx.y's buffer at src + blockIdx.y * stride words):
// the per-rank launches of pack_tiles_kernel cost ~2.5 us each, 18-21 us per
// 8-rank gather, for ~3 us of memory work.
__global__ void unpack_ranks_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t wpp,
                                    uint32_t W, uint32_t tiles_x, uint32_t total_tiles, uint32_t r0, uint32_t nranks,
                                    size_t stride_words)
{
    const uint32_t j = blockIdx.x, rank = r0 + blockIdx.y;
    if (rank >= nranks || rank >= total_tiles) return;
    const uint32_t n_owned = (total_tiles - rank + nranks - 1u) / nranks;
    if (j >= n_owned) return;
    const uint32_t* s = src + (size_t)blockIdx.y * stride_words;
    const uint32_t gt = rank + j * nranks;
    const uint32_t ty = tile_row(gt, tiles_x), tx = tile_col(gt, tiles_x, nranks);
    for (uint32_t w = threadIdx.x; w < 256u * wpp; w += blockDim.x) {
        const uint32_t px = w / wpp, word = w - px * wpp;
        dst[((size_t)(ty * 16u + px / 16u) * W + tx * 16u + px % 16u) * wpp + word] = s[((size_t)j * 256u + px) * wpp + word];
    }
}

__global__ void selftest_math_kernel(int fn, const float* a, const float* b, float* out, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s, c, r = 0.f;
    switch (fn) {
    case 0: sincos_p(a[i], &s, &c); r = s; break;
    case 1: sincos_p(a[i], &s, &c); r = c; break;
    case 2: r = acos_p(a[i]); break;
    case 3: r = atan2_p(a[i], b[i]); break;
    case 4: r = pow_p(a[i], b[i]); break;
    case 5: r = __builtin_fminf(a[i], b[i]); break;
    case 6: r = __builtin_fmaxf(a[i], b[i]); break;
    case 7: r = __int_as_float(f2i(a[i])); break;
    default: r = 0.f;
    }
    out[i] = r;
}

// Flags outside the five exact specialisations -> their feature class
// (vr_cls_*.hip), or the generic kernel (strict traversal).
// VR_FEATURE_CLASSES=0 builds route them all to the generic kernel (A/B builds).
#ifndef VR_FEATURE_CLASSES
#define VR_FEATURE_CLASSES 1
#endif
static void launch_class(const RenderParams& p, uint32_t need, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode)
{
    const uint32_t cls = VR_FEATURE_CLASSES ? feature_class(need) : 0u;
    if (cls == kClassCornellMesh) launch_cls_cornell_mesh(p, n_tiles, stack_depth, s, mode);
    else if (cls == kClassHdriMesh) launch_cls_hdri_mesh(p, n_tiles, stack_depth, s, mode);
    else if (cls == kClassCornellSphere || cls == kClassHdriSphere) launch_cls_sphere(p, n_tiles, stack_depth, s, mode);
    else launch_spec_generic(p, n_tiles, stack_depth, s, mode);
}

// Scene flags -> specialisation (one translation unit each, vr_spec_*.hip).
static void launch_scene(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, bool exec)
{
    const uint32_t need = p.flags & kFeatAll;
    const int mode = exec ? 1 : 0;
    if (need == kFeatCornellMesh) launch_spec_c2(p, n_tiles, stack_depth, s, mode);
    else if (need == kFeatCornellSphere) launch_spec_c1(p, n_tiles, stack_depth, s, mode);
    else if (need == kFeatHdriMesh) launch_spec_c5(p, n_tiles, stack_depth, s, mode);
    else if (need == kFeatHdriMeshTex) launch_spec_c3(p, n_tiles, stack_depth, s, mode);
    else if (need == kFeatHdriBrdfSphere) launch_spec_c4(p, n_tiles, stack_depth, s, mode);
    else launch_class(p, need, n_tiles, stack_depth, s, mode);
}

int launch_render(const RenderParams& p, uint32_t n_tiles, int stack_depth, int count, void* stream)
{
    if (n_tiles == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t blocks = n_tiles * p.split;   // split == 1 for the counting variant
    if (count == 1) launch_counting(p, blocks, stack_depth, s);   // the reference algorithm's event counts
    else if (stack_depth > 32) launch_spec_deep(p, n_tiles, s, count != 0);
    else launch_scene(p, n_tiles, stack_depth, s, count == 2);
    return (int)hipGetLastError();
}

// The render service's session finish pass: per pixel, every launch's path
// results summed in path order launch by launch (the float4 operations of
// finish_kernel, so the accumulation equals frame-by-frame rendering bit for
// bit), the launch's images staged for a deferred gather where one was
// requested (vrhip_comm_gather inside a session), and the final accum /
// RGBA8 / depth.  Staged images are packed like pack_tiles_kernel: owned
// tile j's pixels at [256 j, 256 j + 256), row-major within the tile.
__global__ void __launch_bounds__(kBlockThreads) svc_finish_kernel(const RenderParams p, const SvcFinish f)
{
    const uint32_t tile = blockIdx.x, tid = threadIdx.x;
    const int wave = (int)tid >> 6, lane = (int)tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;
    const uint32_t tile_y = tile_row(gtile, p.tiles_x);
    const uint32_t tile_x = tile_col(gtile, p.tiles_x, p.nranks);
    const uint32_t lx = (uint32_t)((wave & 1) * 8 + (lane & 7)), ly = (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    const uint32_t x = tile_x * 16u + lx, y = tile_y * 16u + ly;
    if (x >= p.wr || y >= p.hr) return;
    const uint32_t ind = x + y * p.W;
    const uint32_t slot = tile * kBlockThreads + tid;
    const uint32_t packed = tile * 256u + ly * 16u + lx;
    vr4 io = f.first_frame != 1u ? p.accum[ind] : mk4(0.f, 0.f, 0.f, 0.f);
    const bool cornell = (p.flags & F_CORNELL) != 0u;
    uint32_t frame = f.first_frame;
    float last_w = 0.f;
    // an F_SPARSE session's escaped pixel: its one result for every path of
    // every launch, in its primary record (primary_kernel), depth term 1
    const bool shared = p.sparse_px && __float_as_int(p.prim[2u * slot].y) == (int)HK_NONE;
    vr4 shared_h = mk4(0.f, 0.f, 0.f, 0.f);
    if (shared) {
        const vr4 b = p.prim[2u * slot + 1u];
        shared_h = mul4s(mk4(b.y, b.z, b.w, 1.f), 1.f / 2.f);
    }
    for (uint32_t L = 0; L < f.n; ++L) {
        const vr3* base = reinterpret_cast<const vr3*>(reinterpret_cast<const uint8_t*>(p.paths) + (size_t)L * p.svc_slot_bytes);
        const uint32_t n_paths = 2u * f.n_frames[L];
        if (shared) {
            for (uint32_t q = 0; q < n_paths; ++q) io = add4(io, shared_h);
            last_w = 1.f;
        } else {
            const float depth = reinterpret_cast<const float*>(p.paths + (size_t)2u * p.svc_kmax * p.path_stride)[slot];
            const vr3* src = base + slot;
            // VR_SVC_FINISH_BATCH results loaded before they are added (in
            // path order): a shard's session has few blocks per CU, and one
            // load in flight per thread left its finish pass latency-bound
            for (uint32_t q0 = 0; q0 < n_paths; q0 += VR_SVC_FINISH_BATCH) {
                vr3 r[VR_SVC_FINISH_BATCH];
#pragma unroll
                for (int j = 0; j < VR_SVC_FINISH_BATCH; ++j)
                    if (q0 + j < n_paths) r[j] = src[(size_t)(q0 + j) * p.path_stride];
#pragma unroll
                for (int j = 0; j < VR_SVC_FINISH_BATCH; ++j) {
                    if (q0 + j < n_paths) {
                        last_w = (cornell && escaped(r[j].x)) ? 0.f : depth;
                        io = add4(io, mul4s(mk4(r[j].x, r[j].y, r[j].z, last_w), 1.f / 2.f));
                    }
                }
            }
        }
        frame += f.n_frames[L];
        if (f.gather[L]) {
            uint8_t* st = f.staging + (size_t)L * f.stage_bytes;
            if (f.gather[L] & 1u) reinterpret_cast<u8x4*>(st)[packed] = tonemap(io, frame - 1u, p.tone_t);
            if (f.gather[L] & 4u) {
                const unsigned char db = f2u8((1.f - last_w) * 255);
                u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
                reinterpret_cast<u8x4*>(st + (size_t)4u * f.stage_pixels)[packed] = dv;
            }
            if (f.gather[L] & 2u) reinterpret_cast<vr4*>(st + (size_t)8u * f.stage_pixels)[packed] = io;
        }
    }
    const unsigned char db = f2u8((1.f - last_w) * 255);
    u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
    p.depth[ind] = dv;
    p.rgba[ind] = tonemap(io, frame - 1u, p.tone_t);
    p.accum[ind] = io;
}

int launch_service(const RenderParams& p, uint32_t n_tiles, int stack_depth, void* stream)
{
    if (n_tiles == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t need = p.flags & kFeatAll;
    if (need == kFeatCornellMesh) launch_spec_c2(p, n_tiles, stack_depth, s, 2);
    else if (need == kFeatHdriMesh) launch_spec_c5(p, n_tiles, stack_depth, s, 2);
    else if (need == kFeatHdriMeshTex) launch_spec_c3(p, n_tiles, stack_depth, s, 2);
    else launch_class(p, need, n_tiles, stack_depth, s, 2);
    return (int)hipGetLastError();
}

int launch_service_finish(const RenderParams& p, const SvcFinish& f, uint32_t n_tiles, void* stream)
{
    if (n_tiles == 0 || f.n == 0) return 0;
    hipLaunchKernelGGL(svc_finish_kernel, dim3(n_tiles), dim3(kBlockThreads), 0, (hipStream_t)stream, p, f);
    return (int)hipGetLastError();
}

int launch_finish(const RenderParams& p, uint32_t n_tiles, void* stream)
{
    if (n_tiles == 0 || !p.use_scratch) return 0;
    hipLaunchKernelGGL(finish_kernel, dim3(n_tiles), dim3(kBlockThreads), 0, (hipStream_t)stream, p);
    return (int)hipGetLastError();
}

int launch_half_to_float(const uint16_t* src, vr4* dst, size_t n, void* stream)
{
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(half_to_float_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, dst, n);
    return (int)hipGetLastError();
}

int launch_pack_tiles(const void* src, void* dst, uint32_t elem_bytes, uint32_t W, uint32_t tiles_x,
                      uint32_t n_owned, uint32_t rank, uint32_t nranks, int unpack, void* stream)
{
    if (n_owned == 0) return 0;
    hipLaunchKernelGGL(pack_tiles_kernel, dim3(n_owned), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t*)src, (uint32_t*)dst, elem_bytes / 4u, W, tiles_x, rank, nranks, unpack);
    return (int)hipGetLastError();
}

int launch_unpack_ranks(const void* src, void* dst, uint32_t elem_bytes, uint32_t W, uint32_t tiles_x,
                        uint32_t total_tiles, uint32_t r0, uint32_t nranks, size_t stride_bytes, void* stream)
{
    if (r0 >= nranks || total_tiles == 0) return 0;
    const uint32_t max_owned = (total_tiles + nranks - 1u) / nranks;
    hipLaunchKernelGGL(unpack_ranks_kernel, dim3(max_owned, nranks - r0), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t*)src, (uint32_t*)dst, elem_bytes / 4u, W, tiles_x, total_tiles, r0, nranks,
                       stride_bytes / 4u);
    return (int)hipGetLastError();
}

// Exhaustive checks of the short sequences against the IEEE operations over
// float bit patterns [lo, hi): fn 0 rcp_rn vs 1.f / x (both signs), fn 1
// sqrt_rn vs sqrtf (positive x).  Counts mismatches, records the smallest
// mismatching pattern.
// fn 2: the table tonemap byte (tone_byte) vs the f64 one (tone_byte_ref)
// over [lo, hi) and -0.0
__global__ void selftest_exact_kernel(int fn, uint32_t lo, uint32_t hi, unsigned long long* n_bad, uint32_t* first_bad,
                                      const float* T)
{
    const uint32_t stride = gridDim.x * blockDim.x;        // hi <= 2^31: b + stride cannot wrap
    unsigned long long bad = 0;
    uint32_t first = 0xffffffffu;
    for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi; b += stride) {
        for (int neg = 0; neg < (fn == 0 || (fn == 2 && b == 0u) ? 2 : 1); ++neg) {
            const uint32_t bits = neg ? (b | 0x80000000u) : b;
            const float x = __uint_as_float(bits);
            bool diff;
            if (fn == 2) {
                diff = tone_byte(x, T) != tone_byte_ref(x);
            } else {
                const float got = fn == 0 ? rcp_rn(x) : sqrt_rn(x);
                const float want = fn == 0 ? 1.f / x : __builtin_sqrtf(x);
                diff = __float_as_uint(got) != __float_as_uint(want);
            }
            if (diff) {
                ++bad;
                first = bits < first ? bits : first;
            }
        }
    }
    if (bad) {
        atomicAdd(n_bad, bad);
        atomicMin(first_bad, first);
    }
}

int launch_selftest_exact(int fn, uint32_t lo, uint32_t hi, unsigned long long* n_bad, uint32_t* first_bad,
                          const float* tone_t, void* stream)
{
    hipLaunchKernelGGL(selftest_exact_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream, fn, lo, hi, n_bad,
                       first_bad, tone_t);
    return (int)hipGetLastError();
}

// The tonemap threshold table (tone_byte): T[k] = the smallest float c in
// [0, 1] whose byte tone_byte_ref(c) >= k, by bisection over the bit
// patterns (tone_byte_ref(1) = 255); T[0] = 0.
__global__ void tone_table_kernel(float* T)
{
    const uint32_t k = threadIdx.x;
    if (k == 0) { T[0] = 0.f; return; }
    uint32_t lo = 0u, hi = 0x3f800000u;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (tone_byte_ref(__uint_as_float(mid)) >= k) hi = mid;
        else lo = mid + 1u;
    }
    T[k] = __uint_as_float(lo);
}

int launch_tone_table(float* T, void* stream)
{
    hipLaunchKernelGGL(tone_table_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, T);
    return (int)hipGetLastError();
}

// Vector-memory gather roof (vrhip_microbench_vmem): every lane issues
// `iters` rounds of 4 independent raw buffer loads of W bytes from a
// 64-B-line table of `n_lines` lines (L2-resident at the sizes used), the
// lanes of a wave split into `distinct` groups that read one address each
// (distinct = 1: one address per wave-instruction, as lanes traversing the
// same node; 64: every lane its own line).  Addresses chain through the
// loaded data, so nothing is hoisted; 4 chains per lane keep it
// throughput-bound.
template <int W>
__global__ void __launch_bounds__(256) vmem_roof_kernel(const uint32_t* tab, uint32_t n_lines, uint32_t distinct,
                                                        int iters, uint32_t* out)
{
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(tab, n_lines * 64u);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t group = lane % distinct;
    const uint32_t wave = (blockIdx.x * 256u + threadIdx.x) >> 6;
    const uint32_t m = n_lines - 1u;                        // n_lines: a power of two
    uint32_t i0 = (wave * 2654435761u + group * 40503u) & m;
    uint32_t i1 = (i0 + 977u) & m, i2 = (i0 + 5003u) & m, i3 = (i0 + 31337u) & m;
    uint32_t acc = 0;
    auto ld = [&](uint32_t line) -> uint32_t {
        const int off = (int)(line * 64u);
        if constexpr (W == 16) { const vr_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0); return v.x ^ v.w; }
        else if constexpr (W == 12) { const vr_u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0); return v.x ^ v.z; }
        else if constexpr (W == 8) { const vr_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0); return v.x ^ v.y; }
        else return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    };
#pragma unroll 1
    for (int i = 0; i < iters; ++i) {
        const uint32_t a = ld(i0), b = ld(i1), c = ld(i2), d = ld(i3);
        acc += a + b + c + d;
        i0 = (i0 * 5u + 7919u + a) & m; i1 = (i1 * 5u + 104729u + b) & m;
        i2 = (i2 * 5u + 1299709u + c) & m; i3 = (i3 * 5u + 15485863u + d) & m;
    }
    if (acc == 0x12345678u) out[0] = acc;      // never true for the zero table: keeps the loads live
}

int launch_vmem_roof(int width, const uint32_t* tab, uint32_t n_lines, uint32_t distinct, int iters,
                     uint32_t blocks, uint32_t* out, void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    switch (width) {
    case 16: hipLaunchKernelGGL(vmem_roof_kernel<16>, dim3(blocks), dim3(256), 0, s, tab, n_lines, distinct, iters, out); break;
    case 12: hipLaunchKernelGGL(vmem_roof_kernel<12>, dim3(blocks), dim3(256), 0, s, tab, n_lines, distinct, iters, out); break;
    case 8: hipLaunchKernelGGL(vmem_roof_kernel<8>, dim3(blocks), dim3(256), 0, s, tab, n_lines, distinct, iters, out); break;
    case 4: hipLaunchKernelGGL(vmem_roof_kernel<4>, dim3(blocks), dim3(256), 0, s, tab, n_lines, distinct, iters, out); break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int launch_selftest_math(int fn, const float* a, const float* b, float* out, size_t n, void* stream)
{
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(selftest_math_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, fn, a, b, out, n);
    return (int)hipGetLastError();
}

} // namespace vr
