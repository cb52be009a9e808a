// vr_params.hpp -- launch parameters shared by the host API (vrhip_api.cpp)
// and the gfx950 kernels (vr_kernel.hip).  Plain C++ types only.
#pragma once
#include <stddef.h>
#include <stdint.h>

// The tile at index gt of the dealing sequence (rank r holds r, r+N, r+2N, ...):
// row gt / tiles_x, column (gt mod tiles_x + row) mod tiles_x when N > 1
// (one rank: row-major, the order the one-GPU kernels were tuned on).  Rotating each
// row by its index deals a rank diagonals: with plain row-major dealing and a
// tile row a multiple of N (every BASELINE size at N = 2, 4, 8) a rank held
// fixed tile columns, and the columns' costs differ -- 8-rank rehearsal, the
// slowest rank's step C2 0.799 -> 0.786 ms, C3 0.218 -> 0.210 ms
// (profiles/r06z).  VR_TILE_STAGGER=0: row-major dealing (A/B builds).
#ifndef VR_TILE_STAGGER
#define VR_TILE_STAGGER 1
#endif
constexpr uint32_t tile_row(uint32_t gt, uint32_t tiles_x) { return gt / tiles_x; }
constexpr uint32_t tile_col(uint32_t gt, uint32_t tiles_x, uint32_t nranks)
{
    return (VR_TILE_STAGGER && nranks > 1u) ? (gt % tiles_x + gt / tiles_x) % tiles_x : gt % tiles_x;
}

namespace vr {

// float4 / float2 with the reference's memory layout (16 B / 8 B aligned)
struct alignas(16) vr4 { float x, y, z, w; };
struct alignas(8) vr2 { float x, y; };
struct vr3 { float x, y, z; };        // packed 12 B (triangle vertices: 3 x dwordx3 per test)
struct alignas(4) u8x4 { unsigned char x, y, z, w; };

enum Flags : uint32_t {
    F_CORNELL = 1u << 0,     // kUseCornellBox      (PathTracer.cu:32)
    F_EXAMPLE = 1u << 1,     // kUseExampleSphere   (:30)
    F_VIEW_BRDF = 1u << 2,   // kViewBRDF           (:31)
    F_MESH = 1u << 3,        // kMeshInitialised    (:29)
    F_BRDF = 1u << 4,        // kHasBRDF            (:28)
    F_TEX_DIFF = 1u << 5,    // kHasDiffuseMap      (:25)
    F_TEX_NORM = 1u << 6,    // kHasNormalMap       (:26)
    F_TEX_SPEC = 1u << 7,    // kHasSpecularMap     (:27)
    F_STRICT = 1u << 8,      // visit every pierced box, as the reference (no t-culling)
    // compile-time only (never in RenderParams::flags): the instrumented copy
    // of the production kernels (vrhip_render_profiled) -- same algorithm,
    // launch shape and results, plus per-lane counts of the memory operations
    // they execute
    F_COUNT_EXEC = 1u << 10,
    // compile-time only: the path kernel of launches with RenderParams::inline_prim
    // (paths trace their own camera ray; a separate instantiation, so the
    // multi-frame kernels keep the registers that code would take)
    F_INLINE_PRIM = 1u << 13,
    // compile-time only: the path kernel of small launches (< 2^24 paths:
    // one frame per call, shards), whose drain is a large share of the
    // launch: it measures per-path costs for the next launch's longest-first
    // order and lets idle lanes help the last traversals (vr_kernel.hip);
    // a separate instantiation, so the whole-frame kernels keep those registers
    F_SMALL = 1u << 14,
    // compile-time only: the render service's persistent kernel (render_service_kernel):
    // consecutive launches of a session from a descriptor ring, tagged
    // primary records, results per launch slot (vrhip_api.cpp Session)
    F_SERVICE = 1u << 15,
    // compile-time only: the path kernel of HDRI mesh launches that skip the
    // pixels whose camera ray escapes (RenderParams::sparse_px): the primary
    // pass stores each such pixel's one shared result and lists the pixels
    // whose camera ray hits the scene; the path kernel runs their paths only
    F_SPARSE = 1u << 16,
};
constexpr int kMaxFramesPerLaunch = 64;

// counting variants, slots [0, kCounters): rays, node visits, vert0 slot
// reads, triangle tests, attribute bytes, texture fetches, HDRI fetches, BRDF
// lookups.  The instrumented production kernels also fill slots
// [kExecCounterBase, +kExecCounters): node visits served from the LDS copy,
// triangle loads issued (36 B each), mesh hits shaded, mesh hits shaded
// through the normal map, and every global lane load issued, by width: 16, 12,
// 8 and 4 B, and paths whose result was the shared escape radiance of
// their pixel's camera ray (render_kernel; no HDRI fetch of their own).
constexpr int kCounters = 8;
constexpr int kExecCounterBase = 16;
constexpr int kExecCounters = 9;
constexpr int kBand = 16;            // block height of the reference launch (PathTracer.cu:887)
constexpr int kBlockThreads = 256;   // 16x16 tile, four 8x8 wave64 sub-tiles
// render_wave_kernel work queues: RenderParams::n_queues counters (a power of
// two, multiple of 8), kQueueStride uint32 apart: VR_QUEUES for launches of
// fewer than 2^25 paths, VR_QUEUES_LARGE above (C5-size launches dequeue
// fastest: 64 heads +4 % there, while C2 / C3 frames and shards prefer 16)
#ifndef VR_QUEUES
#define VR_QUEUES 16
#endif
#ifndef VR_QUEUES_LARGE
#define VR_QUEUES_LARGE 64
#endif
// HDRI scenes (no Cornell box) below 2^25 paths: 32 heads (C3 12,560-12,882
// -> 13,197-13,239 Mpaths/s against 16; C2 prefers 16: 4,105 vs 4,093)
#ifndef VR_QUEUES_HDRI
#define VR_QUEUES_HDRI 32
#endif
#define VR_MAX_QUEUES_ (VR_QUEUES > VR_QUEUES_LARGE ? VR_QUEUES : VR_QUEUES_LARGE)
#define VR_MAX_QUEUES (VR_MAX_QUEUES_ > VR_QUEUES_HDRI ? VR_MAX_QUEUES_ : VR_QUEUES_HDRI)
static_assert((VR_QUEUES & (VR_QUEUES - 1)) == 0 && VR_QUEUES % 8 == 0, "VR_QUEUES: power of two, multiple of 8");
static_assert((VR_QUEUES_LARGE & (VR_QUEUES_LARGE - 1)) == 0 && VR_QUEUES_LARGE % 8 == 0,
              "VR_QUEUES_LARGE: power of two, multiple of 8");
static_assert((VR_QUEUES_HDRI & (VR_QUEUES_HDRI - 1)) == 0 && VR_QUEUES_HDRI % 8 == 0,
              "VR_QUEUES_HDRI: power of two, multiple of 8");
constexpr uint32_t kQueueStride = 256;

// ---- render service (vrhip_set_service; vr_kernel.hpp service_body) --------
// A session is a run of render launches on one persistent kernel: the host
// appends launch descriptors to a ring in host-pinned memory and bumps
// `posted`; a polling wave mirrors them into device memory; every wave takes
// chunks of launch L, then L + 1, ... so the launches' drains overlap.
// launch slots per session: a session's drain, finish pass and primary pass
// are paid once per this many launches (r06: 32 -> 128, the 8-way C3 shard
// steps of a 100-step run 0.229 -> see DESIGN 6)
#ifndef VR_SVC_SLOTS
#define VR_SVC_SLOTS 128
#endif
constexpr uint32_t kSvcMaxLaunches = VR_SVC_SLOTS;
struct SvcLaunch {                                 // one launch of a session (272 B)
    uint32_t first_frame, n_frames, pad0, pad1;
    uint32_t times[kMaxFramesPerLaunch];
};
constexpr uint32_t kSvcLaunchWords = (uint32_t)(sizeof(SvcLaunch) / 4);
struct SvcHostCtl {                                // host-pinned (coherent)
    uint32_t posted;                               // host: launches posted, desc[0, posted) are valid
    uint32_t closed;                               // host: 1 = no launch follows `posted` (written after it)
    uint32_t pad0[30];
    // device (the ring wave): 0 while the kernel serves; launches consumed |
    // kSvcClosed once it stops.  Retiring on its own (idle) it writes this
    // BEFORE its last look at `posted`, and the host reads it AFTER storing
    // `posted` (svc_post), so a launch posted as the kernel retires is seen
    // as taken by exactly one side (svc_ring_wave, vrhip_api.cpp svc_post)
    uint32_t retired;
    uint32_t pad1[31];
    SvcLaunch desc[kSvcMaxLaunches];
};
constexpr uint32_t kSvcClosed = 0x80000000u;
struct SvcDevCtl {                                 // device memory, zeroed when a session opens
    uint32_t ctl;                                  // mirror of the host ring: posted | closed (kSvcClosed), only grows
    uint32_t pad0[31];
    uint32_t sparse_n;                             // F_SPARSE sessions: pixels listed by the primary pass
    uint32_t pad1[31];
    SvcLaunch desc[kSvcMaxLaunches];               // device copies of the descriptors (sc1 stores, then ctl)
};
// per launch: work-queue heads and drained-queue mask, kQueueStride words apart
constexpr uint32_t kSvcQctlWords = (VR_MAX_QUEUES + 1u) * kQueueStride;
// the session finish pass (svc_finish_kernel): per launch, its frame count
// and which images (bit 0 RGBA8, 1 accum, 2 depth: vrhip_comm_gather's
// `what`) to stage for a deferred gather
struct SvcFinish {
    uint32_t n;                                    // launches in the session
    uint32_t first_frame;                          // frame number of launch 0's first frame
    uint32_t n_frames[kSvcMaxLaunches];
    uint32_t gather[kSvcMaxLaunches];
    uint8_t* staging;                              // per launch: stage_bytes (owned pixels x 24 B: rgba, depth, accum)
    size_t stage_bytes;
    uint32_t stage_pixels;                         // pixels per staged image (the most any rank owns)
};

// the finish pass's completion flag: arrival-count groups (a power of two)
constexpr uint32_t kSyncGroups = 256;
struct RenderParams {
    vr4 cam_o, cam_d, cx, cy;        // cx, cy precomputed exactly as PathTracer.cu:833-836
    uint32_t W, H, wr, hr;           // wr/hr: rendered region (grid truncation, :888-889)
    const float* cam_sxy;            // camera-ray screen offsets per column [W] then per row [H] (:842-843)
    float fresnel_coef, fresnel_pow;
    uint32_t flags;
    uint32_t tiles_x;                // wr / 16
    uint32_t rank, nranks;           // 16x16 tiles dealt round-robin: rank owns tiles rank + j*nranks
    uint32_t first_frame, n_frames;
    uint32_t split;                  // path groups per pixel (blocks per tile)
    uint32_t use_scratch;            // 1: paths store radiance to `paths`, finish_kernel accumulates
    uint32_t path_stride;            // owned tiles * 256 (scratch row length)
    // per-path radiances [2*n_frames][path_stride] and, per slot, the
    // pixel's depth term, from which finish_kernel rebuilds each path's .w
    // (vr_kernel.hip store_path)
    vr3* paths;
    float* path_w;
    vr4* prim;                       // per owned pixel: the camera ray's closest hit (2 x vr4, primary_kernel)
    uint32_t* chunk_ctr;             // render_wave_kernel's work queue heads (zeroed by finish_kernel)
    uint32_t wave_blocks;            // render_wave_kernel: CUs to fill with one resident set of blocks
    uint32_t waves_cap;              // render_wave_kernel: at most this many waves per SIMD (0: the kernel's residency)
    // longest-first scheduling (render_wave_kernel): each path's cost (node
    // visits / 2, saturated to a byte; same indexing as `paths`; nullptr: not
    // measured), summed per sub-tile by finish_kernel into sub_cost, and the
    // order the previous launch on this scratch measured (per XCD, order_cap
    // entries each; nullptr: band order)
    uint8_t* path_cost;
    uint32_t* sub_cost;
    const uint32_t* sub_order;
    uint32_t order_cap;
    uint32_t small_blocks;           // render_wave_kernel: 256-thread blocks (launches of < 2^24 paths)
    uint32_t n_queues;               // render_wave_kernel: work queue heads in use (VR_QUEUES / VR_QUEUES_LARGE)
    uint32_t inline_prim;            // paths trace their own camera ray (no primary_kernel pass; F_INLINE_PRIM kernel)
    const float* tone_t;             // the tonemap threshold table (vr_kernel.hpp tone_byte; nullptr: f64 pow)
    const vr4* bvh;
    const vr4* bvh16;                // same nodes, conservative fp16 boxes, 32 B each (culled traversal)
    uint32_t n_nodes;                // inner nodes in bvh (4 rows each, area-ordered)
    const vr3* verts;                // 3 vertices per triangle, compact leaf order (face normal at shading)
    const vr3* tri_e;                // per triangle (v0, v1 - v0, v2 - v0): the traversal's copy
    // per triangle: its leaf's path from the root of the binary tree (bit i =
    // child taken at depth i) under a leading 1 bit -- the equal-t tie-break
    // of the culled traversal (ref_first in vr_kernel.hip)
    const unsigned long long* tpath;
    uint32_t n_tris;                 // triangles in verts/normals/tangents/uvs
    const vr4* normals;
    const vr4* tangents;
    const vr2* uvs;
    const vr4* hdr;
    uint32_t hdr_w, hdr_h;
    const vr4* tex[3];
    uint32_t tex_w[3], tex_h[3];
    const float* brdf;
    vr4* accum;
    u8x4* rgba;
    u8x4* depth;
    unsigned long long* counters;    // kCounters entries (counting variant only)
    // render service launches (F_SERVICE) only
    SvcHostCtl* svc_host;            // device pointer of the host-pinned descriptor ring
    SvcDevCtl* svc_dev;
    uint32_t* svc_qctl;              // kSvcQctlWords per launch slot
    size_t svc_slot_bytes;           // result scratch per launch slot: 2 svc_kmax rows of path_stride vr3, then path_w
    uint32_t svc_kmax;               // frames per launch a slot holds
    uint32_t svc_idle_ticks;         // 100 MHz ticks with no new launch after which the service retires
    // F_SPARSE launches (nullptr otherwise): the slots of the owned pixels
    // whose camera ray hits the scene, appended by primary_kernel one wave
    // (8x8 sub-tile) at a time (their count at sparse_count(p), reset by
    // finish_kernel / zeroed when a session opens)
    uint32_t* sparse_px;
    // a synchronous call's completion flag (nullptr: none): the finish pass's
    // last block stores sync_seq to host-coherent sync_flag once every block's
    // results are visible device-wide (sync_ctr: its block counter, left at 0)
    uint32_t* sync_flag;
    uint32_t* sync_ctr;              // kSyncGroups group words 256 B apart, then the top word
    uint32_t sync_seq;
    uint32_t times[kMaxFramesPerLaunch];
};

// host-side launchers implemented in vr_kernel.hip
// count: 0 production kernels, 1 reference-algorithm counting variant,
// 2 instrumented production kernels (F_COUNT_EXEC)
int launch_render(const RenderParams& p, uint32_t n_tiles, int stack_depth, int count, void* stream);
// use_scratch launches: sums the per-path results of launch_render in path order
int launch_finish(const RenderParams& p, uint32_t n_tiles, void* stream);
// render service: the persistent kernel of a session (mesh scenes), and the
// session's finish pass (sums every launch's results in path order)
int launch_service(const RenderParams& p, uint32_t n_tiles, int stack_depth, void* stream);
int launch_service_finish(const RenderParams& p, const SvcFinish& f, uint32_t n_tiles, void* stream);
// sorts the sub-tiles of each XCD by the costs a launch measured (for the next launch on the same scratch)
int launch_order(uint32_t* cost, uint32_t* order, uint32_t n_sub, uint32_t cap, void* stream);
int launch_half_to_float(const uint16_t* src, vr4* dst, size_t n, void* stream);
int launch_pack_tiles(const void* src, void* dst, uint32_t elem_bytes, uint32_t W, uint32_t tiles_x,
                      uint32_t n_owned, uint32_t rank, uint32_t nranks, int unpack, void* stream);
// the gathering rank: ranks r0..nranks-1's packed buffers (stride_bytes apart,
// from src) scattered into the image in one launch
int launch_unpack_ranks(const void* src, void* dst, uint32_t elem_bytes, uint32_t W, uint32_t tiles_x,
                        uint32_t total_tiles, uint32_t r0, uint32_t nranks, size_t stride_bytes, void* stream);
int launch_vmem_roof(int width, const uint32_t* tab, uint32_t n_lines, uint32_t distinct, int iters,
                     uint32_t blocks, uint32_t* out, void* stream);
int launch_selftest_math(int fn, const float* a, const float* b, float* out, size_t n, void* stream);
int launch_selftest_exact(int fn, uint32_t lo, uint32_t hi, unsigned long long* n_bad, uint32_t* first_bad,
                          const float* tone_t, void* stream);
// the tonemap threshold table (256 floats; vr_kernel.hpp tone_byte)
int launch_tone_table(float* T, void* stream);

} // namespace vr
