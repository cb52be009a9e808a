// vrhip_api.cpp -- C ABI of libvrhip.so (declared in include/vrhip.h).
//
// Host half of the MI355X backend: the device-side counterpart of
// vRendererCuda (src/vRendererCuda.cpp) and the cu_* device ABI
// (cuda/include/PathTracer.cuh:107-165), re-designed around one context per
// GPU, status codes instead of exit(0) (src/vRendererCuda.cpp:454-467), flags
// passed by value in the launch instead of __constant__ symbol copies
// (cuda/src/PathTracer.cu:976-1001), and multi-frame render steps.
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <hip/hip_gl_interop.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <algorithm>
#include <array>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/vrhip.h"
#include "vr_bvh.hpp"
#include "vr_exr.hpp"
#include "vr_merl.hpp"
#include "vr_params.hpp"

using vr::vr3;
using vr::vr2;
using vr::vr4;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) { g_last_error = msg; return code; }

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(VRHIP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
    } while (0)

template <typename T>
void dfree(T*& p) { if (p) { (void)hipFree((void*)p); p = nullptr; } }

} // namespace

// Launches of at most this many paths per pixel trace the camera ray in the
// path kernel instead of a separate primary pass (RenderParams::inline_prim).
#ifndef VR_INLINE_PRIM_PATHS
#define VR_INLINE_PRIM_PATHS 2
#endif
// Path streams (see render_impl): launch i's kernels wait for the finish
// pass of launch i - VR_PATH_STREAMS, the last reader of the same scratch.
// multi-frame shards on the small-launch kernels (vr_kernel.hip launch_wave)
#ifndef VR_SHARD_SMALL
#define VR_SHARD_SMALL 0
#endif
#ifndef VR_PATH_STREAMS
#define VR_PATH_STREAMS 3
#endif

struct vrhip_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint32_t W = 0, H = 0;
    vr4* accum = nullptr;
    float* cam_sxy = nullptr;                   // camera-ray screen offsets: W column values, then H row values
    vr::u8x4* rgba = nullptr;
    vr::u8x4* depth = nullptr;
    // camera (vCamera, cuda/include/PathTracer.cuh:58-84)
    float cam_o[3] = { 0.f, 0.f, 150.f }, cam_d[3] = { 0.f, 0.f, -1.f };
    float cam_up[3] = { 0.f, 1.f, 0.f }, cam_right[3] = { 1.f, 0.f, 0.f };
    float fov_scale = 0.f;
    uint32_t frame = 1;                         // m_frame (src/vRendererCuda.cpp:24)
    float fresnel_coef = 0.1f, fresnel_pow = 3.f; // src/vRendererCuda.cpp:27-28
    bool cornell = false, example = false, view_brdf = false;
    bool strict = false;          // exact reference traversal (no t-culling)
    // mesh
    vr4* bvh = nullptr; vr4* bvh16 = nullptr; vr3* verts = nullptr; vr3* tri_e = nullptr; unsigned long long* tpath = nullptr; vr4* normals = nullptr; vr4* tangents = nullptr; vr2* uvs = nullptr;
    size_t n_bvh = 0, n_slots = 0;
    uint32_t bvh_depth = 0, bvh_nodes = 0, dev_nodes = 0, dev_tris = 0;
    bool mesh = false;
    // environment / textures / brdf
    vr4* hdr = nullptr; uint32_t hdr_w = 0, hdr_h = 0;
    vr4* tex[3] = { nullptr, nullptr, nullptr }; uint32_t tex_w[3] = { 0, 0, 0 }, tex_h[3] = { 0, 0, 0 };
    float* brdf = nullptr;
    // sharding
    uint32_t rank = 0, nranks = 1;
    // path groups per pixel (0: automatic) and their result scratch
    uint32_t path_split = 0;
    uint32_t cu_count = 256;
    // Render launches take the path streams in turn, each with its own
    // scratch, so a launch's paths can start while the previous launch
    // drains; finish passes stay in order on `stream` (see render_impl)
    struct Lane {
        hipStream_t s = nullptr;
        vr4* paths = nullptr;
        size_t paths_cap = 0;        // float4 elements
        vr4* prim = nullptr;         // primary hits, 2 float4 per owned pixel
        size_t prim_cap = 0;         // float4 elements
        uint32_t* chunk_ctr = nullptr;   // wave kernel work queue heads
        // longest-first scheduling: per sub-tile costs measured by a launch
        // on this scratch and the per-XCD order sorted from them, in two
        // slots used by turns (ordered launch i measures into slot oi and
        // takes the order launch i-2 left there: its sort is long finished,
        // so the launch waits for nothing -- with one slot, a one-frame
        // call's launch waited for the sort of the call before, ≈ 12 µs of
        // cross-stream hand-off per synchronous frame, r05)
        uint32_t* sub_cost[2] = { nullptr, nullptr };
        uint32_t* sub_order[2] = { nullptr, nullptr };
        size_t sub_cap = 0;          // sub-tiles the buffers hold
        uint32_t order_nsub[2] = { 0, 0 };   // sub-tile count each slot's order was sorted for (0: none)
        uint32_t oi = 0;             // the slot the next ordered launch uses
        uint32_t* px_list = nullptr;     // F_SPARSE launches: the pixels whose camera ray hits (RenderParams::sparse_px)
        size_t px_cap = 0;
        hipEvent_t done = nullptr;   // recorded on `s` after the render kernels
        hipEvent_t finished = nullptr;   // recorded on `stream` after the finish pass that read this scratch
        hipEvent_t ordered[2] = { nullptr, nullptr };   // recorded on `s` after the order pass of each slot
        bool order_pending[2] = { false, false };       // an order pass was queued on the slot since a launch waited for it
        bool used = false;
    } lane[VR_PATH_STREAMS];
    uint32_t parity = 0;
    int overlap = -1;            // vrhip_set_overlap: 1 always, 0 never, -1 small launches only
    bool cost_order = true;      // longest-first sub-tile order for small launches (VRHIP_COST_ORDER=0: off)
    bool join = true;            // the next launches must wait for everything queued on `stream`
    hipEvent_t ev_join = nullptr;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // render-kernel start/stop event pairs not yet added to the totals (read
    // without blocking at the next render, all of them by vrhip_kernel_stats),
    // and recycled events
    struct Span { hipEvent_t first, second; uint32_t launches; };
    std::deque<Span> kev_pending;
    std::vector<hipEvent_t> kev_free;
    bool timed = false;          // ev1 marks the end of the last render
    bool ev0_valid = false;      // ev0 marks its start (kernel timing on)
    // vrhip_set_kernel_timing (VRHIP_KERNEL_TIMING=0: off): span events around
    // every launch's render kernels (vrhip_kernel_stats) and each call
    // (vrhip_last_kernel_ms)
    bool kernel_timing = true;
    float* tone_t = nullptr;     // the tonemap threshold table (vr_kernel.hpp tone_byte), filled at creation
    double kernel_ms_total = 0.0;    // union of the launches' render-kernel spans (overlapping launches count once)
    uint64_t launches_total = 0;
    uint32_t last_split = 1, last_use_scratch = 0, last_kind = 0;   // vrhip_last_launch_info
    // spans as [start, end) in ms after kev_origin (the start event of the
    // first span since the last reset), merged into disjoint intervals: launches
    // on different path streams can start out of queue order
    hipEvent_t kev_origin = nullptr;
    std::vector<std::pair<double, double>> kev_union;
    unsigned long long* counters = nullptr;
    // GL interop (colour, depth textures registered by the display host)
    hipGraphicsResource_t gl_res[2] = { nullptr, nullptr };
    // render service (vrhip_set_service): a session of launches on one
    // persistent kernel (vr_kernel.hpp service_body), see svc_open
    struct Session {
        bool open = false;
        hipStream_t s = nullptr;                  // the service stream
        // descriptor rings in host-pinned coherent memory, one per session in
        // turn: a closed session's kernel may still read its ring while the
        // next session fills the other (ring_done: after that kernel)
        vr::SvcHostCtl* rings[2] = { nullptr, nullptr };
        vr::SvcHostCtl* rings_dev[2] = { nullptr, nullptr };
        hipEvent_t ring_done[2] = { nullptr, nullptr };
        bool ring_used[2] = { false, false };
        uint32_t ring_i = 0;
        uint32_t cur_ring = 0;                    // the open (or last) session's ring
        // per ring: the launches its last session summed, and whether the
        // kernel's count of consumed launches (SvcHostCtl::retired) was checked
        uint32_t ring_posted[2] = { 0, 0 };
        bool ring_checked[2] = { true, true };
        vr::SvcHostCtl* host = nullptr;           // the open session's ring
        vr::SvcDevCtl* dev = nullptr;             // device mirror of the ring
        uint32_t* qctl = nullptr; size_t qctl_slots = 0;    // work-queue heads per launch slot
        uint8_t* scratch = nullptr; size_t scratch_cap = 0; // launch slots' path results
        vr4* prim = nullptr; size_t prim_cap = 0;           // the session's primary records, 2 float4 per owned pixel
        uint32_t* subs = nullptr; size_t subs_cap = 0;      // F_SPARSE sessions: the pixels whose camera ray hits
        uint8_t* staging = nullptr; size_t staging_cap = 0; // deferred gathers: per launch slot
        uint32_t slots = 0, kmax = 0, posted = 0;
        size_t slot_bytes = 0;
        int stack = 16;
        uint32_t n_tiles = 0;
        vr::RenderParams p{};                     // the session's launch parameters
        vr::RenderParams key{};                   // what must not change within a session (svc_key)
        vr::SvcFinish fin{};
        std::vector<std::pair<uint32_t, int>> gathers;   // deferred vrhip_comm_gather: (launch, what)
        std::chrono::steady_clock::time_point last_post;
        hipEvent_t k0 = nullptr, k1 = nullptr;    // the service kernel's span
        hipEvent_t finished = nullptr;            // recorded on `stream` after the session's finish pass
        bool finished_used = false;
        // recorded on `stream` right after the finish pass, before the
        // session's deferred gathers; the next session's kernel waits for it
        // instead of for everything on `stream` when nothing it reads was
        // queued there since (stream_epoch unchanged), so it overlaps them
        hipEvent_t summed = nullptr;
        uint64_t summed_epoch = 0;
        bool summed_valid = false;
    } svc;
    // bumped by everything that queues work the render kernels read on
    // `stream` (uploads and other quiesce() callers, clears): Session::summed
    uint64_t stream_epoch = 0;
    int service = -1;                             // 1 every production mesh launch, 0 never, -1 automatic
    // vrhip_set_service_timing (test hook; 0 = default): the kernel's idle
    // limit, the host's post window, a host delay between the window check
    // and the post (forces the retire-vs-post race)
    uint32_t svc_idle_us = 0, svc_window_us = 0, svc_post_delay_us = 0;
    uint64_t svc_refused = 0;                     // launches a retiring session kernel did not take
    // vrhip_service_info: sessions opened, launches they took, gathers deferred
    // to a session's close, sessions the scratch allocation could not open
    uint64_t svc_sessions = 0, svc_served = 0, svc_deferred = 0, svc_alloc_fallbacks = 0;
    size_t svc_budget = 0;                        // vrhip_set_service_budget (0: VRHIP_SERVICE_BYTES / 24 GiB)
    // multi-device renderer (vrhip_create_multi): the lead context holds every
    // member context (itself first); settings fan out to all of them
    std::vector<vrhip_ctx*> group;
    // one-frame launches as a HIP graph (VRHIP_GRAPH=1; one_frame_graph): the
    // path kernel + finish pass captured once per longest-first order slot,
    // their kernel arguments updated per frame
    struct FrameGraph {
        hipGraph_t g = nullptr;
        hipGraphExec_t x = nullptr;
        hipGraphNode_t kn[2] = { nullptr, nullptr };
        hipKernelNodeParams kp[2] = {};
        vr::RenderParams key{};               // the launch parameters except the frame's number and seed
        vr::RenderParams arg{};               // this frame's parameters (the nodes' argument)
        bool valid = false;
    } fgraph[2];
    bool use_graph = false;
    uint64_t graph_launches = 0, graph_captures = 0;
    // completion flag of a synchronous one-frame call (VRHIP_SYNC_FLAG): the
    // finish pass's last block stores the call's number to host-coherent
    // memory, and vrhip_sync polls it instead of waiting for the stream's
    // completion signal (vr_kernel.hip finish_arrive)
    int sync_flag_mode = 1;
    uint32_t* sync_flag = nullptr;   // host-coherent
    uint32_t* sync_ctr = nullptr;    // device: the finish pass's block arrivals
    uint32_t sync_seq = 0;
    uint32_t flag_armed = 0;         // the number the last queued work ends with (0: none)
    bool flag_synced = false;        // the last sync saw it: no render in flight
    bool stream_shared = false;      // the caller has the stream (vrhip_get/set_stream): no flag
    uint64_t sync_flag_waits = 0, sync_stream_waits = 0;
    // the lead of a group: renders since the colour / depth tiles were last
    // gathered (the gather runs when the lead's images are next needed)
    bool group_stale = false;
    // multi-GPU tile gather (vrhip_comm_*): one RCCL communicator per context
    ncclComm_t comm = nullptr;
    uint8_t* comm_send = nullptr;    // this rank's packed tiles (largest element, 16 B/pixel)
    uint8_t* comm_recv = nullptr;    // rank 0: n_ranks packed buffers, comm_slot bytes apart
    size_t comm_slot = 0;            // bytes per rank slot (max owned pixels x 16 B)
    uint32_t comm_rank = 0, comm_n = 0;   // the communicator's rank and size (tiling fixed while it exists)
};

// the finish pass's arrival counters: vr::kSyncGroups group words 256 B apart, then the top word
constexpr size_t kSyncCtrBytes = (64u * vr::kSyncGroups + 64u) * sizeof(uint32_t);
// Largest finish pass that carries the completion flag (tiles of 16x16):
// counting a 3840x2160 pass's 32,400 block arrivals cost more than the flag
// saves (C5 one frame per call +0.6 %, r06zt)
#ifndef VR_SYNC_FLAG_MAX_TILES
#define VR_SYNC_FLAG_MAX_TILES 8192
#endif
static void svc_free(vrhip_ctx* c);
static int svc_close(vrhip_ctx* c);
static int refuse_multi(vrhip_ctx* c, const char* what);
static int multi_gather(vrhip_ctx* c, int what);
static int multi_images(vrhip_ctx* c);

namespace {

// Reference default camera fov: Camera::getFovScale (src/Camera.cpp:4,119-123)
float default_fov_scale()
{
    const float kDegInRad = (float)(M_PI / 180.f);
    const float fovRad = 75.f * kDegInRad;
    return std::tan(fovRad / 2.f);
}

int set_device(vrhip_ctx* c) { HIP_TRY(hipSetDevice(c->device)); return VRHIP_OK; }

int clear_accum(vrhip_ctx* c)
{
    int rc = svc_close(c);                        // the open session's results come first
    if (rc != VRHIP_OK) return rc;
    ++c->stream_epoch;
    c->frame = 1;
    HIP_TRY(hipMemsetAsync(c->accum, 0, sizeof(vr4) * (size_t)c->W * c->H, c->stream));
    return VRHIP_OK;
}

uint32_t rendered_rows(const vrhip_ctx* c) { return (c->H / 16u) * 16u; }

// 16x16 tiles of the rendered region, dealt round-robin: rank r owns tiles
// r, r + n, r + 2n, ... (row-major tile order)
uint32_t owned_tiles_of(uint32_t W, uint32_t H, uint32_t rank, uint32_t n_ranks)
{
    const uint32_t total = (W / 16u) * (H / 16u);
    return total > rank ? (total - rank + n_ranks - 1u) / n_ranks : 0u;
}

// Device mesh layout (see vr_kernel.hip): the reference nodes with leaf
// children re-encoded as ~((first_tri << 7) | count) into compact per-triangle
// arrays (3 slots per triangle, terminator slots dropped).  Built from the
// reference flattening (src/vRendererCuda.cpp:204-279) so the triangles a
// leaf tests, and their order, are exactly the reference's.
struct DeviceMesh {
    std::vector<vr4> nodes, normals, tangents;
    std::vector<vr4> nodes16;        // 2 x 16 B per node: conservative fp16 boxes + child indices
    std::vector<vr3> tris;           // packed 12 B vertices (vertex .w never reaches a result)
    std::vector<vr3> tri_e;          // per triangle v0, v1 - v0, v2 - v0 (fp32, the kernel's own subtractions)
    std::vector<unsigned long long> tpath;   // per triangle: leaf path from the root under a leading 1 bit
    std::vector<vr2> uvs;
};

constexpr int kLeafCountBits = 7;

// Per compact triangle, the path from the root to its leaf (bit i = the child
// taken at depth i) under a leading 1 bit: the key the kernel's equal-t
// tie-break (ref_first) uses to find the two leaves' lowest common ancestor.
// Paths depend only on the tree's shape, so the node renumbering below keeps them.
void tri_paths(DeviceMesh& dm)
{
    dm.tpath.assign(std::max<size_t>(dm.tris.size() / 3, 1), 0ull);
    if (dm.nodes.empty()) return;
    struct Item { size_t off; unsigned long long bits; int depth; };
    std::vector<Item> st{ { 0, 0ull, 0 } };
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        for (int ch = 0; ch < 2; ++ch) {
            int32_t idx;
            std::memcpy(&idx, &dm.nodes[it.off + 3].x + ch, 4);
            const unsigned long long bits = it.bits | ((unsigned long long)ch << it.depth);
            if (idx >= 0) { st.push_back({ (size_t)idx, bits, it.depth + 1 }); continue; }
            const uint32_t code = (uint32_t)~idx;
            const uint32_t first = code >> kLeafCountBits, count = code & ((1u << kLeafCountBits) - 1u);
            for (uint32_t t = first; t < first + count; ++t) dm.tpath[t] = (1ull << (it.depth + 1)) | bits;
        }
    }
}

// Renumbers the inner nodes so that node i is the i-th largest box by surface
// area (a parent always precedes its children; the root stays at 0).  The
// kernel keeps a prefix of this array in LDS: the boxes a random ray is most
// likely to enter.  Only addresses change -- every node keeps its boxes and
// child order, so the traversal visits the same nodes in the same order.
#ifndef VR_TOP_NODES
#define VR_TOP_NODES 1024
#endif
constexpr size_t kTopNodes = VR_TOP_NODES;    // >= any kernel's LDS node cache

void order_nodes_by_area(DeviceMesh& dm)
{
    const size_t n = dm.nodes.size() / 4;
    if (n == 0) return;
    auto child_area = [&](size_t node, int ch) {
        const vr4& a = dm.nodes[4 * node + ch];            // x and y extents of child ch
        const vr4& z = dm.nodes[4 * node + 2];
        const float dx = a.y - a.x, dy = a.w - a.z, dz = ch ? z.w - z.z : z.y - z.x;
        return dx * dy + dy * dz + dz * dx;
    };
    auto child = [&](size_t node, int ch) {
        int32_t idx;
        std::memcpy(&idx, &dm.nodes[4 * node + 3].x + ch, 4);
        return idx;
    };
    std::vector<int32_t> newoff(n, -1);
    std::vector<size_t> order;
    order.reserve(n);
    // the first kTop nodes: largest boxes first (the LDS-cached prefix)
    std::priority_queue<std::pair<float, int64_t>> pq;   // (area, -node): ties by address
    pq.push({ INFINITY, 0 });
    newoff[0] = 0;
    while (!pq.empty() && order.size() < kTopNodes) {
        const size_t node = (size_t)(-pq.top().second);
        pq.pop();
        newoff[node] = (int32_t)(4 * order.size());
        order.push_back(node);
        for (int ch = 0; ch < 2; ++ch) {
            const int32_t idx = child(node, ch);
            if (idx < 0 || newoff[idx / 4] != -1) continue;
            newoff[idx / 4] = -2;                          // queued
            pq.push({ child_area(node, ch), -(int64_t)(idx / 4) });
        }
    }
    // the rest: depth-first from the frontier, the two children of a node
    // placed side by side (a ray that enters one often enters the other, and
    // they share a cache line)
    std::vector<size_t> frontier;
    while (!pq.empty()) { frontier.push_back((size_t)(-pq.top().second)); pq.pop(); }
    std::sort(frontier.begin(), frontier.end(), [&](size_t a, size_t b) { return a < b; });
    std::vector<size_t> st;
    auto place = [&](size_t node) { newoff[node] = (int32_t)(4 * order.size()); order.push_back(node); };
    for (size_t f : frontier) {
        place(f);
        st.push_back(f);
        while (!st.empty()) {
            const size_t node = st.back();
            st.pop_back();
            size_t kids[2];
            int nk = 0;
            for (int ch = 0; ch < 2; ++ch) {
                const int32_t idx = child(node, ch);
                if (idx >= 0 && newoff[idx / 4] == -1) kids[nk++] = (size_t)(idx / 4);
            }
            for (int k = 0; k < nk; ++k) place(kids[k]);
            for (int k = nk - 1; k >= 0; --k) st.push_back(kids[k]);   // first child's subtree next
        }
    }
    std::vector<vr4> out(4 * order.size());
    for (size_t i = 0; i < order.size(); ++i) {
        for (int r = 0; r < 4; ++r) out[4 * i + r] = dm.nodes[4 * order[i] + r];
        for (int ch = 0; ch < 2; ++ch) {
            float* slot = &out[4 * i + 3].x + ch;
            int32_t idx;
            std::memcpy(&idx, slot, 4);
            if (idx >= 0) std::memcpy(slot, &newoff[idx / 4], 4);
        }
    }
    dm.nodes.swap(out);
}

// IEEE binary16 bits of x rounded toward -inf (down) or +inf (up), so the
// half box always contains the float box.  Out-of-range values become
// -inf / +inf on the outward side.
uint16_t half_bits_directed(float x, bool up)
{
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const float ax = std::fabs(x);
    auto half_to_float = [](uint16_t h) {
        const uint32_t s = (h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
        float f;
        if (e == 0) f = std::ldexp((float)m, -24);
        else if (e == 31) f = m ? NAN : INFINITY;
        else f = std::ldexp((float)(m | 0x400u), (int)e - 25);
        return s ? -f : f;
    };
    // truncation toward zero of |x| to half precision
    uint16_t mag;
    if (ax >= 65504.f) {
        mag = 0x7bffu;                                   // max finite
    } else if (ax < std::ldexp(1.f, -14)) {
        mag = (uint16_t)(ax / std::ldexp(1.f, -24));     // subnormal, truncated
    } else {
        int e;
        const float m = std::frexp(ax, &e);              // ax = m * 2^e, m in [0.5, 1)
        const uint32_t mant = (uint32_t)std::ldexp(m, 11) & 0x3ffu;   // 10 fraction bits, truncated
        mag = (uint16_t)(((uint32_t)(e - 1 + 15) << 10) | mant);
    }
    uint16_t h = (uint16_t)(sign | mag);
    // truncation moved |x| toward zero; step one ulp outward where needed
    const float hv = half_to_float(h);
    const bool below = hv < x, above = hv > x;
    if (up && below) h = sign ? (uint16_t)(h - 1) : (uint16_t)(h + 1);
    if (!up && above) h = sign ? (uint16_t)(h + 1) : (uint16_t)(h - 1);
    if ((h & 0x7fffu) == 0x7c00u || ((h & 0x7fffu) > 0x7c00u)) h = (uint16_t)((h & 0x8000u) | 0x7c00u);
    if (up && ax >= 65504.f && x > 0.f && half_to_float(h) < x) h = 0x7c00u;          // +inf
    if (!up && ax >= 65504.f && x < 0.f && half_to_float(h) > x) h = 0xfc00u;         // -inf
    return h;
}

// fp16 copy of the node array for the t-culled traversal: per node
// [c0.lo.x c0.hi.x c0.lo.y c0.hi.y c0.lo.z c0.hi.z c1.lo.x c1.hi.x]
// [c1.lo.y c1.hi.y c1.lo.z c1.hi.z idx0 idx1], lows rounded down and highs up.
void build_nodes16(DeviceMesh& dm)
{
    const size_t n = dm.nodes.size() / 4;
    dm.nodes16.assign(2 * n, vr4{ 0, 0, 0, 0 });
    for (size_t i = 0; i < n; ++i) {
        const vr4 n0 = dm.nodes[4 * i], n1 = dm.nodes[4 * i + 1], nz = dm.nodes[4 * i + 2], ni = dm.nodes[4 * i + 3];
        const float v[12] = { n0.x, n0.y, n0.z, n0.w, nz.x, nz.y, n1.x, n1.y, n1.z, n1.w, nz.z, nz.w };
        uint16_t h[16];
        for (int k = 0; k < 12; ++k) h[k] = half_bits_directed(v[k], (k & 1) != 0);
        std::memcpy(&h[12], &ni.x, 4);
        std::memcpy(&h[14], &ni.y, 4);
        std::memcpy(&dm.nodes16[2 * i], h, 32);
    }
}

bool to_device_layout(const float* bvh, size_t n_bvh_f4, const vr4* verts, const vr4* normals,
                      const vr4* tangents, const vr2* uvs, DeviceMesh& dm, std::string& why)
{
    // The input must be a tree (vr::validate_flat, which every upload runs
    // first, rejects a node or leaf run with two parents): each triangle then
    // has ONE root path, the key of the equal-t tie-break (tri_paths).  A
    // shared node or leaf is refused here too rather than merged, since a
    // merged copy would give its triangles the path of one parent only.
    dm.nodes.assign((const vr4*)bvh, (const vr4*)bvh + n_bvh_f4);
    std::vector<size_t> st{ 0 };
    std::vector<uint8_t> seen(n_bvh_f4 / 4, 0);
    std::unordered_map<int32_t, int> leaf_seen;
    while (!st.empty()) {
        const size_t off = st.back();
        st.pop_back();
        if (seen[off / 4]) { why = "flattened BVH is not a tree (a node has two parents)"; return false; }
        seen[off / 4] = 1;
        float* idxf = &dm.nodes[off + 3].x;
        for (int ch = 0; ch < 2; ++ch) {
            int32_t idx;
            std::memcpy(&idx, &idxf[ch], 4);
            if (idx >= 0) { st.push_back((size_t)idx); continue; }
            if (!leaf_seen.emplace(idx, 1).second) { why = "flattened BVH is not a tree (a leaf has two parents)"; return false; }
            const size_t first = dm.tris.size() / 3;
            size_t s = (size_t)(~idx), count = 0;
            for (;;) {
                uint32_t b;
                std::memcpy(&b, &verts[s].x, 4);
                if (b == 0x80000000u) break;
                for (int k = 0; k < 3; ++k) {
                    dm.tris.push_back(vr3{ verts[s + k].x, verts[s + k].y, verts[s + k].z });
                    dm.normals.push_back(normals[s + k]);
                    dm.tangents.push_back(tangents[s + k]);
                    dm.uvs.push_back(uvs[s + k]);
                }
                s += 3;
                ++count;
            }
            if (count >= (1u << kLeafCountBits)) { why = "leaf with >= 128 triangles"; return false; }
            if (first >= (1u << (31 - kLeafCountBits))) { why = "more than 16M triangle references"; return false; }
            const int32_t code = ~(int32_t)((first << kLeafCountBits) | count);
            std::memcpy(&idxf[ch], &code, 4);
        }
    }
    tri_paths(dm);
    order_nodes_by_area(dm);
    build_nodes16(dm);
    if (dm.tris.empty()) {
        dm.tris.push_back(vr3{ 0, 0, 0 });
        dm.normals.push_back(vr4{ 0, 0, 0, 0 });
        dm.tangents = dm.normals;
        dm.uvs.push_back(vr2{ 0, 0 });
    }
    // The Moller-Trumbore edges are the same fp32 subtractions whichever side
    // performs them; precomputed, the triangle test reads v0 and both edges
    // and skips 6 VALU ops per test.  The face normal at shading keeps using
    // the vertices (v0 - v1 is not -(v1 - v0) for signed zeros).
    dm.tri_e.resize(dm.tris.size());
    for (size_t t = 0; t + 2 < dm.tris.size(); t += 3) {
        const vr3 a = dm.tris[t], b = dm.tris[t + 1], d = dm.tris[t + 2];
        dm.tri_e[t] = a;
        dm.tri_e[t + 1] = vr3{ b.x - a.x, b.y - a.y, b.z - a.z };
        dm.tri_e[t + 2] = vr3{ d.x - a.x, d.y - a.y, d.z - a.z };
    }
    return true;
}

// Waits for the path streams' render kernels (they read the scene and their
// scratch) and makes the next launches wait for all work queued on `stream`.
// Every call that replaces device buffers or the stream goes through here.
void quiesce(vrhip_ctx* c)
{
    (void)svc_close(c);
    ++c->stream_epoch;
    if (c->svc.s) (void)hipStreamSynchronize(c->svc.s);
    for (auto& l : c->lane)
        if (l.s) (void)hipStreamSynchronize(l.s);
    c->join = true;
}

template <typename T>
int upload(vrhip_ctx* c, T*& dst, const void* src, size_t bytes)
{
    quiesce(c);
    dfree(dst);
    HIP_TRY(hipMalloc((void**)&dst, bytes ? bytes : 16));
    if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return VRHIP_OK;
}

} // namespace

extern "C" {

const char* vrhip_last_error(void) { return g_last_error.c_str(); }
int vrhip_abi_version(void) { return VRHIP_ABI_VERSION; }

// SHA-256 of the sources, include/vrhip.h and the compile flags this library
// was built from, tagged so build.py can read it from the file without
// loading it (vrenderer_pathtracer_amd/build.py passes it in)
#ifndef VRHIP_BUILD_ID
#define VRHIP_BUILD_ID "vrhip-build-id:unknown"
#endif
const char* vrhip_build_id(void)
{
    static const char id[] = VRHIP_BUILD_ID;
    static const char tag[] = "vrhip-build-id:";
    return std::strncmp(id, tag, sizeof(tag) - 1) == 0 ? id + sizeof(tag) - 1 : id;
}

int vrhip_device_count(int* count)
{
    if (!count) return fail(VRHIP_ERR_INVALID, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *count = 0; return fail(VRHIP_ERR_NO_DEVICE, hipGetErrorString(e)); }
    *count = n;
    return VRHIP_OK;
}

int vrhip_create(int device, uint32_t width, uint32_t height, vrhip_ctx** out)
{
    if (!out || width == 0 || height == 0 || width > 65535 || height > 65535)
        return fail(VRHIP_ERR_INVALID, "bad create arguments (1..65535 pixels per side)");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(VRHIP_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= n) return fail(VRHIP_ERR_INVALID, "device index out of range");
    vrhip_ctx* c = new vrhip_ctx();
    c->device = device;
    c->W = width; c->H = height;
    c->fov_scale = default_fov_scale();
    if (const char* e = std::getenv("VRHIP_COST_ORDER")) c->cost_order = std::atoi(e) != 0;
    if (const char* e = std::getenv("VRHIP_KERNEL_TIMING")) c->kernel_timing = std::atoi(e) != 0;
    if (const char* e = std::getenv("VRHIP_GRAPH")) c->use_graph = std::atoi(e) != 0;
    if (const char* e = std::getenv("VRHIP_SYNC_FLAG")) c->sync_flag_mode = std::atoi(e) != 0 ? 1 : 0;
    if (const char* e = std::getenv("VRHIP_SERVICE")) c->service = std::max(-1, std::min(1, std::atoi(e)));
    int rc;
    if ((rc = set_device(c)) != VRHIP_OK) { delete c; return rc; }
    auto cleanup = [&](int code) { vrhip_destroy(c); return code; };
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(VRHIP_ERR_HIP, "hipStreamCreate failed"));
    c->stream = c->own_stream;
    for (auto& l : c->lane) {
        if (hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&l.done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l.finished, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l.ordered[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l.ordered[1], hipEventDisableTiming) != hipSuccess)
            return cleanup(fail(VRHIP_ERR_HIP, "path stream setup failed"));
    }
    if (hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(VRHIP_ERR_HIP, "hipEventCreate failed"));
    if (hipMalloc((void**)&c->tone_t, 256 * sizeof(float)) != hipSuccess ||
        vr::launch_tone_table(c->tone_t, c->stream) != 0)
        return cleanup(fail(VRHIP_ERR_HIP, "tonemap table setup failed"));
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->cu_count = (uint32_t)cus;
    const size_t npx = (size_t)width * height;
    if (hipMalloc((void**)&c->accum, sizeof(vr4) * npx) != hipSuccess ||
        hipMalloc((void**)&c->rgba, 4 * npx) != hipSuccess ||
        hipMalloc((void**)&c->depth, 4 * npx) != hipSuccess)
        return cleanup(fail(VRHIP_ERR_NOMEM, "hipMalloc of frame buffers failed"));
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess)
        return cleanup(fail(VRHIP_ERR_HIP, "hipEventCreate failed"));
    {
        // the camera ray's screen offsets (PathTracer.cu:842-843), evaluated
        // in double as there, once per column and row: the kernels index
        // them instead of dividing in f64 per ray
        std::vector<float> sxy((size_t)width + height);
        for (uint32_t x = 0; x < width; ++x) sxy[x] = (float)((0.25 + (double)x) / (double)width - 0.5);
        for (uint32_t y = 0; y < height; ++y) sxy[(size_t)width + y] = (float)((0.25 + (double)y) / (double)height - 0.5);
        if (hipMalloc((void**)&c->cam_sxy, sizeof(float) * sxy.size()) != hipSuccess)
            return cleanup(fail(VRHIP_ERR_NOMEM, "hipMalloc of the camera table failed"));
        if (hipMemcpy(c->cam_sxy, sxy.data(), sizeof(float) * sxy.size(), hipMemcpyHostToDevice) != hipSuccess)
            return cleanup(fail(VRHIP_ERR_HIP, "camera table upload failed"));
    }
    if (hipMemsetAsync(c->rgba, 0, 4 * npx, c->stream) != hipSuccess ||
        hipMemsetAsync(c->depth, 0, 4 * npx, c->stream) != hipSuccess)
        return cleanup(fail(VRHIP_ERR_HIP, "hipMemset failed"));
    if ((rc = clear_accum(c)) != VRHIP_OK) return cleanup(rc);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return cleanup(fail(VRHIP_ERR_HIP, "sync failed"));
    *out = c;
    return VRHIP_OK;
}

int vrhip_destroy(vrhip_ctx* c)
{
    if (!c) return VRHIP_OK;
    if (!c->group.empty()) {                          // a multi-device context: every member, the lead last
        std::vector<vrhip_ctx*> ms;
        ms.swap(c->group);
        for (vrhip_ctx* m : ms) { (void)hipSetDevice(m->device); (void)svc_close(m); if (m->stream) (void)hipStreamSynchronize(m->stream); }
        for (size_t i = ms.size(); i-- > 1;) vrhip_destroy(ms[i]);
    }
    (void)hipSetDevice(c->device);
    (void)svc_close(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    quiesce(c);
    dfree(c->accum); dfree(c->rgba); dfree(c->depth); dfree(c->cam_sxy);
    dfree(c->bvh); dfree(c->bvh16); dfree(c->verts); dfree(c->tri_e); dfree(c->tpath); dfree(c->normals); dfree(c->tangents); dfree(c->uvs);
    dfree(c->hdr); dfree(c->tex[0]); dfree(c->tex[1]); dfree(c->tex[2]); dfree(c->brdf);
    for (int i = 0; i < 2; ++i)
        if (c->gl_res[i]) (void)hipGraphicsUnregisterResource(c->gl_res[i]);
    dfree(c->counters); dfree(c->tone_t);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    dfree(c->comm_send); dfree(c->comm_recv);
    for (auto& l : c->lane) {
        dfree(l.paths); dfree(l.prim); dfree(l.chunk_ctr); dfree(l.px_list);
        for (int i = 0; i < 2; ++i) { dfree(l.sub_cost[i]); dfree(l.sub_order[i]); }
        if (l.done) (void)hipEventDestroy(l.done);
        for (int i = 0; i < 2; ++i)
            if (l.ordered[i]) (void)hipEventDestroy(l.ordered[i]);
        if (l.finished) (void)hipEventDestroy(l.finished);
        if (l.s) (void)hipStreamDestroy(l.s);
    }
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (auto& pr : c->kev_pending) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    svc_free(c);
    for (hipEvent_t e : c->kev_free) (void)hipEventDestroy(e);
    if (c->kev_origin) (void)hipEventDestroy(c->kev_origin);
    for (auto& G : c->fgraph) {
        if (G.x) (void)hipGraphExecDestroy(G.x);
        if (G.g) (void)hipGraphDestroy(G.g);
    }
    if (c->sync_flag) (void)hipHostFree(c->sync_flag);
    dfree(c->sync_ctr);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return VRHIP_OK;
}

int vrhip_set_stream(vrhip_ctx* c, void* s)
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_set_stream");
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    c->stream_shared = true;            // the caller may queue its own work on it: vrhip_sync waits for the stream
    // work queued on the old stream (finish passes) must not reorder with the new one
    if (c->stream && hipSetDevice(c->device) == hipSuccess) {
        (void)svc_close(c);
        (void)hipStreamSynchronize(c->stream);
    }
    quiesce(c);
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return VRHIP_OK;
}

void* vrhip_get_stream(vrhip_ctx* c)
{
    if (!c) return nullptr;
    c->stream_shared = true;            // the caller may queue its own work on it: vrhip_sync waits for the stream
    c->flag_armed = 0;
    return (void*)c->stream;
}

static int one_set_camera(vrhip_ctx* c, const float origin[3], const float dir[3], const float up[3],
                     const float right[3], float fov_scale)
{
    if (!c || !origin || !dir || !up || !right) return fail(VRHIP_ERR_INVALID, "bad camera arguments");
    std::memcpy(c->cam_o, origin, 12); std::memcpy(c->cam_d, dir, 12);
    std::memcpy(c->cam_up, up, 12); std::memcpy(c->cam_right, right, 12);
    c->fov_scale = fov_scale;
    int rc = set_device(c); if (rc) return rc;
    return clear_accum(c);
}

static int one_clear(vrhip_ctx* c)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = set_device(c); if (rc) return rc;
    return clear_accum(c);
}

static int one_set_fresnel(vrhip_ctx* c, float coef, float power)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    c->fresnel_coef = coef; c->fresnel_pow = power;
    return VRHIP_OK;
}

static int one_use_cornell_box(vrhip_ctx* c, int e) { if (!c) return fail(VRHIP_ERR_INVALID, "null ctx"); c->cornell = e != 0; return VRHIP_OK; }
static int one_use_example_sphere(vrhip_ctx* c, int e) { if (!c) return fail(VRHIP_ERR_INVALID, "null ctx"); c->example = e != 0; return VRHIP_OK; }
static int one_set_strict_traversal(vrhip_ctx* c, int e) { if (!c) return fail(VRHIP_ERR_INVALID, "null ctx"); c->strict = e != 0; return VRHIP_OK; }
static int one_use_brdf(vrhip_ctx* c, int e) { if (!c) return fail(VRHIP_ERR_INVALID, "null ctx"); c->view_brdf = e != 0; return VRHIP_OK; }

static int one_upload_mesh_flat(vrhip_ctx* c, const float* bvh, size_t n_bvh_f4, const float* verts,
                           const float* normals, const float* tangents, const float* uvs, size_t n_slots)
{
    if (!c || !bvh || !verts || !normals || !tangents || !uvs) return fail(VRHIP_ERR_INVALID, "null mesh array");
    uint32_t depth = 0, nodes = 0;
    int v = vr::validate_flat(bvh, n_bvh_f4, verts, n_slots, &depth, &nodes);
    if (v != 0) return fail(VRHIP_ERR_BVH, "flattened BVH failed validation (code " + std::to_string(v) + ")");
    if (depth > 62) return fail(VRHIP_ERR_BVH, "BVH deeper than 62 levels");
    DeviceMesh dm;
    std::string why;
    if (!to_device_layout(bvh, n_bvh_f4, (const vr4*)verts, (const vr4*)normals, (const vr4*)tangents,
                          (const vr2*)uvs, dm, why))
        return fail(VRHIP_ERR_BVH, why);
    int rc = set_device(c); if (rc) return rc;
    const size_t nt = dm.tris.size();
    if ((rc = upload(c, c->bvh, dm.nodes.data(), dm.nodes.size() * 16))) return rc;
    if ((rc = upload(c, c->bvh16, dm.nodes16.data(), dm.nodes16.size() * 16))) return rc;
    if ((rc = upload(c, c->verts, dm.tris.data(), nt * sizeof(vr3)))) return rc;
    if ((rc = upload(c, c->tri_e, dm.tri_e.data(), nt * sizeof(vr3)))) return rc;
    if ((rc = upload(c, c->tpath, dm.tpath.data(), dm.tpath.size() * sizeof(unsigned long long)))) return rc;
    if ((rc = upload(c, c->normals, dm.normals.data(), nt * 16))) return rc;
    if ((rc = upload(c, c->tangents, dm.tangents.data(), nt * 16))) return rc;
    if ((rc = upload(c, c->uvs, dm.uvs.data(), nt * 8))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->n_bvh = n_bvh_f4; c->n_slots = n_slots;
    c->bvh_depth = depth; c->bvh_nodes = nodes;
    c->dev_nodes = (uint32_t)(dm.nodes.size() / 4);
    c->dev_tris = (uint32_t)(nt / 3);
    c->mesh = true;
    return VRHIP_OK;
}

int vrhip_upload_mesh_indexed(vrhip_ctx* c, const float* positions, const float* normals, const float* tangents,
                              const float* uvs, uint32_t n_verts, const uint32_t* tris, uint32_t n_tris,
                              uint32_t max_leaf_tris)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    vr::FlatMesh m;
    if (vr::build_flat(positions, normals, tangents, uvs, n_verts, tris, n_tris, max_leaf_tris, m) != 0)
        return fail(VRHIP_ERR_INVALID, "BVH build failed (empty mesh or bad indices)");
    return vrhip_upload_mesh_flat(c, (const float*)m.bvh.data(), m.bvh.size(), (const float*)m.verts.data(),
                                  (const float*)m.normals.data(), (const float*)m.tangents.data(),
                                  (const float*)m.uvs.data(), m.verts.size());
}

#ifndef VR_SERVICE_HDRI_FRAMES
#define VR_SERVICE_HDRI_FRAMES 1
#endif
// whole frames of Cornell-box mesh scenes on the render service too (its
// 7-wave Cornell kernel, r05: C2 4,185 -> 4,313 Mpaths/s at 16 frames per
// step; on the 6-wave kernel of round 4 they lost, 4,111 -> 4,021)
#ifndef VR_SERVICE_CORNELL_FRAMES
#define VR_SERVICE_CORNELL_FRAMES 1
#endif

static int one_upload_hdr(vrhip_ctx* c, const float* rgba, uint32_t w, uint32_t h)
{
    if (!c || !rgba || w == 0 || h == 0) return fail(VRHIP_ERR_INVALID, "bad hdr arguments");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = upload(c, c->hdr, rgba, (size_t)w * h * 16))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->hdr_w = w; c->hdr_h = h;
    return VRHIP_OK;
}

static int one_upload_hdr_half(vrhip_ctx* c, const uint16_t* rgba_half, uint32_t w, uint32_t h)
{
    if (!c || !rgba_half || w == 0 || h == 0) return fail(VRHIP_ERR_INVALID, "bad hdr arguments");
    int rc = set_device(c); if (rc) return rc;
    const size_t n = (size_t)w * h;
    uint16_t* tmp = nullptr;
    HIP_TRY(hipMalloc((void**)&tmp, n * 8));
    quiesce(c);
    dfree(c->hdr);
    if (hipMalloc((void**)&c->hdr, n * 16) != hipSuccess) { dfree(tmp); return fail(VRHIP_ERR_NOMEM, "hdr alloc"); }
    HIP_TRY(hipMemcpyAsync(tmp, rgba_half, n * 8, hipMemcpyHostToDevice, c->stream));
    if (vr::launch_half_to_float(tmp, c->hdr, n, c->stream) != 0) { dfree(tmp); return fail(VRHIP_ERR_HIP, "half convert"); }
    HIP_TRY(hipStreamSynchronize(c->stream));
    dfree(tmp);
    c->hdr_w = w; c->hdr_h = h;
    return VRHIP_OK;
}

static int one_upload_texture(vrhip_ctx* c, int type, const float* rgba, uint32_t w, uint32_t h)
{
    if (!c || !rgba || w == 0 || h == 0 || type < 0 || type > 2) return fail(VRHIP_ERR_INVALID, "bad texture arguments");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = upload(c, c->tex[type], rgba, (size_t)w * h * 16))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->tex_w[type] = w; c->tex_h[type] = h;
    return VRHIP_OK;
}

static int one_upload_brdf(vrhip_ctx* c, const float* table, size_t n_floats)
{
    const size_t n = 90u * 90u * 360u / 2u;    // BRDF_SAMPLING_RES_* (include/vRenderer.h:23-25)
    if (!c || !table || n_floats != 3 * n) return fail(VRHIP_ERR_INVALID, "BRDF table must hold 3*1458000 floats");
    int rc = set_device(c); if (rc) return rc;
    // The device copy is interleaved (entry i's three channels adjacent): one
    // lookup touches one cache line instead of three, 5.8 MB apart.
    std::vector<float> rgb(3 * n);
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) rgb[3 * i + k] = table[k * n + i];
    if ((rc = upload(c, c->brdf, rgb.data(), 3 * n * sizeof(float)))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return VRHIP_OK;
}

int vrhip_load_merl(const char* path, float* table, size_t n_floats)
{
    if (!path || !table || n_floats != vr::kMerlFloats)
        return fail(VRHIP_ERR_INVALID, "BRDF table must hold 3*1458000 floats");
    std::string why;
    if (vr::read_merl(path, table, why) != 0) return fail(VRHIP_ERR_INVALID, why);
    return VRHIP_OK;
}

int vrhip_load_exr(const char* path, uint16_t* rgba_half, size_t n_values, uint32_t* width, uint32_t* height)
{
    if (!path || !width || !height) return fail(VRHIP_ERR_INVALID, "null argument");
    std::vector<uint16_t> px;
    uint32_t w = 0, h = 0;
    std::string why;
    if (vr::read_exr_rgba_half(path, px, w, h, why) != 0) return fail(VRHIP_ERR_INVALID, why);
    *width = w;
    *height = h;
    if (!rgba_half) return VRHIP_OK;                 // size query
    if (n_values < px.size()) return fail(VRHIP_ERR_INVALID, "output too small for 4*w*h half values");
    std::memcpy(rgba_half, px.data(), px.size() * 2);
    return VRHIP_OK;
}

int vrhip_gl_register_image(vrhip_ctx* c, int which, unsigned int gl_texture, unsigned int gl_target)
{
    if (!c || which < 0 || which > 1) return fail(VRHIP_ERR_INVALID, "bad GL registration arguments");
    int rc = set_device(c); if (rc) return rc;
    if (c->gl_res[which]) { HIP_TRY(hipGraphicsUnregisterResource(c->gl_res[which])); c->gl_res[which] = nullptr; }
    const hipError_t e = hipGraphicsGLRegisterImage(&c->gl_res[which], gl_texture, gl_target,
                                                    hipGraphicsRegisterFlagsWriteDiscard);
    if (e != hipSuccess) {
        c->gl_res[which] = nullptr;
        (void)hipGetLastError();        // not sticky: later launches check hipGetLastError
        return fail(VRHIP_ERR_HIP, std::string("hipGraphicsGLRegisterImage: ") + hipGetErrorString(e));
    }
    return VRHIP_OK;
}

int vrhip_gl_present(vrhip_ctx* c)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = multi_images(c); if (rc) return rc;
    if ((rc = set_device(c)) != VRHIP_OK) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    const void* src[2] = { c->rgba, c->depth };
    for (int i = 0; i < 2; ++i) {
        if (!c->gl_res[i]) continue;
        hipArray_t arr = nullptr;
        HIP_TRY(hipGraphicsMapResources(1, &c->gl_res[i], c->stream));
        hipError_t e = hipGraphicsSubResourceGetMappedArray(&arr, c->gl_res[i], 0, 0);
        if (e == hipSuccess)
            e = hipMemcpy2DToArrayAsync(arr, 0, 0, src[i], (size_t)c->W * 4, (size_t)c->W * 4, c->H,
                                        hipMemcpyDeviceToDevice, c->stream);
        const hipError_t u = hipGraphicsUnmapResources(1, &c->gl_res[i], c->stream);
        if (e != hipSuccess) return fail(VRHIP_ERR_HIP, std::string("GL present: ") + hipGetErrorString(e));
        if (u != hipSuccess) return fail(VRHIP_ERR_HIP, std::string("GL unmap: ") + hipGetErrorString(u));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return VRHIP_OK;
}

constexpr int kDebugSlots = vr::kExecCounterBase + vr::kExecCounters;

static int ensure_counters(vrhip_ctx* c)
{
    if (!c->counters) {
        HIP_TRY(hipMalloc((void**)&c->counters, sizeof(unsigned long long) * kDebugSlots));
        HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kDebugSlots, c->stream));
    }
    return VRHIP_OK;
}

// Adds the render-kernel times of completed launches to the totals; with
// `wait`, waits for all of them.  Never blocks otherwise, so a render call
// does not wait for the previous one (launches pipeline, see render_impl).
// Launches on the path streams can overlap and need not start in queue
// order: every span is placed on one time line (ms after kev_origin) and
// the total is the length of the union of the spans, so it never exceeds the
// wall time they cover and is never less than the longest span.
static int account_pending(vrhip_ctx* c, bool wait)
{
    while (!c->kev_pending.empty()) {
        auto pr = c->kev_pending.front();
        if (wait) {
            HIP_TRY(hipEventSynchronize(pr.second));
        } else {
            const hipError_t q = hipEventQuery(pr.second);
            if (q == hipErrorNotReady) break;
            if (q != hipSuccess) return fail(VRHIP_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
        }
        bool keep_start = false;
        if (!c->kev_origin) { c->kev_origin = pr.first; keep_start = true; }
        float t0 = 0.f, t1 = 0.f;
        HIP_TRY(hipEventElapsedTime(&t0, c->kev_origin, pr.first));
        HIP_TRY(hipEventElapsedTime(&t1, c->kev_origin, pr.second));
        if (t1 > t0) {
            // insert [t0, t1) and merge the intervals it touches
            auto& u = c->kev_union;
            double lo = t0, hi = t1;
            std::vector<std::pair<double, double>> out;
            out.reserve(u.size() + 1);
            for (const auto& iv : u) {
                if (iv.second < lo || iv.first > hi) out.push_back(iv);
                else { lo = std::min(lo, iv.first); hi = std::max(hi, iv.second); }
            }
            out.emplace_back(lo, hi);
            std::sort(out.begin(), out.end());
            u.swap(out);
        }
        c->launches_total += pr.launches;
        c->kev_pending.pop_front();
        if (!keep_start) c->kev_free.push_back(pr.first);
        c->kev_free.push_back(pr.second);
    }
    double tot = 0.0;
    for (const auto& iv : c->kev_union) tot += iv.second - iv.first;
    c->kernel_ms_total = tot;
    return VRHIP_OK;
}

static int take_event(vrhip_ctx* c, hipEvent_t* e)
{
    if (!c->kev_free.empty()) { *e = c->kev_free.back(); c->kev_free.pop_back(); return VRHIP_OK; }
    HIP_TRY(hipEventCreate(e));
    return VRHIP_OK;
}

// Path groups per pixel for a sphere-only launch of n_tiles tiles x k frames
// (mesh scenes use the path-pool kernel: no groups).  A thread runs its
// pixel's paths back to back; with one group it accumulates them in registers
// (no result scratch, no finish pass), so one group is the choice whenever
// the launch has blocks enough to fill the GPU, and for one-frame launches
// (2 paths per thread: little imbalance to hide).  Otherwise the paths are
// split into the smallest power of two of groups that gives 16 blocks per CU
// (four resident blocks per CU, four rounds).  Measured (1xMI355X, 16-frame
// steps, scripts/split_sweep.py): C4 (8,040 tiles) split 1 0.634 ms, 2 0.638,
// 4 0.639, 8 0.678; one frame per call 0.089 ms against 0.105-0.145; C1
// (1,024 tiles) split 1 0.434, 2 0.319, 4 0.296, 8 0.299, 16 0.310; one frame
// per call 0.062 (split 1) against 0.068.
// Sphere-only HDRI scenes (C4): path groups per pixel at least this many.
// Their pixels split into camera-ray escapes -- one result for all paths,
// stored once (kSharedMissW) -- and the few on the example sphere, whose 2K
// paths (BRDF lookups, HDRI fetches: dependent gathers) one thread would run
// back to back, the launch's critical path.  C4 at 16 frames per launch
// (r04, scripts/c4_probe.py): 1 group 0.470 ms, 2 0.323, 4 0.246, 8 0.253,
// 16 0.362 (every group recomputes the camera ray and sphere tests).
#ifndef VR_SPHERE_SPLIT
#define VR_SPHERE_SPLIT 4
#endif
// HDRI mesh launches with a primary pass: escaped camera rays' pixels take
// one shared result and leave the path kernel (F_SPARSE; 0: every path runs, A/B builds)
#ifndef VR_SPARSE_HDRI
#define VR_SPARSE_HDRI 1
#endif
static uint32_t choose_split(const vrhip_ctx* c, uint32_t n_tiles, uint32_t k, bool shared_escape)
{
    uint32_t t = c->path_split;
    if (t == 0) {
        const uint32_t target = c->cu_count * 16u;
        t = 1;
        if (k > 1)
            while (n_tiles * t < target && t < 2u * k) t *= 2;
        // (launches of 4 frames or more: one frame per call keeps its 2 paths
        // in one thread -- direct accumulation, no finish pass: C4 0.084 ms
        // per frame against 0.093 with 2 groups)
        if (shared_escape && k >= 4) t = std::max<uint32_t>(t, VR_SPHERE_SPLIT);
    }
    return std::max<uint32_t>(1u, std::min<uint32_t>(t, 2u * k));
}

// Entries per XCD in a longest-first order list: the most sub-tiles one XCD's
// bands (VR_XCD_BANDS sub-tiles each, dealt round-robin to 8 XCDs) can hold.
#ifndef VR_XCD_BANDS
#define VR_XCD_BANDS 128
#endif
static size_t order_cap(size_t n_sub) { return (n_sub / (8u * VR_XCD_BANDS) + 1u) * VR_XCD_BANDS; }

// Scratch of one path stream, allocated when the stream is first used and
// grown when a launch needs more (growing waits for every reader first).
static int ensure_lane(vrhip_ctx* c, vrhip_ctx::Lane& l, size_t need, uint32_t path_stride)
{
    const size_t prim_need = 2 * (size_t)path_stride;
    if ((l.paths && need > l.paths_cap) || (l.prim && prim_need > l.prim_cap)) {
        quiesce(c);                                       // the finish passes read the scratch too
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (need > l.paths_cap) {
        dfree(l.paths);
        l.paths_cap = 0;
        HIP_TRY(hipMalloc((void**)&l.paths, need * sizeof(vr4)));
        l.paths_cap = need;
    }
    if (prim_need > l.prim_cap) {
        dfree(l.prim);
        l.prim_cap = 0;
        HIP_TRY(hipMalloc((void**)&l.prim, prim_need * sizeof(vr4)));
        l.prim_cap = prim_need;
    }
    const size_t n_sub = path_stride / 64u;
    if (path_stride > l.px_cap) {                         // the F_SPARSE pixel list: one word per owned pixel
        dfree(l.px_list);
        l.px_cap = 0;
        HIP_TRY(hipMalloc((void**)&l.px_list, (size_t)path_stride * sizeof(uint32_t)));
        l.px_cap = path_stride;
    }
    if (n_sub > l.sub_cap) {                              // the order buffers hold 8 XCD lists of order_cap(n_sub)
        l.sub_cap = 0;
        for (int i = 0; i < 2; ++i) {
            dfree(l.sub_cost[i]); dfree(l.sub_order[i]);
            l.order_nsub[i] = 0;
            HIP_TRY(hipMalloc((void**)&l.sub_cost[i], n_sub * sizeof(uint32_t)));
            HIP_TRY(hipMalloc((void**)&l.sub_order[i], 8u * order_cap(n_sub) * sizeof(uint32_t)));
        }
        l.sub_cap = n_sub;
    }
    if (!l.chunk_ctr) {
        const size_t bytes = sizeof(uint32_t) * vr::kQueueStride * (VR_MAX_QUEUES + 1);   // heads + drained-queue mask
        HIP_TRY(hipMalloc((void**)&l.chunk_ctr, bytes));
        HIP_TRY(hipMemsetAsync(l.chunk_ctr, 0, bytes, c->stream));

        HIP_TRY(hipEventRecord(c->ev_join, c->stream));
        HIP_TRY(hipStreamWaitEvent(l.s, c->ev_join, 0));
    }
    return VRHIP_OK;
}


// ---- render service sessions ------------------------------------------------
// Back-to-back render calls on mesh scenes (vrhip_set_service: automatically
// behind a launch still in flight for the launches that overlap on the path
// streams -- shards and small frames -- or always) post their launches to
// ONE persistent kernel (vr_kernel.hpp service_body) through a descriptor
// ring in host-pinned memory, so a launch's drain overlaps the next launch's
// paths.  Each launch writes its paths' results to its own scratch slot; when
// the session closes -- at the next call that is not a render (sync, read-back,
// upload, any setting or buffer access: svc_close), when its slots are full,
// or when a launch does not fit the session -- one finish pass sums every
// pixel's paths launch by launch in path order, stages the images of
// launches whose gather was deferred (vrhip_comm_gather inside a session),
// and the gathers run.  Results are bit-identical to launch-by-launch
// rendering; only their time of arrival changes.
#ifndef VR_SVC_IDLE_MS
#define VR_SVC_IDLE_MS 20            // the kernel retires after this long without a new launch
#endif
#ifndef VR_SVC_POST_MS
#define VR_SVC_POST_MS 5             // the host posts to a session only within this of its last post
#endif

static void svc_free(vrhip_ctx* c)
{
    auto& S = c->svc;
    if (S.s) (void)hipStreamSynchronize(S.s);
    for (int i = 0; i < 2; ++i) {
        if (S.rings[i]) (void)hipHostFree(S.rings[i]);
        if (S.ring_done[i]) (void)hipEventDestroy(S.ring_done[i]);
        S.rings[i] = S.rings_dev[i] = nullptr;
        S.ring_done[i] = nullptr;
        S.ring_used[i] = false;
    }
    S.host = nullptr;
    dfree(S.dev); dfree(S.qctl); dfree(S.scratch); dfree(S.prim); dfree(S.staging); dfree(S.subs);
    S.qctl_slots = S.scratch_cap = S.prim_cap = S.staging_cap = S.subs_cap = 0;
    if (S.k0) (void)hipEventDestroy(S.k0);
    if (S.k1) (void)hipEventDestroy(S.k1);
    if (S.finished) (void)hipEventDestroy(S.finished);
    if (S.summed) (void)hipEventDestroy(S.summed);
    if (S.s) (void)hipStreamDestroy(S.s);
    S.k0 = S.k1 = S.finished = S.summed = nullptr;
    S.summed_valid = false;
    S.s = nullptr;
    S.open = false;
}

// The launch parameters that must stay fixed within a session (scene,
// camera, flags, tiling, frame buffers): per-launch fields cleared.
static vr::RenderParams svc_key(const vr::RenderParams& p)
{
    vr::RenderParams k = p;
    k.first_frame = k.n_frames = 0;
    std::memset(k.times, 0, sizeof(k.times));
    k.split = k.use_scratch = k.small_blocks = k.inline_prim = 0;
    k.paths = nullptr; k.path_w = nullptr; k.prim = nullptr; k.chunk_ctr = nullptr;
    k.path_cost = nullptr; k.sub_cost = nullptr; k.sub_order = nullptr; k.order_cap = 0;
    k.counters = nullptr; k.n_queues = 0;
    return k;
}

// Launch slots a session of launches of up to kmax frames gets (0 or 1:
// the service cannot take such launches; they take the launch path).  The
// scratch budget (VRHIP_SERVICE_BYTES, default 24 GiB of the 288 GiB HBM)
// holds every slot's path results: 24 B per pixel and frame.
static uint32_t svc_slots(const vrhip_ctx* c, uint32_t path_stride, uint32_t kmax, size_t* slot_bytes_out)
{
    const size_t stride = path_stride;
    const size_t slot_bytes = ((12u * 2u * (size_t)kmax * stride + 4u * stride) + 255u) & ~(size_t)255u;
    static const size_t env_budget = [] {
        const char* e = std::getenv("VRHIP_SERVICE_BYTES");
        return e ? (size_t)std::atoll(e) : ((size_t)24 << 30);
    }();
    const size_t budget = c->svc_budget ? c->svc_budget : env_budget;
    if (slot_bytes_out) *slot_bytes_out = slot_bytes;
    return (uint32_t)std::min<size_t>(vr::kSvcMaxLaunches, budget / slot_bytes);
}

// The kernel of ring ri's last session has finished: it must have consumed
// every launch the session's finish pass summed (svc_post's hand-shake makes
// that so; this check makes any breach loud instead of a silently wrong image).
static int svc_check_ring(vrhip_ctx* c, uint32_t ri)
{
    auto& S = c->svc;
    if (!S.ring_used[ri] || S.ring_checked[ri] || (S.open && S.cur_ring == ri)) return VRHIP_OK;
    HIP_TRY(hipEventSynchronize(S.ring_done[ri]));
    S.ring_checked[ri] = true;
    const uint32_t r = __atomic_load_n(&S.rings[ri]->retired, __ATOMIC_ACQUIRE);
    if ((r & vr::kSvcClosed) == 0u || (r & ~vr::kSvcClosed) < S.ring_posted[ri])
        return fail(VRHIP_ERR_HIP, "render service: the kernel consumed " + std::to_string(r & ~vr::kSvcClosed) +
                                       " of " + std::to_string(S.ring_posted[ri]) + " launches");
    return VRHIP_OK;
}
// after a host synchronisation: both rings' finished sessions
static int svc_verify(vrhip_ctx* c)
{
    int rc;
    for (uint32_t ri = 0; ri < 2; ++ri)
        if ((rc = svc_check_ring(c, ri)) != VRHIP_OK) return rc;
    return VRHIP_OK;
}

// Closes the open session: the kernel retires once the ring is drained, then
// the finish pass and the deferred gathers run on `stream`.  Asynchronous.
static int svc_close(vrhip_ctx* c)
{
    auto& S = c->svc;
    c->flag_armed = 0;                  // every call that queues work closes the session first
    if (!S.open) return VRHIP_OK;
    S.open = false;
    __atomic_store_n(&S.host->closed, 1u, __ATOMIC_RELEASE);
    S.ring_posted[S.cur_ring] = S.posted;
    S.ring_checked[S.cur_ring] = false;
    HIP_TRY(hipStreamWaitEvent(c->stream, S.k1, 0));
    // the launches the host posted and the kernel took (svc_post): a launch
    // that met a retiring kernel was not counted and went the launch path.
    // A session that took none has nothing to sum: no finish pass (on a fresh
    // accumulation it would tonemap with a frame count of 0) and no gathers
    // (a gather is deferred only behind a launch the session took)
    S.fin.n = S.posted;
    if (S.posted > 0) {
        const int e = vr::launch_service_finish(S.p, S.fin, S.n_tiles, c->stream);
        if (e != 0) return fail(VRHIP_ERR_HIP, std::string("service finish launch: ") + hipGetErrorString((hipError_t)e));
    }
    if (!S.gathers.empty()) {
        HIP_TRY(hipEventRecord(S.summed, c->stream));
        S.summed_epoch = c->stream_epoch;
        S.summed_valid = true;
    }
    // deferred gathers, in call order; rank 0 keeps its own tiles from the
    // finish pass (the final state) and unpacks the other ranks' of every gather
    for (const auto& g : S.gathers) {
        const int what = g.second;
        const size_t esz = what == 1 ? 16u : 4u;
        const size_t off = what == 0 ? 0u : what == 2 ? 4u * (size_t)S.fin.stage_pixels : 8u * (size_t)S.fin.stage_pixels;
        const uint8_t* send = S.staging + (size_t)g.first * S.fin.stage_bytes + off;
        const size_t bytes = (size_t)S.fin.stage_pixels * esz;
        const ncclResult_t r = ncclGather(send, c->comm_recv, bytes, ncclUint8, 0, c->comm, c->stream);
        if (r != ncclSuccess) return fail(VRHIP_ERR_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
        if (c->rank == 0 && c->nranks > 1) {
            void* dst = what == 1 ? (void*)c->accum : what == 2 ? (void*)c->depth : (void*)c->rgba;
            const int ee = vr::launch_unpack_ranks(c->comm_recv + bytes, dst, (uint32_t)esz, c->W, c->W / 16u,
                                                   (c->W / 16u) * (c->H / 16u), 1u, c->nranks, bytes, c->stream);
            if (ee) return fail(VRHIP_ERR_HIP, "unpack launch failed");
        }
    }
    S.gathers.clear();
    HIP_TRY(hipEventRecord(S.finished, c->stream));
    S.finished_used = true;
    // vrhip_last_kernel_ms after a session: its span, kernel start to finish pass
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->flag_synced = false;
    // the session's kernel span: one span covering all its launches
    hipEvent_t a = nullptr, b = nullptr;
    if ((a = S.k0) && (b = S.k1)) {
        S.k0 = S.k1 = nullptr;
        c->kev_pending.push_back({ a, b, S.posted });
    }
    return VRHIP_OK;
}

// Opens a session for launches of up to kmax frames with parameters p.
static int svc_open(vrhip_ctx* c, const vr::RenderParams& p, int stack, uint32_t n_tiles, uint32_t kmax)
{
    auto& S = c->svc;
    if (!S.s) {
        HIP_TRY(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&S.finished, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&S.summed, hipEventDisableTiming));
        for (int i = 0; i < 2; ++i) {
            HIP_TRY(hipHostMalloc((void**)&S.rings[i], sizeof(vr::SvcHostCtl), hipHostMallocCoherent | hipHostMallocMapped));
            HIP_TRY(hipHostGetDevicePointer((void**)&S.rings_dev[i], S.rings[i], 0));
            HIP_TRY(hipEventCreateWithFlags(&S.ring_done[i], hipEventDisableTiming));
        }
        HIP_TRY(hipMalloc((void**)&S.dev, sizeof(vr::SvcDevCtl)));
    }
    // this session's ring: the other one's kernel may still run; this one's
    // kernel (two sessions back) must have retired before the host rewrites it
    const uint32_t ri = S.ring_i;
    S.ring_i ^= 1u;
    int rc;
    if (S.ring_used[ri]) {
        HIP_TRY(hipEventSynchronize(S.ring_done[ri]));
        if ((rc = svc_check_ring(c, ri)) != VRHIP_OK) return rc;
    }
    const size_t stride = p.path_stride;
    size_t slot_bytes = 0;
    uint32_t slots = svc_slots(c, p.path_stride, kmax, &slot_bytes);
    const uint32_t stage_px = owned_tiles_of(c->W, c->H, 0, c->nranks) * 256u;   // rank 0 owns the most tiles
    // staged images serve deferred gathers only, which need a communicator
    // (vrhip_comm_init closes any open session, so none appears mid-session)
    const size_t stage_bytes = c->comm ? (24u * (size_t)stage_px + 255u) & ~(size_t)255u : 0u;
    // the slots' scratch grows into at most half of the device memory free
    // now (plus what the session already holds): several contexts or ranks
    // on one GPU share it, and the launch path needs its own scratch
    if (slots >= 2 && (size_t)slots * slot_bytes > S.scratch_cap) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const size_t avail = (free_b + S.scratch_cap + S.staging_cap) / 2u;
            slots = (uint32_t)std::min<size_t>(slots, avail / (slot_bytes + stage_bytes));
        }
        (void)hipGetLastError();
    }
    if (slots < 2) return fail(VRHIP_ERR_NOMEM, "render service: device memory holds fewer than 2 launch slots");
    auto grow = [&](auto*& ptr, size_t& cap, size_t need) -> int {
        if (need <= cap) return VRHIP_OK;
        // the previous session's kernel and finish pass may still use the old buffer
        if (S.s) HIP_TRY(hipStreamSynchronize(S.s));
        if (S.finished_used) HIP_TRY(hipEventSynchronize(S.finished));
        dfree(ptr);
        cap = 0;
        const hipError_t e = hipMalloc((void**)&ptr, need);
        if (e != hipSuccess) {
            ptr = nullptr;
            (void)hipGetLastError();
            return fail(VRHIP_ERR_NOMEM, std::string("render service scratch: ") + hipGetErrorString(e));
        }
        cap = need;
        return VRHIP_OK;
    };
    if ((rc = grow(S.scratch, S.scratch_cap, (size_t)slots * slot_bytes)) != VRHIP_OK) return rc;
    if ((rc = grow(S.prim, S.prim_cap, 32u * stride)) != VRHIP_OK) return rc;
    if (stage_bytes && (rc = grow(S.staging, S.staging_cap, (size_t)slots * stage_bytes)) != VRHIP_OK) return rc;
    if ((rc = grow(S.qctl, S.qctl_slots, (size_t)slots * vr::kSvcQctlWords * 4u)) != VRHIP_OK) return rc;
    // HDRI scenes: escaped camera rays' pixels leave the session's paths (F_SPARSE)
    const bool sparse = VR_SPARSE_HDRI != 0 && !c->cornell && (p.flags & vr::F_STRICT) == 0u;
    if (sparse && (rc = grow(S.subs, S.subs_cap, 4u * stride)) != VRHIP_OK) return rc;
    if (!S.k0 && (rc = take_event(c, &S.k0)) != VRHIP_OK) return rc;
    if (!S.k1 && (rc = take_event(c, &S.k1)) != VRHIP_OK) return rc;
    S.slot_bytes = slot_bytes; S.slots = slots; S.kmax = kmax; S.posted = 0;
    S.stack = stack; S.n_tiles = n_tiles;
    S.p = p;
    S.p.paths = reinterpret_cast<vr3*>(S.scratch);
    S.p.prim = S.prim;
    S.p.sparse_px = sparse ? S.subs : nullptr;
    S.host = S.rings[ri];
    S.cur_ring = ri;
    S.p.svc_host = S.rings_dev[ri]; S.p.svc_dev = S.dev; S.p.svc_qctl = S.qctl;
    S.p.svc_slot_bytes = slot_bytes; S.p.svc_kmax = kmax;
    S.p.svc_idle_ticks = (c->svc_idle_us ? c->svc_idle_us : (uint32_t)VR_SVC_IDLE_MS * 1000u) * 100u;   // 100 MHz
    S.key = svc_key(p);
    std::memset(&S.fin, 0, sizeof(S.fin));
    S.fin.first_frame = c->frame;
    S.fin.staging = stage_bytes ? S.staging : nullptr; S.fin.stage_bytes = stage_bytes; S.fin.stage_pixels = stage_px;
    S.gathers.clear();
    // the ring: nothing posted, open, the kernel serving (the kernel launch
    // below orders these host stores before the kernel's first read)
    S.host->posted = 0; S.host->closed = 0; S.host->retired = 0;
    // everything queued on `stream` first (uploads, clears, earlier finish
    // passes) -- or, when the last thing queued there that this session's
    // kernels depend on is the previous session's finish pass (its scratch,
    // primary records and pixel list are reused here), only that: its
    // deferred gathers then run beside this session (Session::summed)
    if (S.summed_valid && S.summed_epoch == c->stream_epoch) {
        HIP_TRY(hipStreamWaitEvent(S.s, S.summed, 0));
    } else {
        HIP_TRY(hipEventRecord(c->ev_join, c->stream));
        HIP_TRY(hipStreamWaitEvent(S.s, c->ev_join, 0));
    }
    S.summed_valid = false;
    HIP_TRY(hipMemsetAsync(S.dev, 0, sizeof(vr::SvcDevCtl), S.s));
    HIP_TRY(hipMemsetAsync(S.qctl, 0, (size_t)slots * vr::kSvcQctlWords * 4u, S.s));
    HIP_TRY(hipEventRecord(S.k0, S.s));
    HIP_TRY(hipEventRecord(c->ev0, S.s));
    c->ev0_valid = true;
    const int e = vr::launch_service(S.p, n_tiles, stack, S.s);
    if (e != 0) return fail(VRHIP_ERR_HIP, std::string("service launch: ") + hipGetErrorString((hipError_t)e));
    HIP_TRY(hipEventRecord(S.k1, S.s));
    HIP_TRY(hipEventRecord(S.ring_done[ri], S.s));
    S.ring_used[ri] = true;
    S.ring_checked[ri] = false;
    S.ring_posted[ri] = 0;
    S.open = true;
    ++c->svc_sessions;
    S.last_post = std::chrono::steady_clock::now();
    return VRHIP_OK;
}

// Posts one launch of k frames (first frame c->frame) to the open session.
// false: the session's kernel was retiring (idle) and did not take it -- the
// caller closes the session without it and renders it another way.  The
// hand-shake with svc_ring_wave: the host stores `posted`, fences, reads
// `retired`; the kernel stores `retired`, fences, reads `posted`.  Whichever
// store is first, the other side's load sees it, so the launch is taken by
// the kernel (it saw `posted`) or by the caller (it saw `retired`) -- never
// by neither.
static bool svc_post(vrhip_ctx* c, uint32_t k, const uint32_t* times, uint32_t time_seed)
{
    auto& S = c->svc;
    vr::SvcLaunch& d = S.host->desc[S.posted];
    d.first_frame = c->frame;
    d.n_frames = k;
    for (uint32_t i = 0; i < k; ++i) d.times[i] = times ? times[i] : time_seed;
    __atomic_store_n(&S.host->posted, S.posted + 1u, __ATOMIC_SEQ_CST);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    if (__atomic_load_n(&S.host->retired, __ATOMIC_SEQ_CST) != 0u) return false;
    S.fin.n_frames[S.posted] = k;
    ++S.posted;
    ++c->svc_served;
    S.last_post = std::chrono::steady_clock::now();
    return true;
}

// Whether the open session can take a launch of k frames with parameters p.
static bool svc_fits(const vrhip_ctx* c, const vr::RenderParams& p, uint32_t k)
{
    const auto& S = c->svc;
    if (!S.open || S.posted >= S.slots || k > S.kmax) return false;
    const auto idle = std::chrono::steady_clock::now() - S.last_post;
    const uint32_t window_us = c->svc_window_us ? c->svc_window_us : (uint32_t)VR_SVC_POST_MS * 1000u;
    if (idle > std::chrono::microseconds(window_us)) return false;
    const vr::RenderParams key = svc_key(p);
    return std::memcmp(&key, &S.key, sizeof(key)) == 0;
}

// One-frame launches as a HIP graph (VRHIP_GRAPH=1, experiment): the path
// kernel and the finish pass of a synchronous one-frame call, captured from
// the context stream once per longest-first order slot (the slots' order and
// cost buffers differ), re-captured when any launch parameter but the
// frame's number and seed changes, and launched with those two kernel nodes'
// arguments updated -- one graph launch instead of two kernel launches
// between the host's wake-up and the next frame's path kernel.
static int one_frame_graph(vrhip_ctx* c, const vr::RenderParams& p, uint32_t n_tiles, int stack, uint32_t gi)
{
    auto& G = c->fgraph[gi];
    vr::RenderParams key = p;
    key.first_frame = 0;
    std::memset(key.times, 0, sizeof(key.times));
    if (!G.valid || std::memcmp(&key, &G.key, sizeof(key)) != 0) {
        if (G.x) { (void)hipGraphExecDestroy(G.x); G.x = nullptr; }
        if (G.g) { (void)hipGraphDestroy(G.g); G.g = nullptr; }
        G.valid = false;
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        const int e1 = vr::launch_render(p, n_tiles, stack, 0, c->stream);
        const int e2 = vr::launch_finish(p, n_tiles, c->stream);
        const hipError_t ec = hipStreamEndCapture(c->stream, &G.g);
        if (e1 || e2 || ec != hipSuccess)
            return fail(VRHIP_ERR_HIP, std::string("one-frame graph capture: ") +
                                           hipGetErrorString(ec != hipSuccess ? ec : (hipError_t)(e1 ? e1 : e2)));
        size_t n = 0;
        HIP_TRY(hipGraphGetNodes(G.g, nullptr, &n));
        std::vector<hipGraphNode_t> nodes(n);
        HIP_TRY(hipGraphGetNodes(G.g, nodes.data(), &n));
        int k = 0;
        for (size_t i = 0; i < n; ++i) {
            hipGraphNodeType t;
            HIP_TRY(hipGraphNodeGetType(nodes[i], &t));
            if (t != hipGraphNodeTypeKernel) continue;
            if (k == 2) return fail(VRHIP_ERR_HIP, "one-frame graph: more than two kernel nodes");
            G.kn[k] = nodes[i];
            HIP_TRY(hipGraphKernelNodeGetParams(nodes[i], &G.kp[k]));
            ++k;
        }
        if (k != 2) return fail(VRHIP_ERR_HIP, "one-frame graph: expected the path kernel and the finish pass");
        HIP_TRY(hipGraphInstantiate(&G.x, G.g, nullptr, nullptr, 0));
        G.key = key;
        G.valid = true;
        ++c->graph_captures;
    }
    G.arg = p;
    void* args[1] = { &G.arg };
    for (int k = 0; k < 2; ++k) {
        hipKernelNodeParams kp = G.kp[k];
        kp.kernelParams = args;
        kp.extra = nullptr;
        HIP_TRY(hipGraphExecKernelNodeSetParams(G.x, G.kn[k], &kp));
    }
    HIP_TRY(hipGraphLaunch(G.x, c->stream));
    ++c->graph_launches;
    return VRHIP_OK;
}

// count: 0 production, 1 reference-algorithm counting variant (in place, no
// scratch), 2 instrumented production kernels (same launch shape as 0)
static int render_impl(vrhip_ctx* c, uint32_t n_frames, const uint32_t* times, uint32_t time_seed, int count)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    if (n_frames == 0) return VRHIP_OK;
    if (!c->cornell && !c->hdr)
        return fail(VRHIP_ERR_NO_ENV, "HDRI mode needs an environment map (vrhip_upload_hdr)");
    int rc = set_device(c); if (rc) return rc;
    c->flag_armed = 0;
    vr::RenderParams p;
    std::memset(&p, 0, sizeof(p));
    p.cam_o = vr4{ c->cam_o[0], c->cam_o[1], c->cam_o[2], 0.f };
    p.cam_d = vr4{ c->cam_d[0], c->cam_d[1], c->cam_d[2], 0.f };
    // PathTracer.cu:833-836 in the same fp32 operation order
    const float sx = c->fov_scale * (float)c->W / (float)c->H;
    p.cx = vr4{ sx * c->cam_right[0], sx * c->cam_right[1], sx * c->cam_right[2], 0.f };
    p.cy = vr4{ c->fov_scale * c->cam_up[0], c->fov_scale * c->cam_up[1], c->fov_scale * c->cam_up[2], 0.f };
    p.W = c->W; p.H = c->H;
    p.cam_sxy = c->cam_sxy;
    p.tone_t = c->tone_t;
    p.wr = (c->W / 16u) * 16u; p.hr = rendered_rows(c);
    p.fresnel_coef = c->fresnel_coef; p.fresnel_pow = c->fresnel_pow;
    uint32_t f = 0;
    if (c->cornell) f |= vr::F_CORNELL;
    if (c->example) f |= vr::F_EXAMPLE;
    if (c->view_brdf) f |= vr::F_VIEW_BRDF;
    if (c->strict) f |= vr::F_STRICT;
    // the reference skips the mesh while the example sphere is on
    // (PathTracer.cu:192,268): a sphere scene, whatever mesh is loaded
    if (c->mesh && !c->example) f |= vr::F_MESH;
    if (c->brdf) f |= vr::F_BRDF;
    if (c->tex[0]) f |= vr::F_TEX_DIFF;
    if (c->tex[1]) f |= vr::F_TEX_NORM;
    if (c->tex[2]) f |= vr::F_TEX_SPEC;
    p.flags = f;
    p.tiles_x = p.wr / 16u;
    p.rank = c->rank; p.nranks = c->nranks;
    p.bvh = c->bvh; p.bvh16 = c->bvh16; p.n_nodes = c->mesh ? c->dev_nodes : 0; p.verts = c->verts; p.tri_e = c->tri_e; p.tpath = c->tpath; p.n_tris = c->mesh ? c->dev_tris : 0; p.normals = c->normals; p.tangents = c->tangents; p.uvs = c->uvs;
    p.hdr = c->hdr; p.hdr_w = c->hdr_w; p.hdr_h = c->hdr_h;
    for (int i = 0; i < 3; ++i) { p.tex[i] = c->tex[i]; p.tex_w[i] = c->tex_w[i]; p.tex_h[i] = c->tex_h[i]; }
    p.brdf = c->brdf;
    p.accum = c->accum; p.rgba = c->rgba; p.depth = c->depth;
    const uint32_t n_tiles = owned_tiles_of(c->W, c->H, c->rank, c->nranks);
    // stack entries needed: walk depth + 1
    const int stack = c->bvh_depth <= 15 ? 16 : c->bvh_depth <= 23 ? 24 : c->bvh_depth <= 30 ? 32 : 64;
    if (count) {
        if ((rc = ensure_counters(c)) != VRHIP_OK) return rc;
        HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kDebugSlots, c->stream));
        p.counters = c->counters;
    }
    const uint32_t k_max = std::min<uint32_t>(n_frames, (uint32_t)vr::kMaxFramesPerLaunch);
    // sphere-only HDRI scenes: camera-ray escapes share one result (render_kernel)
    const bool shared_escape = (f & (vr::F_MESH | vr::F_CORNELL)) == 0u;
    const uint32_t split_max = count == 1 ? 1u : choose_split(c, n_tiles, k_max, shared_escape);
    p.path_stride = n_tiles * (uint32_t)vr::kBlockThreads;
    const size_t need = (size_t)2 * k_max * p.path_stride;   // scratch float4s of the largest launch
    // the path-pool kernel is persistent: one resident set of blocks per CU
    // (the launcher sizes it from the kernel's occupancy) draining the work queues
    p.wave_blocks = c->cu_count;
    // VRHIP_WAVES_PER_SIMD: cap the path kernel's resident waves (experiments)
    static const uint32_t env_waves = [] {
        const char* e = std::getenv("VRHIP_WAVES_PER_SIMD");
        return e ? (uint32_t)std::atoi(e) : 0u;
    }();
    p.waves_cap = env_waves;
    const bool wave_kernel = (f & vr::F_MESH) != 0u;   // mesh scenes: the path-pool kernel (scratch + finish pass)
    (void)hipGetLastError();            // launches below report their own errors only
    // counting launches and anything else than a production mesh launch end a session first
    uint32_t done = 0;                  // frames rendered by the service below (the launch path takes the rest)
    {
        const size_t paths_k = (size_t)p.path_stride * 2u * k_max;
        const bool ovl_size = paths_k < ((size_t)1 << 24) || (c->nranks > 1 && paths_k < ((size_t)1 << 25));
        const bool in_flight = c->svc.open || (c->timed && !c->flag_synced && hipEventQuery(c->ev1) == hipErrorNotReady);
        // whole frames take the service too: back-to-back launches then
        // overlap each other's drain and share one primary pass (r04 A/B,
        // 16-frame steps, bit-identical: C3 16,505 -> 18,948, C5 21,630 ->
        // 22,171 Mpaths/s; r05, the 7-wave Cornell service kernel: C2 4,185
        // -> 4,313)
        // (Cornell-box scenes with material features run a feature-class
        // service kernel at 6 waves: C2D's whole frames 3,710 -> 3,687 on it,
        // so they keep the launch path)
        const bool c2_exact = f == (vr::F_CORNELL | vr::F_MESH);
        const bool svc_size = ovl_size || (c->cornell ? (VR_SERVICE_CORNELL_FRAMES != 0 && c2_exact)
                                                      : VR_SERVICE_HDRI_FRAMES != 0);
        // launches whose slots the scratch budget cannot hold twice take the
        // launch path in every mode (4K frames of many frames per launch)
        const bool svc = count == 0 && wave_kernel && stack <= 32 && n_tiles > 0 &&
                         (c->service > 0 || (c->service < 0 && svc_size && in_flight && c->overlap != 0)) &&
                         svc_slots(c, p.path_stride, k_max, nullptr) >= 2u;
        if (!svc) {
            if ((rc = svc_close(c)) != VRHIP_OK) return rc;
        } else {
            p.n_queues = c->cornell ? VR_QUEUES : VR_QUEUES_HDRI;
            static const uint32_t env_q = [] {
                const char* e = std::getenv("VRHIP_QUEUES");
                const uint32_t q = e ? (uint32_t)std::atoi(e) : 0u;
                return (q >= 8 && q <= (uint32_t)VR_MAX_QUEUES && (q & (q - 1)) == 0) ? q : 0u;
            }();
            if (env_q) p.n_queues = env_q;
            bool refused = false;
            while (done < n_frames) {
                const uint32_t k = std::min<uint32_t>(n_frames - done, (uint32_t)vr::kMaxFramesPerLaunch);
                if (c->svc.open && !svc_fits(c, p, k) && (rc = svc_close(c)) != VRHIP_OK) return rc;
                if (!c->svc.open && (rc = svc_open(c, p, stack, n_tiles, k_max)) != VRHIP_OK) {
                    // no scratch for the session's slots (memory shared with
                    // other contexts or ranks): this call's remaining frames
                    // take the launch path, which needs one launch's scratch
                    if (rc != VRHIP_ERR_NOMEM) return rc;
                    ++c->svc_alloc_fallbacks;
                    refused = true;
                    break;
                }
                // (the test hook's delay: only before posts after a session's
                // first -- the first post meets a kernel that just started)
                if (c->svc_post_delay_us && c->svc.posted > 0)
                    std::this_thread::sleep_for(std::chrono::microseconds(c->svc_post_delay_us));
                if (!svc_post(c, k, times ? times + done : nullptr, time_seed)) {
                    // the session's kernel retired as this launch was posted:
                    // close the session without it; this call's remaining
                    // frames take the launch path below
                    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
                    refused = true;
                    ++c->svc_refused;
                    break;
                }
                c->frame += k;
                done += k;
            }
            if (!refused) {
                c->last_split = 1; c->last_use_scratch = 1; c->last_kind = 2;
                return VRHIP_OK;
            }
        }
    }
    if (c->kernel_timing) HIP_TRY(hipEventRecord(c->ev0, c->stream));
    c->ev0_valid = c->kernel_timing;
    while (done < n_frames) {
        const uint32_t k = std::min<uint32_t>(n_frames - done, (uint32_t)vr::kMaxFramesPerLaunch);
        p.first_frame = c->frame;
        p.n_frames = k;
        p.split = std::min<uint32_t>(split_max, 2u * k);
        // the reference counting variant, and sphere-only launches whose
        // pixels run all their paths in one thread (split 1), accumulate in
        // registers in path order (render_kernel's direct mode): no scratch
        // round trip, no finish pass
        p.use_scratch = (count == 1 || (!wave_kernel && p.split == 1u)) ? 0u : 1u;
        for (uint32_t i = 0; i < k; ++i) p.times[i] = times ? times[done + i] : time_seed;
        // Path launches take the VR_PATH_STREAMS path streams in turn: launch
        // i's render kernels wait only for the finish pass of launch i - 3
        // (the last reader of the same scratch), so they start while launch
        // i-1 drains its longest paths -- and are not held up by launch i-1's
        // finish pass, which itself waits for CUs until that drain.  The
        // finish passes run in order on `stream`.  The counting variant
        // accumulates in place on `stream`.
        // Without overlap every launch uses the same path stream, so it waits
        // for the previous one (and its finish pass, below) like a single stream.
        const bool small = (size_t)p.path_stride * 2u * k < ((size_t)1 << 24);
        // automatic overlap only behind a launch still in flight (this call's
        // previous launch, or the last call's): a launch submitted to an idle
        // device (one frame per synchronous call) runs its render and finish
        // kernels on `stream` with no cross-stream waits
        const bool in_flight = done > 0 || (c->timed && !c->flag_synced && hipEventQuery(c->ev1) == hipErrorNotReady);
        // counting launches never overlap: their counters are zeroed on
        // `stream` (above), which a path stream would not wait for
        // automatic overlap for launches under 2^24 paths, and under 2^25 for
        // a rank's shard (C5's 8-way shards of 33 M paths: 8-rank projection
        // 0.757 -> 0.78 of linear); whole 720p frames of 29.5 M paths lose
        // with it (C2 -1.7 %, C3 -6 %: two persistent launches contend), as
        // do C5's 66 M-path 4-way shards (-17 %); sphere scenes (render_kernel,
        // no path pool) overlap up to 2^27 paths: C4's 66 M-path launches
        // 299 -> 481 G paths/s (r04; C3 -6 %, C5 -14 % forced, so meshes keep
        // the limit) -- one launch's tail and finish pass run under the next
        const size_t paths_k = (size_t)p.path_stride * 2u * k;
        const bool ovl_size = paths_k < ((size_t)1 << 24) || (c->nranks > 1 && paths_k < ((size_t)1 << 25)) ||
                              (!wave_kernel && paths_k < ((size_t)1 << 27));
        const bool ovl = count == 0 && (c->overlap > 0 || (c->overlap < 0 && ovl_size && in_flight));
        p.small_blocks = small ? 1u : 0u;
        // (owned pixels < 2^31: the textured one-frame kernels pack the path
        // index into the pixel slot, vr_kernel.hpp wave_body)
        p.inline_prim = (2u * k <= (uint32_t)VR_INLINE_PRIM_PATHS && count != 1 && p.path_stride < (1u << 31)) ? 1u : 0u;
        // HDRI mesh launches with a primary pass skip the pixels whose camera
        // ray escapes: one shared result each, the path kernel over the
        // pixels whose camera ray hits (F_SPARSE, vr_kernel.hpp primary_kernel)
        const bool sparse = VR_SPARSE_HDRI != 0 && wave_kernel && !c->cornell && count != 1 &&
                            (f & vr::F_STRICT) == 0u && !p.inline_prim;
        // (launches over the listed pixels of HDRI scenes -- a fifth of the
        // paths, all of them mesh paths -- take VR_QUEUES like the Cornell
        // box: C3 16 / 32 / 64 heads 16,630 / 16,408 / 16,172 Mpaths/s, r04)
        p.n_queues = (size_t)p.path_stride * 2u * k < ((size_t)1 << 25)
                         ? ((c->cornell || sparse) ? VR_QUEUES : VR_QUEUES_HDRI) : VR_QUEUES_LARGE;
        // VRHIP_QUEUES: work-queue heads for experiments (a power of two, 8..VR_MAX_QUEUES)
        static const uint32_t env_queues = [] {
            const char* e = std::getenv("VRHIP_QUEUES");
            const uint32_t q = e ? (uint32_t)std::atoi(e) : 0u;
            return (q >= 8 && q <= (uint32_t)VR_MAX_QUEUES && (q & (q - 1)) == 0) ? q : 0u;
        }();
        if (env_queues) p.n_queues = env_queues;
        if (!ovl) c->parity = 0;
        auto& l = c->lane[c->parity];
        // overlapped launches run on the lane's path stream, the others on
        // `stream` (in order behind everything queued there)
        const bool on_lane = p.use_scratch && ovl;
        hipStream_t rs = on_lane ? l.s : c->stream;
        if (on_lane && c->join) {           // scene, stream or buffers changed: wait for all of `stream`
            HIP_TRY(hipEventRecord(c->ev_join, c->stream));
            for (auto& ln : c->lane) HIP_TRY(hipStreamWaitEvent(ln.s, c->ev_join, 0));
            c->join = false;
        }
        if (p.use_scratch) {
            // launches that overlap: every path stream's
            // scratch at once -- a lane first used behind a launch in flight
            // would otherwise allocate there (hipMalloc waits for the device)
            // and serialise the overlapped launches; whole frames run on lane 0
            // (only where overlap can happen: never with vrhip_set_overlap(0))
            const bool all_lanes = ovl_size && c->overlap != 0 && count == 0;
            for (auto& ln : c->lane)
                if ((all_lanes || &ln == &l) && (rc = ensure_lane(c, ln, need, p.path_stride)) != VRHIP_OK) return rc;
            if (ovl) c->parity = (c->parity + 1u) % VR_PATH_STREAMS;
            p.paths = reinterpret_cast<vr::vr3*>(l.paths); p.path_w = reinterpret_cast<float*>(p.paths + need);
            p.prim = l.prim; p.chunk_ctr = l.chunk_ctr;
            p.sparse_px = sparse ? l.px_list : nullptr;
            // longest-first: launches whose drain is a large share of them (one
            // frame per call, shards) measure per sub-tile costs and take their
            // sub-tiles in the order the previous launch on this scratch measured
            const uint32_t n_sub = p.path_stride / 64u;
            const bool order = wave_kernel && small && count == 0 && c->cost_order && (VR_SHARD_SMALL != 0 || p.inline_prim);
            // per-path costs after the radiances and depth terms in the scratch
            // (need x 16 B holds need x 12 + path_stride x 4 + need x 1)
            p.path_cost = order ? reinterpret_cast<uint8_t*>(p.path_w + p.path_stride) : nullptr;
            // VRHIP_ORDER_SLOTS=1 (measurement): one slot, the previous launch's order
            static const uint32_t order_slots = [] {
                const char* e = std::getenv("VRHIP_ORDER_SLOTS");
                return (e && std::atoi(e) == 1) ? 1u : 2u;
            }();
            const uint32_t w = order_slots == 2u ? l.oi : 0u;
            p.sub_cost = order ? l.sub_cost[w] : nullptr;
            p.sub_order = (order && l.order_nsub[w] == n_sub) ? l.sub_order[w] : nullptr;
            p.order_cap = (uint32_t)order_cap(n_sub);
            if (on_lane && l.used) HIP_TRY(hipStreamWaitEvent(rs, l.finished, 0));
            // the order pass of this slot (it read the slot's costs, which this
            // launch's finish pass rewrites, and wrote the order this launch
            // reads); a launch that does not order waits for both slots
            for (uint32_t i = 0; i < 2u; ++i) {
                if ((i == w || !order) && l.order_pending[i]) {
                    HIP_TRY(hipStreamWaitEvent(rs, l.ordered[i], 0));
                    l.order_pending[i] = false;
                }
            }
        }
        hipEvent_t k0 = nullptr, k1 = nullptr;
        // per-launch span events (vrhip_kernel_stats) only with kernel timing
        // on (vrhip_set_kernel_timing): recorded on the stream around the
        // render kernels they cost ≈ 8 µs per synchronous one-frame call
        if (n_tiles && c->kernel_timing) {
            if ((rc = take_event(c, &k0)) != VRHIP_OK || (rc = take_event(c, &k1)) != VRHIP_OK) return rc;
            c->kev_pending.push_back({ k0, k1, 1u });
            HIP_TRY(hipEventRecord(k0, rs));
        }
        if (count != 1) {                 // production and its instrumented copy (same shape)
            c->last_split = p.split; c->last_use_scratch = p.use_scratch;
            c->last_kind = wave_kernel ? 1u : 0u;
        }
        // a synchronous one-frame call's path kernel + finish pass as one graph launch (VRHIP_GRAPH)
        const bool graph = c->use_graph && count == 0 && wave_kernel && k == 1u && !on_lane && rs == c->stream &&
                           !k1 && p.inline_prim && p.use_scratch;
        if (graph) {
            const uint32_t gi = (p.sub_cost && p.sub_cost == l.sub_cost[1]) ? 1u : 0u;
            if ((rc = one_frame_graph(c, p, n_tiles, stack, gi)) != VRHIP_OK) return rc;
            c->last_kind = 3u;
        } else {
            int e = vr::launch_render(p, n_tiles, stack, count, rs);
            if (e != 0) return fail(VRHIP_ERR_HIP, std::string("render launch: ") + hipGetErrorString((hipError_t)e));
            if (k1) HIP_TRY(hipEventRecord(k1, rs));
            if (on_lane) {
                HIP_TRY(hipEventRecord(l.done, rs));
                HIP_TRY(hipStreamWaitEvent(c->stream, l.done, 0));
            }
            // a call of one launch on `stream` on a context whose stream
            // nobody else uses: its finish pass is the last work on `stream`,
            // so it can carry the completion flag a following vrhip_sync polls
            const bool arm = c->sync_flag_mode && count == 0 && k == n_frames && done == 0 && !on_lane &&
                             p.use_scratch && n_tiles > 0 && n_tiles <= VR_SYNC_FLAG_MAX_TILES && !c->comm &&
                             c->group.empty() && !c->stream_shared;
            if (arm) {
                if (!c->sync_flag) {
                    HIP_TRY(hipHostMalloc((void**)&c->sync_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
                    *c->sync_flag = 0u;
                }
                if (!c->sync_ctr) {
                    HIP_TRY(hipMalloc((void**)&c->sync_ctr, kSyncCtrBytes));
                    HIP_TRY(hipMemsetAsync(c->sync_ctr, 0, kSyncCtrBytes, c->stream));
                }
                if (++c->sync_seq == 0u) c->sync_seq = 1u;
                p.sync_flag = c->sync_flag; p.sync_ctr = c->sync_ctr; p.sync_seq = c->sync_seq;
            }
            e = vr::launch_finish(p, n_tiles, c->stream);
            if (e != 0) return fail(VRHIP_ERR_HIP, std::string("finish launch: ") + hipGetErrorString((hipError_t)e));
            if (arm) c->flag_armed = p.sync_seq;
            p.sync_flag = nullptr; p.sync_ctr = nullptr;
        }
        int e = 0;
        if (p.use_scratch) {
            HIP_TRY(hipEventRecord(l.finished, c->stream));
            l.used = true;
        }
        if (p.path_cost) {
            // the next launch but one on this scratch takes this launch's
            // order (the slots alternate): sorted on the path stream behind
            // this finish pass, off the context stream, so a synchronous
            // caller waits for it neither here nor at its next launch
            const uint32_t w = p.sub_cost == l.sub_cost[0] ? 0u : 1u;
            HIP_TRY(hipStreamWaitEvent(l.s, l.finished, 0));
            e = vr::launch_order(p.sub_cost, l.sub_order[w], p.path_stride / 64u, p.order_cap, l.s);
            if (e != 0) return fail(VRHIP_ERR_HIP, std::string("order launch: ") + hipGetErrorString((hipError_t)e));
            HIP_TRY(hipEventRecord(l.ordered[w], l.s));
            l.order_pending[w] = true;
            l.order_nsub[w] = p.path_stride / 64u;
            l.oi = w ^ 1u;
        }
        c->frame += k;
        done += k;
    }
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->flag_synced = false;
    // kernel-time accounting of launches already completed: after this call's
    // launches are queued, so its event queries do not delay them (one frame
    // per synchronous call: they sat between the host's wake-up and the launch)
    if ((rc = account_pending(c, false)) != VRHIP_OK) return rc;
    return VRHIP_OK;
}

static int one_render(vrhip_ctx* c, uint32_t n_frames, const uint32_t* times, uint32_t time_seed)
{
    return render_impl(c, n_frames, times, time_seed, 0);
}

int vrhip_render_counted(vrhip_ctx* c, uint32_t n_frames, const uint32_t* times, uint32_t time_seed,
                         uint64_t counters[8])
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_render_counted");
    if (!counters) return fail(VRHIP_ERR_INVALID, "counters is NULL");
    int rc = render_impl(c, n_frames, times, time_seed, 1);
    if (rc) return rc;
    unsigned long long h[vr::kCounters] = {};
    HIP_TRY(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < vr::kCounters; ++i) counters[i] = (uint64_t)h[i];
    return VRHIP_OK;
}

int vrhip_render_profiled(vrhip_ctx* c, uint32_t n_frames, const uint32_t* times, uint32_t time_seed,
                          uint64_t counters[VRHIP_PROFILE_COUNTERS])
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_render_profiled");
    if (!counters) return fail(VRHIP_ERR_INVALID, "counters is NULL");
    static_assert(VRHIP_PROFILE_COUNTERS == vr::kCounters + vr::kExecCounters, "profile counter layout");
    int rc = render_impl(c, n_frames, times, time_seed, 2);
    if (rc) return rc;
    unsigned long long h[vr::kExecCounterBase + vr::kExecCounters] = {};
    HIP_TRY(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < vr::kCounters; ++i) counters[i] = (uint64_t)h[i];
    for (int i = 0; i < vr::kExecCounters; ++i) counters[vr::kCounters + i] = (uint64_t)h[vr::kExecCounterBase + i];
    return VRHIP_OK;
}

int vrhip_microbench_vmem(int device, uint32_t width_bytes, uint32_t distinct, double* lane_loads_per_s)
{
    if (!lane_loads_per_s || distinct == 0 || distinct > 64 || (64 % distinct) != 0 ||
        (width_bytes != 4 && width_bytes != 8 && width_bytes != 12 && width_bytes != 16))
        return fail(VRHIP_ERR_INVALID, "width must be 4/8/12/16 bytes, distinct a divisor of 64");
    HIP_TRY(hipSetDevice(device));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const uint32_t n_lines = 1u << 14;                   // 1 MiB: L2-resident (4 MiB per XCD)
    const uint32_t blocks = (uint32_t)cus * 8u;          // 8 waves per SIMD
    const int iters = 256;
    uint32_t* tab = nullptr;
    HIP_TRY(hipMalloc((void**)&tab, (size_t)n_lines * 64 + 64));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto done = [&](int code) {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        (void)hipFree(tab);
        return code;
    };
    if (hipMemset(tab, 0, (size_t)n_lines * 64 + 64) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess)
        return done(fail(VRHIP_ERR_HIP, "microbench setup failed"));
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {                  // the first launch warms the caches
        if (hipEventRecord(e0, nullptr) != hipSuccess ||
            vr::launch_vmem_roof((int)width_bytes, tab, n_lines, distinct, iters, blocks, tab + n_lines * 16, nullptr) != 0 ||
            hipEventRecord(e1, nullptr) != hipSuccess || hipEventSynchronize(e1) != hipSuccess)
            return done(fail(VRHIP_ERR_HIP, "microbench launch failed"));
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    *lane_loads_per_s = (double)blocks * 256.0 * iters * 4.0 / (best * 1e-3);
    return done(VRHIP_OK);
}

int vrhip_debug_counters(vrhip_ctx* c, uint64_t out[16], int reset)
{
    if (!c || !out) return fail(VRHIP_ERR_INVALID, "null argument");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    if ((rc = ensure_counters(c)) != VRHIP_OK) return rc;
    unsigned long long h[16] = {};
    HIP_TRY(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 16; ++i) out[i] = (uint64_t)h[i];
    if (reset) HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kDebugSlots, c->stream));
    return VRHIP_OK;
}

int vrhip_kernel_stats(vrhip_ctx* c, double* total_ms, uint64_t* launches, int reset)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    if ((rc = account_pending(c, true)) != VRHIP_OK) return rc;
    if (total_ms) *total_ms = c->kernel_ms_total;
    if (launches) *launches = c->launches_total;
    if (reset) {
        c->kernel_ms_total = 0.0;
        c->launches_total = 0;
        c->kev_union.clear();
        if (c->kev_origin) { c->kev_free.push_back(c->kev_origin); c->kev_origin = nullptr; }
    }
    return VRHIP_OK;
}

int vrhip_last_launch_info(vrhip_ctx* c, uint32_t* split, uint32_t* use_scratch, uint32_t* kind)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    if (split) *split = c->last_split;
    if (use_scratch) *use_scratch = c->last_use_scratch;
    if (kind) *kind = c->last_kind;
    return VRHIP_OK;
}

// Waits until the finish pass armed with number `seq` (render_impl) has
// stored it: the host sees the frame complete without the ≈ 13 µs the
// stream's completion signal takes after the kernel (profiles/r06i).  A
// fault or failed launch is caught by the hipStreamQuery made every ≈ 30 µs.
static int wait_flag(vrhip_ctx* c, uint32_t seq)
{
    ++c->sync_flag_waits;
    for (uint32_t n = 1;; ++n) {
        if (__atomic_load_n(c->sync_flag, __ATOMIC_ACQUIRE) == seq) break;
        if ((n & 1023u) == 0u) {
            const hipError_t e = hipStreamQuery(c->stream);
            if (e == hipSuccess) break;                    // drained (the flag is set too)
            if (e != hipErrorNotReady) return fail(VRHIP_ERR_HIP, std::string("sync: ") + hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    c->flag_synced = true;
    return VRHIP_OK;
}

static int one_sync(vrhip_ctx* c)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = set_device(c); if (rc) return rc;
    const uint32_t armed = c->svc.open ? 0u : c->flag_armed;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    if (armed) {
        if ((rc = wait_flag(c, armed)) != VRHIP_OK) return rc;
    } else {
        HIP_TRY(hipStreamSynchronize(c->stream));
        ++c->sync_stream_waits;
    }
    return svc_verify(c);
}

static int one_set_sync_flag(vrhip_ctx* c, int on)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    c->sync_flag_mode = on != 0 ? 1 : 0;
    c->flag_armed = 0;
    return VRHIP_OK;
}

int vrhip_sync_info(vrhip_ctx* c, uint64_t out[VRHIP_SYNC_INFO])
{
    if (!c || !out) return fail(VRHIP_ERR_INVALID, "null argument");
    uint64_t a = 0, b = 0;
    for (vrhip_ctx* m : c->group.empty() ? std::vector<vrhip_ctx*>{ c } : c->group) {
        a += m->sync_flag_waits; b += m->sync_stream_waits;
    }
    out[0] = a; out[1] = b;
    return VRHIP_OK;
}

int vrhip_frame_count(vrhip_ctx* c, uint32_t* frames)
{
    if (!c || !frames) return fail(VRHIP_ERR_INVALID, "null argument");
    *frames = c->frame - 1;
    return VRHIP_OK;
}

static int readback(vrhip_ctx* c, const void* src, void* dst, size_t bytes)
{
    if (!c || !dst) return fail(VRHIP_ERR_INVALID, "null argument");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return svc_verify(c);
}

int vrhip_read_accum(vrhip_ctx* c, float* out)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    if (!c->group.empty()) {                          // the accumulation lives on every device: gather it first
        const int rc = multi_gather(c, 1);
        if (rc != VRHIP_OK) return rc;
    }
    return readback(c, c->accum, out, (size_t)c->W * c->H * 16);
}
int vrhip_read_rgba8(vrhip_ctx* c, uint8_t* out)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    const int rc = multi_images(c);
    return rc ? rc : readback(c, c->rgba, out, (size_t)c->W * c->H * 4);
}
int vrhip_read_depth8(vrhip_ctx* c, uint8_t* out)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    const int rc = multi_images(c);
    return rc ? rc : readback(c, c->depth, out, (size_t)c->W * c->H * 4);
}

int vrhip_device_buffers(vrhip_ctx* c, void** accum, void** rgba8, void** depth8)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    const int rc = multi_images(c); if (rc) return rc;       // a group's lead: the whole image first
    if (set_device(c) == VRHIP_OK) (void)svc_close(c);     // the buffers hold every render so far
    // the caller may read them from its own streams: vrhip_sync then waits
    // for the stream's completion (the end of the kernels' write-back)
    c->stream_shared = true;
    if (accum) *accum = c->accum;
    if (rgba8) *rgba8 = c->rgba;
    if (depth8) *depth8 = c->depth;
    return VRHIP_OK;
}

int vrhip_set_tiling(vrhip_ctx* c, uint32_t rank, uint32_t n_ranks)
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_set_tiling");
    if (!c || n_ranks == 0 || rank >= n_ranks) return fail(VRHIP_ERR_INVALID, "bad tiling");
    // the gather buffers and the RCCL communicator are sized for the
    // communicator's tiling: it cannot change while they exist
    if (c->comm && (rank != c->comm_rank || n_ranks != c->comm_n))
        return fail(VRHIP_ERR_INVALID, "tiling is fixed while a communicator exists (vrhip_comm_destroy first)");
    quiesce(c);
    c->rank = rank; c->nranks = n_ranks;
    return VRHIP_OK;
}

static int one_set_overlap(vrhip_ctx* c, int mode)
{
    if (!c || mode < -1 || mode > 1) return fail(VRHIP_ERR_INVALID, "bad overlap mode");
    c->overlap = mode;
    return VRHIP_OK;
}

static int one_set_service(vrhip_ctx* c, int mode)
{
    if (!c || mode < -1 || mode > 1) return fail(VRHIP_ERR_INVALID, "bad service mode");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    c->service = mode;
    return VRHIP_OK;
}

int vrhip_set_service_timing(vrhip_ctx* c, uint32_t idle_us, uint32_t post_window_us, uint32_t post_delay_us)
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_set_service_timing");
    if (!c || idle_us > 10000000u || post_window_us > 10000000u || post_delay_us > 10000000u)
        return fail(VRHIP_ERR_INVALID, "bad service timing (each at most 10 s)");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    c->svc_idle_us = idle_us; c->svc_window_us = post_window_us; c->svc_post_delay_us = post_delay_us;
    return VRHIP_OK;
}

int vrhip_set_service_budget(vrhip_ctx* c, size_t bytes)
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_set_service_budget");
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    c->svc_budget = bytes;
    return VRHIP_OK;
}

int vrhip_service_stats(vrhip_ctx* c, uint64_t* refused_launches)
{
    if (!c || !refused_launches) return fail(VRHIP_ERR_INVALID, "null argument");
    *refused_launches = c->svc_refused;
    return VRHIP_OK;
}

int vrhip_service_info(vrhip_ctx* c, uint64_t out[VRHIP_SERVICE_INFO])
{
    if (!c || !out) return fail(VRHIP_ERR_INVALID, "null argument");
    out[0] = c->svc_refused;
    out[1] = c->svc_sessions;
    out[2] = c->svc_served;
    out[3] = c->svc_deferred;
    out[4] = c->svc_alloc_fallbacks;
    return VRHIP_OK;
}

static int one_set_path_split(vrhip_ctx* c, uint32_t groups)
{
    if (!c || groups > 2u * vr::kMaxFramesPerLaunch) return fail(VRHIP_ERR_INVALID, "bad path split");
    c->path_split = groups;
    return VRHIP_OK;
}

int vrhip_tile_pixels(uint32_t width, uint32_t height, uint32_t rank, uint32_t n_ranks, uint32_t* pix_out,
                      uint32_t* n_pix)
{
    if (!n_pix || n_ranks == 0 || rank >= n_ranks) return fail(VRHIP_ERR_INVALID, "bad tiling arguments");
    const uint32_t tiles_x = width / 16u, n_owned = owned_tiles_of(width, height, rank, n_ranks);
    *n_pix = n_owned * 256u;
    if (pix_out) {
        for (uint32_t j = 0; j < n_owned; ++j) {
            const uint32_t gt = rank + j * n_ranks, ty = tile_row(gt, tiles_x), tx = tile_col(gt, tiles_x, n_ranks);
            for (uint32_t px = 0; px < 256u; ++px)
                pix_out[j * 256u + px] = (ty * 16u + px / 16u) * width + tx * 16u + px % 16u;
        }
    }
    return VRHIP_OK;
}

int vrhip_owned_pixels(vrhip_ctx* c, uint32_t* n_pix)
{
    if (!c || !n_pix) return fail(VRHIP_ERR_INVALID, "null argument");
    *n_pix = owned_tiles_of(c->W, c->H, c->rank, c->nranks) * 256u;
    return VRHIP_OK;
}

static int elem_size(int what) { return what == 1 ? 16 : 4; }
static const void* buf_of(vrhip_ctx* c, int what) { return what == 1 ? (const void*)c->accum : what == 2 ? (const void*)c->depth : (const void*)c->rgba; }

int vrhip_pack_tiles(vrhip_ctx* c, int what, void* dst)
{
    if (!c || !dst || what < 0 || what > 2) return fail(VRHIP_ERR_INVALID, "bad pack arguments");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    int e = vr::launch_pack_tiles(buf_of(c, what), dst, (uint32_t)elem_size(what), c->W, c->W / 16u,
                                  owned_tiles_of(c->W, c->H, c->rank, c->nranks), c->rank, c->nranks, 0, c->stream);
    if (e) return fail(VRHIP_ERR_HIP, "pack launch failed");
    return VRHIP_OK;
}

int vrhip_unpack_tiles(vrhip_ctx* c, int what, const void* src, uint32_t n_ranks, size_t stride_bytes)
{
    if (!c || !src || what < 0 || what > 2 || n_ranks == 0) return fail(VRHIP_ERR_INVALID, "bad unpack arguments");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    if (stride_bytes) {                   // one launch for every rank's buffer
        const int e = vr::launch_unpack_ranks(src, const_cast<void*>(buf_of(c, what)), (uint32_t)elem_size(what), c->W,
                                              c->W / 16u, (c->W / 16u) * (c->H / 16u), 0u, n_ranks, stride_bytes,
                                              c->stream);
        if (e) return fail(VRHIP_ERR_HIP, "unpack launch failed");
        return VRHIP_OK;
    }
    const char* s = (const char*)src;      // tightly packed: buffers of different lengths, one launch each
    for (uint32_t r = 0; r < n_ranks; ++r) {
        const uint32_t n_owned = owned_tiles_of(c->W, c->H, r, n_ranks);
        int e = vr::launch_pack_tiles(s, const_cast<void*>(buf_of(c, what)), (uint32_t)elem_size(what), c->W,
                                      c->W / 16u, n_owned, r, n_ranks, 1, c->stream);
        if (e) return fail(VRHIP_ERR_HIP, "unpack launch failed");
        s += (size_t)n_owned * 256u * elem_size(what);
    }
    return VRHIP_OK;
}

// ---- multi-GPU tile gather over RCCL ------------------------
static int nccl_fail(ncclResult_t r, const char* what)
{
    return fail(VRHIP_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

static uint32_t max_owned_pixels(uint32_t W, uint32_t H, uint32_t n_ranks)
{
    return owned_tiles_of(W, H, 0, n_ranks) * 256u;       // rank 0 owns the most tiles
}

int vrhip_comm_unique_id(uint8_t id[VRHIP_COMM_ID_BYTES])
{
    if (!id) return fail(VRHIP_ERR_INVALID, "id is NULL");
    static_assert(VRHIP_COMM_ID_BYTES == sizeof(ncclUniqueId), "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
    return VRHIP_OK;
}

int vrhip_comm_init(vrhip_ctx* c, uint32_t rank, uint32_t n_ranks, const uint8_t id[VRHIP_COMM_ID_BYTES])
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_comm_init");
    if (!c || !id || n_ranks == 0 || rank >= n_ranks) return fail(VRHIP_ERR_INVALID, "bad communicator arguments");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
    dfree(c->comm_send); dfree(c->comm_recv);
    if ((rc = vrhip_set_tiling(c, rank, n_ranks)) != VRHIP_OK) return rc;
    c->comm_rank = rank; c->comm_n = n_ranks;
    c->comm_slot = (size_t)max_owned_pixels(c->W, c->H, n_ranks) * 16u;
    const size_t slot = c->comm_slot ? c->comm_slot : 16u;
    if (hipMalloc((void**)&c->comm_send, slot) != hipSuccess ||
        (rank == 0 && hipMalloc((void**)&c->comm_recv, slot * n_ranks) != hipSuccess))
        return fail(VRHIP_ERR_NOMEM, "gather buffers");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&c->comm, (int)n_ranks, u, (int)rank);   // blocks until every rank joins
    if (r != ncclSuccess) { c->comm = nullptr; return nccl_fail(r, "ncclCommInitRank"); }
    return VRHIP_OK;
}

int vrhip_comm_gather(vrhip_ctx* c, int what)
{
    if (c && !c->group.empty()) {                     // the group's own communicators
        if (what < 0 || what > 2) return fail(VRHIP_ERR_INVALID, "bad gather arguments");
        return multi_gather(c, what);
    }
    if (!c || what < 0 || what > 2) return fail(VRHIP_ERR_INVALID, "bad gather arguments");
    if (!c->comm) return fail(VRHIP_ERR_INVALID, "vrhip_comm_init has not been called");
    int rc = set_device(c); if (rc) return rc;
    if (c->service > 0 && c->svc.open && c->svc.posted > 0 && c->svc.fin.staging) {
        // explicit service mode only: inside a session the image after its
        // last launch is staged by the session's finish pass and gathered
        // when the session closes (the caller syncs before any host-side
        // wait on the other ranks, include/vrhip.h).  In automatic mode the
        // gather closes the session and is enqueued now (below, through
        // vrhip_pack_tiles), so no rank's collective waits on a host call
        c->svc.fin.gather[c->svc.posted - 1u] |= 1u << what;
        c->svc.gathers.emplace_back(c->svc.posted - 1u, what);
        ++c->svc_deferred;
        return VRHIP_OK;
    }
    // pack -> gather -> (rank 0) unpack, all on the context stream, behind the
    // finish passes that wrote the images
    if (c->rank != c->comm_rank || c->nranks != c->comm_n)
        return fail(VRHIP_ERR_INVALID, "tiling differs from the communicator's");
    const size_t bytes = (size_t)max_owned_pixels(c->W, c->H, c->nranks) * (size_t)elem_size(what);
    if (bytes > c->comm_slot) return fail(VRHIP_ERR_INVALID, "gather payload exceeds the communicator's buffers");
    if ((rc = vrhip_pack_tiles(c, what, c->comm_send)) != VRHIP_OK) return rc;
    const ncclResult_t r = ncclGather(c->comm_send, c->comm_recv, bytes, ncclUint8, 0, c->comm, c->stream);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGather");
    if (c->rank == 0) return vrhip_unpack_tiles(c, what, c->comm_recv, c->nranks, bytes);
    return VRHIP_OK;
}

int vrhip_comm_destroy(vrhip_ctx* c)
{
    if (c && !c->group.empty()) return refuse_multi(c, "vrhip_comm_destroy");
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    int rc = set_device(c); if (rc) return rc;
    if ((rc = svc_close(c)) != VRHIP_OK) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->comm) {
        const ncclResult_t r = ncclCommDestroy(c->comm);
        c->comm = nullptr;
        if (r != ncclSuccess) return nccl_fail(r, "ncclCommDestroy");
    }
    dfree(c->comm_send); dfree(c->comm_recv);
    return VRHIP_OK;
}

int vrhip_last_kernel_ms(vrhip_ctx* c, float* ms)
{
    if (!c || !ms) return fail(VRHIP_ERR_INVALID, "null argument");
    if (set_device(c) == VRHIP_OK) (void)svc_close(c);
    if (!c->timed || !c->ev0_valid) { *ms = 0.f; return VRHIP_OK; }   // no render, or kernel timing off
    HIP_TRY(hipEventSynchronize(c->ev1));
    HIP_TRY(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return VRHIP_OK;
}

static int one_set_kernel_timing(vrhip_ctx* c, int on)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    c->kernel_timing = on != 0;
    return VRHIP_OK;
}

int vrhip_bvh_info(vrhip_ctx* c, uint32_t* depth, uint32_t* n_nodes, uint32_t* n_slots)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    if (depth) *depth = c->bvh_depth;
    if (n_nodes) *n_nodes = c->bvh_nodes;
    if (n_slots) *n_slots = (uint32_t)c->n_slots;
    return VRHIP_OK;
}

int vrhip_selftest_math(int device, int fn, const float* a, const float* b, float* out, size_t n)
{
    if (!a || !b || !out) return fail(VRHIP_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(device));
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc((void**)&da, n * 4 + 4));
    HIP_TRY(hipMalloc((void**)&db, n * 4 + 4));
    HIP_TRY(hipMalloc((void**)&dout, n * 4 + 4));
    HIP_TRY(hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice));
    int e = vr::launch_selftest_math(fn, da, db, dout, n, nullptr);
    if (e) return fail(VRHIP_ERR_HIP, "selftest launch failed");
    HIP_TRY(hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost));
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
    return VRHIP_OK;
}

static int selftest_exact(int fn, int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches,
                          uint32_t* first_bad)
{
    if (!mismatches || !first_bad) return fail(VRHIP_ERR_INVALID, "null argument");
    if (lo_bits > hi_bits || hi_bits > 0x80000000u) return fail(VRHIP_ERR_INVALID, "bit range outside [0, 2^31]");
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 16));
    uint32_t* df = (uint32_t*)(d + 1);
    const uint32_t init_first = 0xffffffffu;
    HIP_TRY(hipMemset(d, 0, 8));
    HIP_TRY(hipMemcpy(df, &init_first, 4, hipMemcpyHostToDevice));
    float* T = nullptr;
    if (fn == 2) {                                        // the tonemap table under test
        HIP_TRY(hipMalloc((void**)&T, 256 * sizeof(float)));
        if (vr::launch_tone_table(T, nullptr)) { (void)hipFree(d); (void)hipFree(T); return fail(VRHIP_ERR_HIP, "tone table launch failed"); }
    }
    int e = vr::launch_selftest_exact(fn, lo_bits, hi_bits, d, df, T, nullptr);
    if (e) { (void)hipFree(d); if (T) (void)hipFree(T); return fail(VRHIP_ERR_HIP, "selftest launch failed"); }
    unsigned long long n = 0;
    HIP_TRY(hipMemcpy(&n, d, 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    if (T) (void)hipFree(T);
    *mismatches = n;
    return VRHIP_OK;
}

int vrhip_selftest_rcp(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches, uint32_t* first_bad)
{
    return selftest_exact(0, device, lo_bits, hi_bits, mismatches, first_bad);
}

int vrhip_selftest_sqrt(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches, uint32_t* first_bad)
{
    return selftest_exact(1, device, lo_bits, hi_bits, mismatches, first_bad);
}

int vrhip_selftest_tonemap(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches, uint32_t* first_bad)
{
    return selftest_exact(2, device, lo_bits, hi_bits, mismatches, first_bad);
}

int vrhip_build_flat(const float* positions, const float* normals, const float* tangents, const float* uvs,
                     uint32_t n_verts, const uint32_t* tris, uint32_t n_tris, uint32_t max_leaf_tris,
                     float* bvh_out, size_t* n_bvh_f4, float* verts_out, float* normals_out,
                     float* tangents_out, float* uvs_out, size_t* n_slots)
{
    if (!n_bvh_f4 || !n_slots) return fail(VRHIP_ERR_INVALID, "size outputs are required");
    vr::FlatMesh m;
    if (vr::build_flat(positions, normals, tangents, uvs, n_verts, tris, n_tris, max_leaf_tris, m) != 0)
        return fail(VRHIP_ERR_INVALID, "BVH build failed (empty mesh or bad indices)");
    const bool fill = bvh_out && verts_out && normals_out && tangents_out && uvs_out;
    if (fill) {
        if (*n_bvh_f4 < m.bvh.size() || *n_slots < m.verts.size()) return fail(VRHIP_ERR_INVALID, "output arrays too small");
        std::memcpy(bvh_out, m.bvh.data(), m.bvh.size() * 16);
        std::memcpy(verts_out, m.verts.data(), m.verts.size() * 16);
        std::memcpy(normals_out, m.normals.data(), m.normals.size() * 16);
        std::memcpy(tangents_out, m.tangents.data(), m.tangents.size() * 16);
        std::memcpy(uvs_out, m.uvs.data(), m.uvs.size() * 8);
    }
    *n_bvh_f4 = m.bvh.size();
    *n_slots = m.verts.size();
    return VRHIP_OK;
}

int vrhip_validate_flat(const float* bvh, size_t n_bvh_f4, const float* verts, size_t n_slots,
                        uint32_t* depth, uint32_t* n_nodes)
{
    int v = vr::validate_flat(bvh, n_bvh_f4, verts, n_slots, depth, n_nodes);
    if (v != 0) return fail(VRHIP_ERR_BVH, "validation failed (code " + std::to_string(v) + ")");
    return VRHIP_OK;
}


// ---- multi-device renderer (SURVEY 8b create_multi) -------------------------
// One vrhip_ctx over several GPUs of this process: a member context per
// device, each owning the 16x16 tiles i, i + n, ... of the image; the RCCL
// communicators made in one call (ncclCommInitAll); every setting and upload
// fanned out; vrhip_render renders every device's tiles and gathers the RGBA8
// and depth tiles to the lead device (one grouped ncclGather each), whose
// images are then the whole frame (read-back, GL presentation).  The
// reference's single caller creates one renderer (src/NGLScene.cpp:82-89):
// through this context it drives all the devices named in VRHIP_DEVICES
// (integration/vRendererHIP.cpp).

} // extern "C"
template <typename F>
static int fanout(vrhip_ctx* c, F&& f)
{
    if (!c) return fail(VRHIP_ERR_INVALID, "null ctx");
    if (c->group.empty()) return f(c);
    for (vrhip_ctx* m : c->group) {
        const int rc = f(m);
        if (rc != VRHIP_OK) return rc;
    }
    return VRHIP_OK;
}
extern "C" {

static int refuse_multi(vrhip_ctx* c, const char* what)
{
    return fail(VRHIP_ERR_INVALID, std::string(what) + " is not available on a multi-device context (vrhip_create_multi)");
}

// every member's `what` tiles to the lead: pack on each member's stream, one
// grouped ncclGather (one thread drives all ranks), unpack on the lead
static int multi_gather(vrhip_ctx* c, int what)
{
    const size_t esz = what == 1 ? 16u : 4u;
    const size_t bytes = (size_t)max_owned_pixels(c->W, c->H, (uint32_t)c->group.size()) * esz;
    int rc;
    for (vrhip_ctx* m : c->group) {
        if ((rc = set_device(m)) != VRHIP_OK) return rc;
        if ((rc = svc_close(m)) != VRHIP_OK) return rc;
        if ((rc = vr::launch_pack_tiles(buf_of(m, what), m->comm_send, (uint32_t)esz, m->W, m->W / 16u,
                                        owned_tiles_of(m->W, m->H, m->rank, m->nranks), m->rank, m->nranks, 0,
                                        m->stream)) != 0)
            return fail(VRHIP_ERR_HIP, "pack launch failed");
    }
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (vrhip_ctx* m : c->group) {
        r = ncclGather(m->comm_send, m->comm_recv, bytes, ncclUint8, 0, m->comm, m->stream);
        if (r != ncclSuccess) { (void)ncclGroupEnd(); return nccl_fail(r, "ncclGather"); }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
    if ((rc = set_device(c)) != VRHIP_OK) return rc;
    const uint32_t n = (uint32_t)c->group.size();
    if (n > 1 && vr::launch_unpack_ranks(c->comm_recv + bytes, const_cast<void*>(buf_of(c, what)), (uint32_t)esz,
                                         c->W, c->W / 16u, (c->W / 16u) * (c->H / 16u), 1u, n, bytes, c->stream) != 0)
        return fail(VRHIP_ERR_HIP, "unpack launch failed");       // (the lead's own tiles are in place)
    return VRHIP_OK;
}

// The lead's colour and depth images after the last render: the members'
// render-service sessions close and their RGBA8 and depth tiles are gathered
// (two grouped ncclGathers), once per run of render calls -- so back-to-back
// renders with no read in between keep their sessions open across calls.
static int multi_images(vrhip_ctx* c)
{
    if (!c || c->group.empty() || !c->group_stale) return VRHIP_OK;
    int rc = multi_gather(c, 0);
    if (rc == VRHIP_OK) rc = multi_gather(c, 2);
    if (rc == VRHIP_OK) c->group_stale = false;
    return rc;
}

int vrhip_create_multi(const int* devices, uint32_t n_devices, uint32_t width, uint32_t height, vrhip_ctx** out)
{
    if (!out || !devices || n_devices == 0 || n_devices > 64)
        return fail(VRHIP_ERR_INVALID, "bad multi-device arguments (1..64 devices)");
    *out = nullptr;
    for (uint32_t i = 0; i < n_devices; ++i)
        for (uint32_t j = 0; j < i; ++j)
            if (devices[i] == devices[j]) return fail(VRHIP_ERR_INVALID, "a device appears twice");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(VRHIP_ERR_NO_DEVICE, "no HIP device");
    for (uint32_t i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= n) return fail(VRHIP_ERR_INVALID, "device index out of range");
    std::vector<vrhip_ctx*> ms(n_devices, nullptr);
    auto undo = [&](int code) {
        for (vrhip_ctx* m : ms)
            if (m) { m->group.clear(); vrhip_destroy(m); }
        return code;
    };
    int rc;
    for (uint32_t i = 0; i < n_devices; ++i) {
        if ((rc = vrhip_create(devices[i], width, height, &ms[i])) != VRHIP_OK) return undo(rc);
        ms[i]->rank = i; ms[i]->nranks = n_devices;
    }
    std::vector<ncclComm_t> comms(n_devices, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), (int)n_devices, devices);
    if (r != ncclSuccess) return undo(nccl_fail(r, "ncclCommInitAll"));
    const size_t slot = (size_t)max_owned_pixels(width, height, n_devices) * 16u;
    for (uint32_t i = 0; i < n_devices; ++i) {
        vrhip_ctx* m = ms[i];
        m->comm = comms[i];
        m->comm_rank = i; m->comm_n = n_devices; m->comm_slot = slot;
        if ((rc = set_device(m)) != VRHIP_OK) return undo(rc);
        if (hipMalloc((void**)&m->comm_send, slot ? slot : 16u) != hipSuccess ||
            (i == 0 && hipMalloc((void**)&m->comm_recv, (slot ? slot : 16u) * n_devices) != hipSuccess))
            return undo(fail(VRHIP_ERR_NOMEM, "gather buffers"));
    }
    ms[0]->group = ms;
    (void)set_device(ms[0]);
    *out = ms[0];
    return VRHIP_OK;
}

int vrhip_device_group(vrhip_ctx* c, uint32_t* n_devices, int* devices)
{
    if (!c || !n_devices) return fail(VRHIP_ERR_INVALID, "null argument");
    const uint32_t n = c->group.empty() ? 1u : (uint32_t)c->group.size();
    if (devices)
        for (uint32_t i = 0; i < n; ++i) devices[i] = c->group.empty() ? c->device : c->group[i]->device;
    *n_devices = n;
    return VRHIP_OK;
}

int vrhip_set_camera(vrhip_ctx* c, const float origin[3], const float dir[3], const float up[3], const float right[3],
                     float fov_scale)
{ return fanout(c, [&](vrhip_ctx* m) { return one_set_camera(m, origin, dir, up, right, fov_scale); }); }
int vrhip_clear(vrhip_ctx* c) { return fanout(c, [&](vrhip_ctx* m) { return one_clear(m); }); }
int vrhip_set_fresnel(vrhip_ctx* c, float coef, float power)
{ return fanout(c, [&](vrhip_ctx* m) { return one_set_fresnel(m, coef, power); }); }
int vrhip_use_cornell_box(vrhip_ctx* c, int e) { return fanout(c, [&](vrhip_ctx* m) { return one_use_cornell_box(m, e); }); }
int vrhip_use_example_sphere(vrhip_ctx* c, int e) { return fanout(c, [&](vrhip_ctx* m) { return one_use_example_sphere(m, e); }); }
int vrhip_set_strict_traversal(vrhip_ctx* c, int e) { return fanout(c, [&](vrhip_ctx* m) { return one_set_strict_traversal(m, e); }); }
int vrhip_use_brdf(vrhip_ctx* c, int e) { return fanout(c, [&](vrhip_ctx* m) { return one_use_brdf(m, e); }); }
int vrhip_upload_mesh_flat(vrhip_ctx* c, const float* bvh, size_t n_bvh_f4, const float* verts, const float* normals,
                           const float* tangents, const float* uvs, size_t n_slots)
{ return fanout(c, [&](vrhip_ctx* m) { return one_upload_mesh_flat(m, bvh, n_bvh_f4, verts, normals, tangents, uvs, n_slots); }); }
int vrhip_upload_hdr(vrhip_ctx* c, const float* rgba, uint32_t w, uint32_t h)
{ return fanout(c, [&](vrhip_ctx* m) { return one_upload_hdr(m, rgba, w, h); }); }
int vrhip_upload_hdr_half(vrhip_ctx* c, const uint16_t* rgba_half, uint32_t w, uint32_t h)
{ return fanout(c, [&](vrhip_ctx* m) { return one_upload_hdr_half(m, rgba_half, w, h); }); }
int vrhip_upload_texture(vrhip_ctx* c, int type, const float* rgba, uint32_t w, uint32_t h)
{ return fanout(c, [&](vrhip_ctx* m) { return one_upload_texture(m, type, rgba, w, h); }); }
int vrhip_upload_brdf(vrhip_ctx* c, const float* table, size_t n_floats)
{ return fanout(c, [&](vrhip_ctx* m) { return one_upload_brdf(m, table, n_floats); }); }
int vrhip_set_overlap(vrhip_ctx* c, int mode) { return fanout(c, [&](vrhip_ctx* m) { return one_set_overlap(m, mode); }); }
int vrhip_set_path_split(vrhip_ctx* c, uint32_t groups) { return fanout(c, [&](vrhip_ctx* m) { return one_set_path_split(m, groups); }); }
int vrhip_set_service(vrhip_ctx* c, int mode) { return fanout(c, [&](vrhip_ctx* m) { return one_set_service(m, mode); }); }
int vrhip_set_kernel_timing(vrhip_ctx* c, int on) { return fanout(c, [&](vrhip_ctx* m) { return one_set_kernel_timing(m, on); }); }
int vrhip_set_sync_flag(vrhip_ctx* c, int on) { return fanout(c, [&](vrhip_ctx* m) { return one_set_sync_flag(m, on); }); }
int vrhip_sync(vrhip_ctx* c)
{
    const int rc = multi_images(c);                  // a group: the lead's images are complete after a sync
    return rc ? rc : fanout(c, [&](vrhip_ctx* m) { return one_sync(m); });
}

int vrhip_render(vrhip_ctx* c, uint32_t n_frames, const uint32_t* times, uint32_t time_seed)
{
    if (!c || c->group.empty()) return one_render(c, n_frames, times, time_seed);
    // every device renders its tiles (asynchronously, on its own render
    // service when calls come back to back); the colour and depth tiles go to
    // the lead when its images are next needed (multi_images: read-back, GL
    // present, device buffers, sync)
    for (vrhip_ctx* m : c->group) {
        const int rc = one_render(m, n_frames, times, time_seed);
        if (rc != VRHIP_OK) return rc;
    }
    c->group_stale = true;
    return VRHIP_OK;
}

} // extern "C"
