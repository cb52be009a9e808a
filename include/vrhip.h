/*
 * vrhip.h -- C ABI of libvrhip.so, the MI355X (gfx950) path-tracing backend
 * that drops in behind the reference's vRenderer interface as vRendererHIP.
 *
 * Plain C: opaque handle, plain pointers and sizes, int status codes
 * (0 = VRHIP_OK, never exit()).  All host pointers are copied; the library
 * never frees caller memory.  Calls on one context are not re-entrant (the
 * reference runs everything on the Qt GUI thread, src/NGLScene.cpp:249-472).
 *
 * Each entry point names the reference interface it replaces.  Reference
 * paths are relative to the v0q/vRenderer_PathTracer repository root.
 */
#ifndef VRHIP_H
#define VRHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VRHIP_ABI_VERSION 6

typedef enum vrhip_status {
    VRHIP_OK = 0,
    VRHIP_ERR_INVALID = -1,      /* bad argument / handle */
    VRHIP_ERR_HIP = -2,          /* HIP runtime error (see vrhip_last_error) */
    VRHIP_ERR_NO_ENV = -3,       /* HDRI mode with no environment loaded */
    VRHIP_ERR_BVH = -4,          /* malformed or too-deep flattened BVH */
    VRHIP_ERR_NO_DEVICE = -5,
    VRHIP_ERR_NOMEM = -6,
    VRHIP_ERR_COMM = -7          /* RCCL error (see vrhip_last_error) */
} vrhip_status;

/* vTextureType, cuda/include/PathTracer.cuh:86 */
typedef enum vrhip_texture_type { VRHIP_TEX_DIFFUSE = 0, VRHIP_TEX_NORMAL = 1, VRHIP_TEX_SPECULAR = 2 } vrhip_texture_type;

typedef struct vrhip_ctx vrhip_ctx;

/* Thread-local text of the last error. */
const char *vrhip_last_error(void);
int vrhip_abi_version(void);
/* SHA-256 (hex) of the sources, this header and the compile flags the
 * library was built from; the Python loader rebuilds when it differs from
 * the files on disk, and bench.py / smoke() print it. */
const char *vrhip_build_id(void);
int vrhip_device_count(int *count);

/* ---- lifetime -------------------------------------------------------- */
/* replaces vRendererCuda::init (src/vRendererCuda.cpp:38-55): allocates the
 * float4[W*H] accumulation buffer and the RGBA8 colour/depth images on
 * `device`, zero-fills, frame counter = 1.  1 <= width, height <= 65535. */
int vrhip_create(int device, uint32_t width, uint32_t height, vrhip_ctx **out);
/* One renderer over several GPUs of this process (SURVEY 8(b) "create_multi";
 * no reference counterpart: the reference's caller creates one renderer,
 * src/NGLScene.cpp:82-89).  A member context per device in `devices` (no
 * repeats), member i rendering the 16x16 tiles vrhip_set_tiling deals rank i
 * of n; the
 * RCCL communicators are made in one call (ncclCommInitAll).  The returned
 * context is the lead (devices[0]): every setting and upload on it fans out
 * to all members; vrhip_render renders every device's tiles (each member
 * with its own render service for back-to-back calls, vrhip_set_service), and
 * the RGBA8 and depth tiles are gathered to the lead (one grouped ncclGather
 * each) when the lead's images are next needed -- vrhip_read_rgba8/depth8,
 * vrhip_gl_present, vrhip_device_buffers, vrhip_sync -- so read-back and GL
 * presentation show the whole frame; vrhip_read_accum gathers the
 * accumulation first; vrhip_comm_gather gathers the given image.  Refused on
 * it: vrhip_set_tiling, vrhip_set_stream, vrhip_comm_init/destroy, the
 * service test hooks, the counting renders.  n = 1 is allowed (the same code,
 * a one-rank communicator). */
int vrhip_create_multi(const int *devices, uint32_t n_devices, uint32_t width, uint32_t height, vrhip_ctx **out);
/* The devices of a context (one for vrhip_create, the group for
 * vrhip_create_multi, lead first); `devices` may be NULL (count only). */
int vrhip_device_group(vrhip_ctx *ctx, uint32_t *n_devices, int *devices);
/* replaces vRendererCuda::cleanUp + cu_cleanUp (src/vRendererCuda.cpp:167-199,
 * cuda/src/PathTracer.cu:1009-1030). NULL is a no-op. */
int vrhip_destroy(vrhip_ctx *ctx);
/* Run subsequent work on this hipStream_t (NULL = the context's own stream). */
int vrhip_set_stream(vrhip_ctx *ctx, void *hip_stream);
void *vrhip_get_stream(vrhip_ctx *ctx);

/* ---- per-frame state -------------------------------------------------- */
/* replaces vRendererCuda::updateCamera (src/vRendererCuda.cpp:69-98): copies
 * the camera (xyz used, w = 0 as in the reference), resets frame = 1 and
 * clears the accumulation buffer. */
int vrhip_set_camera(vrhip_ctx *ctx, const float origin[3], const float dir[3],
                     const float up[3], const float right[3], float fov_scale);
/* replaces vRendererCuda::clearBuffer (src/vRendererCuda.cpp:100-105) and
 * cu_fillFloat4 (cuda/src/PathTracer.cu:1003-1007). */
int vrhip_clear(vrhip_ctx *ctx);
/* Stores the Fresnel parameters passed by value to every launch
 * (include/vRenderer.h:139-145; the base class then calls clearBuffer). */
int vrhip_set_fresnel(vrhip_ctx *ctx, float coef, float power);
/* replace cu_useCornellBox / cu_useExampleSphere / cu_useBRDF
 * (cuda/src/PathTracer.cu:976-989); flags travel by value in the launch. */
int vrhip_use_cornell_box(vrhip_ctx *ctx, int enable);
int vrhip_use_example_sphere(vrhip_ctx *ctx, int enable);
int vrhip_use_brdf(vrhip_ctx *ctx, int enable);
/* Traversal mode.  Default (0): children whose slab entry lies beyond the
 * closest hit so far (x 1.0009765625) are skipped -- the reference visits
 * every box the ray's line pierces (span end clamped to 1e20,
 * cuda/src/PathTracer.cu:316,322); skipping them leaves the closest hit
 * unchanged except in fp32 rounding corner cases.  1: visit
 * every pierced box exactly as the reference. */
int vrhip_set_strict_traversal(vrhip_ctx *ctx, int enable);

/* ---- scene uploads ---------------------------------------------------- */
/* replaces the device half of vRendererCuda::initMesh
 * (src/vRendererCuda.cpp:282-317) + cu_meshInitialised
 * (cuda/src/PathTracer.cu:997-1001): takes the flattened arrays in exactly
 * the reference layout (bvh: float4[n_bvh_f4], node = 4 float4 as in
 * :271-278; verts/normals/tangents: float4[n_slots]; uvs: float2[n_slots];
 * leaf runs end with a 0x80000000 terminator slot).  The library validates
 * the tree, records its depth and builds its own device layout. */
int vrhip_upload_mesh_flat(vrhip_ctx *ctx,
                           const float *bvh, size_t n_bvh_f4,
                           const float *verts, const float *normals,
                           const float *tangents, const float *uvs, size_t n_slots);
/* Convenience: indexed triangle mesh (vHVert/vHTriangle, include/vDataTypes.h)
 * -> native binned-SAH BVH -> reference flattening -> upload.  positions,
 * normals, tangents: float[3*n_verts]; uvs: float[2*n_verts] (may be NULL);
 * tris: uint32[3*n_tris]. */
int vrhip_upload_mesh_indexed(vrhip_ctx *ctx, const float *positions, const float *normals,
                              const float *tangents, const float *uvs, uint32_t n_verts,
                              const uint32_t *tris, uint32_t n_tris, uint32_t max_leaf_tris);
/* replaces vRendererCuda::loadHDR (src/vRendererCuda.cpp:320-340) +
 * cu_setHDRDim: rgba float4[w*h] (or half4 with the _half variant, the
 * Imf::Rgba layout, converted on the device). */
int vrhip_upload_hdr(vrhip_ctx *ctx, const float *rgba, uint32_t w, uint32_t h);
int vrhip_upload_hdr_half(vrhip_ctx *ctx, const uint16_t *rgba_half, uint32_t w, uint32_t h);
/* replaces the device half of vRendererCuda::loadTexture
 * (src/vRendererCuda.cpp:342-411) + cu_bindTexture: rgba float4[w*h]
 * (already gamma-converted by the caller, as the reference host does). */
int vrhip_upload_texture(vrhip_ctx *ctx, int type, const float *rgba, uint32_t w, uint32_t h);
/* replaces the device half of vRendererCuda::loadBRDF
 * (src/vRendererCuda.cpp:413-437) + cu_bindBRDF: float[3*90*90*180] planar
 * R,G,B MERL table.  Copies (interleaving the channels on the device, so a
 * lookup reads one cache line); does NOT take ownership (the C++ adapter
 * reproduces the reference's delete[]). */
int vrhip_upload_brdf(vrhip_ctx *ctx, const float *table, size_t n_floats);

/* replaces vBRDFLoader::loadBinary (src/BRDFLoader.cpp:15-50): reads a MERL
 * .binary file (3 int32 dims, then 3*90*90*180 doubles, planar R,G,B) into
 * `table` as floats in the same order.  Host only; the caller passes the
 * table to vrhip_upload_brdf.  VRHIP_ERR_INVALID on a dimension mismatch or
 * short file (the reference prints and returns nullptr). */
int vrhip_load_merl(const char *path, float *table, size_t n_floats);

/* replaces the OpenEXR read in NGLScene::loadHDRMap (src/NGLScene.cpp:205-231,
 * Imf::RgbaInputFile over the data window): a single-part scanline .exr
 * (NONE, RLE, ZIPS or ZIP compression; HALF/FLOAT/UINT channels) as half RGBA
 * (Imf::Rgba layout, FLOAT samples rounded to half; missing R/G/B = 0,
 * A = 1), ready for vrhip_upload_hdr_half.  Pass rgba_half = NULL to query
 * the size.  Host only. */
int vrhip_load_exr(const char *path, uint16_t *rgba_half, size_t n_values, uint32_t *width, uint32_t *height);

/* ---- display interop ---------------------------------------------------- */
/* replaces vRendererCuda::registerTextureBuffer / registerDepthBuffer
 * (src/vRendererCuda.cpp:57-67): registers an OpenGL texture (which = 0:
 * colour, 1: depth; target e.g. GL_TEXTURE_2D = 0x0DE1) with HIP.  Needs the
 * caller's GL context current. */
int vrhip_gl_register_image(vrhip_ctx *ctx, int which, unsigned int gl_texture, unsigned int gl_target);
/* Copies the RGBA8 colour and depth images into the registered textures
 * (map, device-to-array copy, unmap); the reference's kernel wrote them
 * through surfaces (src/vRendererCuda.cpp:117-162). Synchronous. */
int vrhip_gl_present(vrhip_ctx *ctx);

/* ---- rendering -------------------------------------------------------- */
/* replaces vRendererCuda::render (src/vRendererCuda.cpp:107-165) +
 * cu_runRenderKernel (cuda/src/PathTracer.cu:870-892), for n_frames
 * consecutive frames in one device pass.  times[i] is the _time RNG seed of
 * frame i (the reference uses wall-clock ms); times may be NULL, then
 * `time_seed` is used for every frame.  Enqueues and returns; call
 * vrhip_sync for the reference's synchronous behaviour.  The path kernels
 * run on the context stream or, behind a launch still in flight, on the
 * context's three internal path streams (see vrhip_set_overlap);
 * the finish pass that writes the accumulation, colour and depth images runs
 * on the context stream after them, so work queued on the context stream
 * afterwards (reads, vrhip_pack_tiles, a collective) sees the results. */
int vrhip_render(vrhip_ctx *ctx, uint32_t n_frames, const uint32_t *times, uint32_t time_seed);
/* Same render, through the counting kernel variant (identical results, plus
 * per-event counts for the roofline's algorithmic bytes):
 * counters[0..7] = rays (intersectScene calls), inner-node visits (64 B),
 * terminator slot reads (16 B; 0 with the device layout), triangle tests
 * (48 B), hit
 * attribute bytes, texture fetches (16 B), HDRI fetches (16 B), BRDF lookups
 * (12 B).  Synchronous. */
int vrhip_render_counted(vrhip_ctx *ctx, uint32_t n_frames, const uint32_t *times, uint32_t time_seed,
                         uint64_t counters[8]);
/* Same render as vrhip_render -- the production kernels' algorithm (t-culled
 * traversal unless strict, primary hit shared by a pixel's paths, last bounce
 * without material sampling), the scene specialisation's launch shape
 * (block size, waves per SIMD, node-loop threshold, work queues) and results
 * -- through an instrumented instantiation of that specialisation that
 * counts the memory operations its kernels issue (the roofline's executed
 * bytes; no reference counterpart).  Launches of one frame take the primary
 * pass here (production traces their camera rays in the path kernel), and
 * counting launches never overlap a launch in flight.
 * counters[0..7] as vrhip_render_counted but for the executed work
 * (attribute bytes include the 36 B of vertices a mesh hit's face normal
 * reads), then [8] node visits served from the block's LDS copy of the tree
 * top, [9] triangle loads issued
 * (36 B each; an odd leaf's last pair loads its triangle twice), [10] mesh
 * hits shaded, [11] of those through the normal map, [12..15] every global
 * lane load the production kernels issue, by width: 16 B, 12 B, 8 B, 4 B
 * (nodes, triangles, primary records, attributes, texels, BRDF entries),
 * [16] paths that took their pixel's shared escape radiance (sphere-only HDRI
 * scenes: a camera ray that escapes gives every path of the pixel the same
 * result, fetched once per pixel and launch).
 * Synchronous. */
#define VRHIP_PROFILE_COUNTERS 17
int vrhip_render_profiled(vrhip_ctx *ctx, uint32_t n_frames, const uint32_t *times, uint32_t time_seed,
                          uint64_t counters[VRHIP_PROFILE_COUNTERS]);
/* Waits until every render queued on the context is complete: the
 * accumulation, colour and depth images hold it (cudaStreamSynchronize in
 * vRendererCuda::render, src/vRendererCuda.cpp:107-165).  After a call of one
 * launch on the context stream (one frame per call, the reference's cadence)
 * it returns as soon as the finish pass's last block has stored its results:
 * the pass counts its blocks' arrivals and the last one stores the call's
 * number to host-coherent memory, which vrhip_sync polls -- about 8 us
 * before the stream's own completion signal reaches the host.  Work the
 * library or the caller queues on the context stream afterwards is ordered
 * behind the pass as usual.  A context whose stream or buffers were handed
 * out (vrhip_get_stream, vrhip_set_stream, vrhip_device_buffers: the caller
 * may read the images from its own streams) always waits for the stream, as
 * does a context with a communicator.  vrhip_set_sync_flag(ctx, 0), or
 * VRHIP_SYNC_FLAG=0 in the environment at creation, turns the flag off. */
int vrhip_sync(vrhip_ctx *ctx);
int vrhip_set_sync_flag(vrhip_ctx *ctx, int on);
/* Synchronisations since the context was created (diagnostics): out[0] ended
 * by the completion flag, out[1] by waiting for the stream. */
#define VRHIP_SYNC_INFO 2
int vrhip_sync_info(vrhip_ctx *ctx, uint64_t out[VRHIP_SYNC_INFO]);
/* Path groups per pixel for vrhip_render in sphere-only scenes (no
 * reference counterpart: a launch shape knob; mesh scenes use the persistent
 * path kernel, whose work queues need none).  A launch of k frames has 2k
 * paths per pixel; with groups > 1 they are split into that many contiguous
 * runs on different workgroups and summed in path order afterwards, so
 * results are unchanged.  0 (default) picks the smallest power of two that
 * gives every CU enough workgroups; 1 disables the split.  At most 128. */
int vrhip_set_path_split(vrhip_ctx *ctx, uint32_t groups);
/* Overlap of consecutive render launches (no reference counterpart: a
 * scheduling knob; results are unchanged).  The path kernels of launch i+1
 * may start on another of three internal path streams while launch i drains
 * its last paths; finish passes (accumulation, tonemap) stay in order on the
 * context stream, and any upload, tiling or stream change first waits for
 * the path streams.  mode 1: always, 0: never (launches run one after the
 * other), -1 (default): when a launch has fewer than 2^24 paths, or fewer
 * than 2^25 on a tiled rank (small or sharded frames, where the drain of a
 * launch is a large share of it). */
int vrhip_set_overlap(vrhip_ctx *ctx, int mode);
/* Render service (no reference counterpart: a scheduling mode; results are
 * unchanged bit for bit).  Consecutive vrhip_render calls of a mesh scene run
 * as one session on ONE persistent kernel: each launch is posted to a
 * descriptor ring the running kernel reads, so the drain of a launch (its
 * last, longest paths) overlaps the next launch's paths instead of ending a
 * kernel.  The images are summed, in path order, by one finish pass when the
 * session closes: at the next call on the context that is not vrhip_render or
 * vrhip_comm_gather (sync, read-back, upload, any setting, ...), when its 128
 * launch slots are used, or when a launch does not fit it (another scene,
 * camera or tiling, more frames than its slots hold).  vrhip_comm_gather
 * inside a session gathers the image as of that call when the session closes.
 * mode 1: every production mesh launch; 0: never; -1 (default, also
 * VRHIP_SERVICE): launches that overlap on the path streams (fewer than 2^24
 * paths, or 2^25 on a tiled rank) when the previous launch is still in flight
 * -- unsynchronised back-to-back calls, not the first call of a burst; also
 * whole frames of HDRI mesh scenes behind a launch in flight.  Launches whose
 * result slots the service's scratch budget (VRHIP_SERVICE_BYTES, default 24
 * GiB; a session's slots also take at most half of the device memory free when
 * it opens) cannot hold twice take the ordinary launch path in every mode, as
 * do the launches of a session whose scratch allocation fails.  The
 * open session's kernel retires after 20 ms without a new launch; a launch
 * posted while it retires is detected (a store-fence-load hand-shake on the
 * ring) and rendered through the launch path instead.
 * Gathers (vrhip_comm_gather) inside a session:
 *   mode -1 (automatic): the gather closes the session and is enqueued at
 *   once, like outside a session -- no collective ever waits on a later host
 *   call, whatever the caller does next.
 *   mode 1 (explicit): the gather is DEFERRED -- the image as of that call is
 *   staged by the session's finish pass and its ncclGather enqueued when the
 *   session closes, so consecutive steps keep one session (their drains
 *   overlap).  The caller then owns the ordering: a rank must close its
 *   session before it blocks on anything the other ranks' gathers wait for
 *   (a host barrier, a device-wide synchronise).  Calls that close a session:
 *   vrhip_sync, vrhip_read_accum/rgba8/depth8, vrhip_device_buffers,
 *   vrhip_gl_present, vrhip_pack_tiles/unpack_tiles, vrhip_last_kernel_ms,
 *   vrhip_kernel_stats, vrhip_debug_counters, vrhip_set_camera, vrhip_clear,
 *   every upload, vrhip_set_stream, vrhip_set_tiling, vrhip_set_service
 *   (and its timing / budget hooks), vrhip_comm_init/destroy, vrhip_destroy,
 *   the counting renders, and a vrhip_render that does not fit the session.
 *   Calls that do NOT close it: the flag setters (Cornell box, example sphere,
 *   BRDF, strict traversal, Fresnel -- the next vrhip_render then no longer
 *   fits and closes it), vrhip_set_overlap, vrhip_set_path_split,
 *   vrhip_set_kernel_timing, and the queries vrhip_frame_count,
 *   vrhip_last_launch_info, vrhip_owned_pixels, vrhip_service_stats/info,
 *   vrhip_device_group, vrhip_bvh_info, vrhip_get_stream. */
int vrhip_set_service(vrhip_ctx *ctx, int mode);
/* Render-service timing (test hook, no reference counterpart; 0 = default):
 * the session kernel's idle limit (20 ms), the host's window for posting to
 * an open session after its last post (5 ms), and a host delay inserted
 * between that window check and the post -- with a delay longer than the idle
 * limit every post after a session's first meets a retired kernel, which
 * exercises the hand-shake above.  Each at most 10 s. */
int vrhip_set_service_timing(vrhip_ctx *ctx, uint32_t idle_us, uint32_t post_window_us, uint32_t post_delay_us);
/* Scratch budget of the render service's launch slots on this context
 * (bytes; 0 = VRHIP_SERVICE_BYTES or 24 GiB).  A launch whose slot the budget
 * cannot hold twice takes the ordinary launch path. */
int vrhip_set_service_budget(vrhip_ctx *ctx, size_t bytes);
/* Launches that met a retiring session kernel and took the launch path
 * instead (since the context was created). */
int vrhip_service_stats(vrhip_ctx *ctx, uint64_t *refused_launches);
/* Render-service counts since the context was created (diagnostics; no
 * reference counterpart): out[0] launches refused by a retiring kernel (as
 * vrhip_service_stats), [1] sessions opened, [2] launches sessions took,
 * [3] gathers deferred to a session's close (explicit mode 1 only), [4]
 * sessions not opened because their scratch could not be allocated (those
 * launches took the launch path). */
#define VRHIP_SERVICE_INFO 5
int vrhip_service_info(vrhip_ctx *ctx, uint64_t out[VRHIP_SERVICE_INFO]);
/* Frames rendered since the last clear (vRendererCuda::getFrameCount,
 * include/vRendererCuda.h:124). */
int vrhip_frame_count(vrhip_ctx *ctx, uint32_t *frames);

/* ---- read-back -------------------------------------------------------- */
int vrhip_read_accum(vrhip_ctx *ctx, float *out_rgba_f32);       /* float4[W*H] */
int vrhip_read_rgba8(vrhip_ctx *ctx, uint8_t *out_rgba8);        /* uchar4[W*H] */
int vrhip_read_depth8(vrhip_ctx *ctx, uint8_t *out_rgba8);       /* uchar4[W*H] */
/* Device pointers of the resident buffers (for GL interop / RCCL gather). */
int vrhip_device_buffers(vrhip_ctx *ctx, void **accum, void **rgba8, void **depth8);

/* ---- multi-GPU image-tile sharding ------------------------------------ */
/* Render only the 16x16 tiles dealt to `rank`: rank r holds the tiles at
 * positions s = r, r + n_ranks, r + 2 n_ranks, ... of the dealing sequence,
 * and position s is the tile in row s / tiles_x, column
 * (s % tiles_x + s / tiles_x) % tiles_x (tiles_x = width / 16; each row
 * rotated by its index, ABI 5 -- ABI 4 dealt row-major, which gives every
 * rank fixed columns when tiles_x is a multiple of n_ranks); with
 * n_ranks == 1 the order stays row-major.  Every rank gets
 * the same number of tiles (+-1) spread over the whole image.
 * Seeds use global pixel coordinates, so the union of the ranks' tiles equals
 * the 1-GPU image bit for bit.  VRHIP_ERR_INVALID while a communicator
 * (vrhip_comm_init) with another tiling exists. */
int vrhip_set_tiling(vrhip_ctx *ctx, uint32_t rank, uint32_t n_ranks);
/* Host-only (no device): linear pixel indices (y * width + x) that rank
 * `rank` of n_ranks owns, in packed order (owned tile j holds packed pixels
 * [256j, 256j + 256), row-major inside the tile).  pix_out may be NULL to
 * query *n_pix. */
int vrhip_tile_pixels(uint32_t width, uint32_t height, uint32_t rank, uint32_t n_ranks, uint32_t *pix_out,
                      uint32_t *n_pix);
/* Number of pixels this rank owns (256 per owned tile). */
int vrhip_owned_pixels(vrhip_ctx *ctx, uint32_t *n_pix);
/* Pack this rank's owned pixels (RGBA8 if what == 0, float4 accum if 1,
 * depth8 if 2) contiguously into dst (device pointer), in packed order. */
int vrhip_pack_tiles(vrhip_ctx *ctx, int what, void *dst_device);
/* On the gathering rank: scatter n_ranks packed buffers from src (device;
 * rank r's buffer starts at r * stride_bytes, stride_bytes = 0 means
 * tightly packed) into this context's full image `what`. */
int vrhip_unpack_tiles(vrhip_ctx *ctx, int what, const void *src_device, uint32_t n_ranks, size_t stride_bytes);

/* ---- multi-GPU tile gather over RCCL (xGMI) ----------------------------- */
/* The reference is single-GPU; its per-pixel seeds use global pixel
 * coordinates (cuda/src/PathTracer.cu:817-818), so ranks rendering disjoint
 * tile sets reproduce the 1-GPU image bit for bit.  One process (or thread)
 * per GPU, one context per rank:
 *   rank 0: vrhip_comm_unique_id(id); hand `id` to every rank out of band
 *   (MPI, a file, a socket, torch.distributed ...);
 *   every rank: vrhip_comm_init(ctx, rank, n, id) -- joins the communicator
 *   (ncclCommInitRank: blocks until all n ranks have called it) and sets the
 *   tiling (vrhip_set_tiling(ctx, rank, n));
 *   per accumulation step, after vrhip_render: vrhip_comm_gather(ctx, what).
 * VRHIP_COMM_ID_BYTES = sizeof(ncclUniqueId). */
#define VRHIP_COMM_ID_BYTES 128
int vrhip_comm_unique_id(uint8_t id[VRHIP_COMM_ID_BYTES]);
int vrhip_comm_init(vrhip_ctx *ctx, uint32_t rank, uint32_t n_ranks, const uint8_t id[VRHIP_COMM_ID_BYTES]);
/* Every rank packs its tiles of image `what` (0 RGBA8, 1 float4 accumulation,
 * 2 depth8), ONE ncclGather brings them to rank 0, and rank 0 scatters them
 * into its full image -- all enqueued on the context stream behind the
 * render's finish passes (no host synchronisation).  Rank 0's image `what`
 * then holds the whole frame.  Inside a render-service session it closes the
 * session first (automatic service mode, the default), or, in explicit
 * service mode 1, is deferred to the session's close -- then call vrhip_sync
 * before any host-side barrier between ranks (vrhip_set_service). */
int vrhip_comm_gather(vrhip_ctx *ctx, int what);
/* Leaves the communicator (waits for the context stream first).  vrhip_destroy does it too. */
int vrhip_comm_destroy(vrhip_ctx *ctx);

/* ---- diagnostics ------------------------------------------------------ */
/* Kernel time of the last vrhip_render (ms, HIP events on the context stream;
 * requires vrhip_sync first; 0 with kernel timing off).  After a
 * render-service session: the session's span, from its kernel's start to its
 * finish pass's end (all its launches). */
int vrhip_last_kernel_ms(vrhip_ctx *ctx, float *ms);
/* Kernel timing (diagnostics; no reference counterpart): on (default; also
 * VRHIP_KERNEL_TIMING=1) the library records HIP events around each call and
 * around every launch's render kernels for vrhip_last_kernel_ms and
 * vrhip_kernel_stats; off, it records none on the launch path -- they sit
 * between the kernels on the stream and cost about 8 µs per synchronous
 * one-frame call (C2 0.712 -> 0.704 ms per frame), so a host at the
 * reference's one-frame cadence that does not read them turns them off. */
int vrhip_set_kernel_timing(vrhip_ctx *ctx, int on);
/* Accumulated render-kernel time (ms) and launch count since the last reset,
 * from HIP events recorded around every launch's render kernels
 * (primary_kernel + render_wave_kernel, or render_kernel) on the stream they
 * run on; the finish pass is not included.  With launch overlap a launch's
 * span includes time shared with the neighbouring launch.  Waits for the
 * pending launches. */
int vrhip_kernel_stats(vrhip_ctx *ctx, double *total_ms, uint64_t *launches, int reset);
/* Shape of the last production launch of vrhip_render (measurement; no
 * reference counterpart): path groups per pixel (sphere-only scenes), whether
 * the paths' results went through the result scratch and the finish pass (1)
 * or were accumulated in registers in path order (0), and the kernel family
 * (0 render_kernel, 1 path-pool kernel, 2 render service, 3 path-pool kernel
 * + finish pass as one graph launch: VRHIP_GRAPH=1, one-frame calls). */
int vrhip_last_launch_info(vrhip_ctx *ctx, uint32_t *split, uint32_t *use_scratch, uint32_t *kind);
/* Vector-memory gather roof of `device` (the ceiling the path kernel's
 * node, triangle and attribute fetches run against; no reference
 * counterpart): raw buffer loads of width_bytes (4, 8, 12 or 16) per lane
 * from a 1 MiB L2-resident table, 4 independent chains per lane, 8 waves per
 * SIMD on every CU, the 64 lanes of a wave reading `distinct` addresses
 * (1: one per wave-instruction ... 64: one per lane).  *lane_loads_per_s =
 * lane loads (one per active lane per instruction) per second, best of 3
 * warm launches.  Synchronous; a few ms. */
int vrhip_microbench_vmem(int device, uint32_t width_bytes, uint32_t distinct, double *lane_loads_per_s);
/* Raw debug slots: [0..7] the last counted render's counters; [8..13] phase
 * cycle totals (spheres, mesh traversal, hit materialisation, shading,
 * tonemap, whole kernel) written only by a -DVR_TIMING diagnostic build. */
int vrhip_debug_counters(vrhip_ctx *ctx, uint64_t out[16], int reset);
/* Depth of the uploaded BVH and the traversal stack size in use. */
int vrhip_bvh_info(vrhip_ctx *ctx, uint32_t *depth, uint32_t *n_nodes, uint32_t *n_slots);
/* Evaluate the device libm on n inputs (test hook: 0 sin, 1 cos, 2 acos,
 * 3 atan2, 4 pow, 5 fmin, 6 fmax, 7 f2i); a,b,out host arrays of n floats. */
int vrhip_selftest_math(int device, int fn, const float *a, const float *b, float *out, size_t n);
/* Compare the kernels' reciprocal (rcp_rn: v_rcp_f32 + one Newton step, used
 * for 1/det in the triangle test) with IEEE 1/x for every float bit pattern in
 * [lo_bits, hi_bits) and its negation (test hook; hi_bits <= 2^31).
 * *mismatches = count, *first_bad = smallest mismatching pattern or ~0u. */
int vrhip_selftest_rcp(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t *mismatches, uint32_t *first_bad);
/* The same for the kernels' square root (sqrt_rn: v_sqrt_f32 + the neighbour
 * tests of the IEEE expansion) against sqrtf, positive patterns only. */
int vrhip_selftest_sqrt(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t *mismatches, uint32_t *first_bad);
/* Exhaustive check of the table tonemap (no reference counterpart): the
 * colour byte the kernels take from the context's threshold table against
 * the byte of f2u8(pow(c, 1/2.2) * 255) (PathTracer.cu:850-866, the f64
 * pow), for every float bit pattern c in [lo_bits, hi_bits) (and -0.0 when
 * lo_bits is 0); the range [0, 0x3f800001) is every clamped channel value. */
int vrhip_selftest_tonemap(int device, uint32_t lo_bits, uint32_t hi_bits, uint64_t *mismatches, uint32_t *first_bad);

/* ---- host-side helpers (no device needed) ----------------------------- */
/* Native BVH build + reference flattening (src/vRendererCuda.cpp:204-279)
 * into caller arrays.  Call once with NULL outputs to get the sizes. */
int vrhip_build_flat(const float *positions, const float *normals, const float *tangents,
                     const float *uvs, uint32_t n_verts, const uint32_t *tris, uint32_t n_tris,
                     uint32_t max_leaf_tris,
                     float *bvh_out, size_t *n_bvh_f4,
                     float *verts_out, float *normals_out, float *tangents_out, float *uvs_out,
                     size_t *n_slots);
/* Check a flattened tree; returns VRHIP_OK and its depth / inner-node count. */
int vrhip_validate_flat(const float *bvh, size_t n_bvh_f4, const float *verts, size_t n_slots,
                        uint32_t *depth, uint32_t *n_nodes);

#ifdef __cplusplus
}
#endif
#endif /* VRHIP_H */
