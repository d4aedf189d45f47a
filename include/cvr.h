/*
 * cvr.h - C ABI of the MI355X volumetric path tracer (libcvr.so).
 *
 * This is the drop-in boundary for the reference's kernel-launcher layer
 * (Fe0437/CudaVolumeRenderer, implementation/src/RenderKernelLauncher.h:20-174)
 * and for the CudaVolPath driver above it (CudaVolPath.{h,cpp}).  Plain C
 * types only: pointers, sizes, status codes.  Every call returns 0 (CVR_OK) or
 * a negative CVR_ERR_* and never exits the process (the reference's
 * CHECK_CUDA_ERROR calls exit(), Debug.h:19-37); the message is available from
 * cvr_last_error().
 *
 * Unlike the reference, launch parameters live in a per-context struct passed
 * by value to the kernels (the reference keeps them in module-global
 * __constant__ symbols, RenderKernelLauncher.cu:67-72), so one process can
 * hold one context per GPU.
 */
#ifndef CVR_H_
#define CVR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CVR_ABI_VERSION 4  /* 3: cvr_render_frame takes the host buffer size; 4: cvr_stats.words */

enum {
  CVR_OK = 0,
  CVR_ERR_INVALID = -1,     /* bad argument */
  CVR_ERR_HIP = -2,         /* HIP runtime failure */
  CVR_ERR_STATE = -3,       /* call out of lifecycle order */
  CVR_ERR_IO = -4,          /* file / parse error */
  CVR_ERR_UNSUPPORTED = -5, /* kernel or feature not available */
  CVR_ERR_NOMEM = -6
};

/* Config::Kernel order and names (Config.h:87-95, :210-213). */
typedef enum {
  CVR_KERNEL_NAIVE_SK = 0,
  CVR_KERNEL_NAIVE_MK = 1,
  CVR_KERNEL_REGENERATION_SK = 2,
  CVR_KERNEL_STREAMING_MK = 3,
  CVR_KERNEL_STREAMING_SK = 4,
  CVR_KERNEL_SORTING_SK = 5,
  CVR_KERNEL_UNKNOWN = 6
} cvr_kernel;

/* Scene type names of the --scene-type flag (ConfigParser.cpp:16-18). */
typedef enum {
  CVR_SCENE_AUTO = 0,
  CVR_SCENE_MITSUBA_XML = 1,
  CVR_SCENE_VDB = 2,
  CVR_SCENE_RAW = 3,
  CVR_SCENE_MHD = 4,
  CVR_SCENE_VDB_SPARSE = 5 /* extension: read a VDB straight into 8^3 leaves (cvr_scene_sparse_medium);
                              Vdb/Auto do so by themselves above 2^30 voxels */
} cvr_scene_type;

/* Options for cvr_set_option. */
typedef enum {
  CVR_OPT_MAX_SEGMENTS = 1,   /* safety cap on segments per path (default 1<<20, 0 = none) */
  CVR_OPT_CHUNK = 2,          /* paths per wave dequeue (persistent schedulers); 0 (default): 256, the
                                 wave pool 64..256 by the paths each of its waves gets */
  CVR_OPT_EVENT_THRESHOLD = 3,/* lanes per wave that must wait before events run */
  CVR_OPT_GRID = 4,           /* persistent grid size in blocks (0 = occupancy); for the wave-pool scheduler in
                                 waves, rounded down to whole workgroups (four waves on sparse media) */
  CVR_OPT_SCATTER_EPS = 5,    /* -1 kernel default, 0 off, 1 on */
  CVR_OPT_SCHEDULER = 6,      /* how paths map onto threads: 0 single persistent kernel, 1 wavefront
                                 pair (streamingMK's multi-kernel structure), 2 workgroup path pool
                                 in LDS (streamingSK's block streaming), 3 wave-private path pool in
                                 LDS (the default for every kernel id; round 4 and before: naiveSK 4,
                                 streamingSK 2, streamingMK 1, naiveMK its own per-item kernel), 4 one
                                 path per work-item (naiveSK's structure; naiveMK: k_naive_mk).
                                 naiveMK runs the wave pool with 3 and k_naive_mk with any other
                                 value (its per-bounce kernels with CVR_OPT_MK_COMPACTION 1).  Scheduling only: results depend on the
                                 kernel id, not on the scheduler. */
  CVR_OPT_POOL = 7,           /* wavefront ray-slot pool size (default 2^21) */
  CVR_OPT_TIMING = 8,         /* 1: time every wavefront kernel (track_ms / events_ms) */
  CVR_OPT_CELLS = 9           /* 1 (default): corner-replicated density cells (8x density bytes
                                 in HBM, 2 x 16 B loads per Woodcock step); applies at set_medium */,
  CVR_OPT_WAVES = 10,         /* register/LDS budget in waves per SIMD: persistent kernel 4 (default), 5, 6,
                                 8; wave-pool kernel 3, 4, 5, 6 (default: 5; 6 is dense only
                                 and spills) */
  CVR_OPT_ORDER = 11,         /* 2 (default): 8x8-pixel blocks, samples innermost, each XCD band's blocks in
                                 2-D Morton order; 1: the same blocks row-major; 0: path-id order */
  CVR_OPT_QUEUES = 12,        /* work bands / queues, one per XCD (default 8) */
  CVR_OPT_BOUNDS = 13,        /* brick bounds: log2 brick size 1..5, 0 = off (default 2 dense,
                                 3 sparse; sparse caps at 3); next cvr_set_medium.  Results are
                                 identical either way. */
  CVR_OPT_TAIL = 14,          /* pool scheduler: lanes below which a wave ends a track phase (16) */
  CVR_OPT_BATCH = 15,         /* wave-pool scheduler: idle lanes that trigger a refill (8) */
  CVR_OPT_RNG_BINDING = 16,   /* regenerationSK: 0 (default) RNG bound to the path id (Q2 fixed:
                                 deterministic, scheduler-independent); 1 the reference's binding,
                                 Rng(seed + tid) per persistent thread, roulette draw after an
                                 escape, isect kept across a thread's paths
                                 (RegenerationVolPTsk_kernel.cuh:146-232).  streamingSK / sortingSK:
                                 1 runs the reference's block scheduler, 256-thread blocks with
                                 Rng(seed + gtid) per thread, one segment per iteration and a
                                 stable Morton-sort compaction that moves paths between threads
                                 (StreamingVolPTsk_kernel.cuh:328-349, SortingVolPTsk_kernel.cuh
                                 :306-330, its deferred albedo included).  streamingMK: 1 runs the
                                 reference's regenerate / extend kernel pair per iteration of a host
                                 loop, a new path's Rng(seed + path_id) becoming its thread's state
                                 and the states staying with the threads when compaction moves the
                                 paths (StreamingVolPTmk_kernel.cuh:26-253).  Thread-bound results
                                 depend on which thread takes which path: deterministic only for a
                                 one-wave (regenerationSK) or one-block (streaming/sorting/
                                 streamingMK) launch, CVR_OPT_GRID 1.  Reproduced quirk Q23
                                 (streamingSK / sortingSK): the sort key of an inactive thread is
                                 morton3D(1,1,1) = 2^30 - 1 (MortonSort.h:39-43), which an active
                                 path whose origin lies within 1/1024 of box_max on all three axes
                                 also gets; the stable tie-break on the thread index can then place
                                 that path past n_active, where the next regeneration overwrites it
                                 (dropped without a splat, not counted as truncated), as in the
                                 reference's cub sort.  streamingMK with 1 blocks the host until the
                                 render ends (one stream sync per iteration, as the reference's host
                                 loop). */
  CVR_OPT_MORTON = 17,         /* workgroup pool scheduler (CVR_OPT_SCHEDULER 2): 1 sorts each track phase's paths by the
                                 Morton code of their origin in the box (MortonSort.h:28-49,
                                 StreamingVolPTsk_kernel.cuh:188-216); default 0 (measured slower
                                 here).  Scheduling only: results are unchanged. */
  CVR_OPT_WORLD_TO_AABB = 18,  /* quirk Q4: 0 (default) the reference's worldToAABB, p - min/extent
                                 (operator precedence, Utilities.cuh:129-132); 1 the intended
                                 (p - min)/extent, computed as (p - box_min) * ((res - 1)/extent) (the
                                 grid scale folded in: shift = box_min, gx = (res - 1)/extent).  The two
                                 agree for the unit box of VDB/Raw/MHD scenes. */
  CVR_OPT_SUBQUEUES = 20,      /* wave-pool scheduler: work queues per XCD band (1..8, default 8), each
                                 over a contiguous part of the band, so that small dequeue chunks do not
                                 contend on one head.  Scheduling only. */
  CVR_OPT_INFLIGHT = 23,       /* wave-pool scheduler: renders the caller keeps in flight on this device
                                 (default 1).  Sets the grid of small launches (CVR_OPT_GRID 0): below 64
                                 paths per wave of the occupancy grid half of it (a quarter with renders
                                 in flight), below 1024 paths per wave half of it with renders in flight,
                                 else all of it.  Scheduling only. */
  CVR_OPT_UNIFORM_ALBEDO = 25, /* dense media: 1 (default) a grid whose voxels all hold the same rgb is
                                 read as that constant (the 8 taps interpolated with the same
                                 operations, no loads: the same result); 0 always load.  Takes
                                 effect at the next cvr_set_medium. */
  CVR_OPT_FRAME_FLUSH = 24,    /* cvr_render_frame, one part, wave-pool scheduler, pinned or registered
                                 host image: 1 (default) the launch itself stores each 8x8 block's
                                 normalised pixels into the host image once all its paths have
                                 ended (cvr_frame_flush_info); 0 normalise + copy after the launch.
                                 Same image either way (C2: 5.14 vs 5.29 ms per call).  2 (tests):
                                 the flushers give up at once, so the call takes its fallback copy. */
  CVR_OPT_SAMPLE_ORDER = 27,   /* wave-pool scheduler, pixel-block work order: 0 within an 8x8 block the
                                 units run sample by sample, the 64 pixels innermost; 1 pixel by pixel
                                 with the samples innermost, and each event batch sums its escapes per
                                 pixel before the framebuffer atomics (C3: 2.23 -> 0.99 GB written per
                                 launch; a launch with cvr_render_frame's in-launch output keeps
                                 order 0 and per-lane atomics).  -1 (default) = 0: order 1 costs C2 / C3 2.7% / 3.6%
                                 and C5 2.2% (with the empty-region mask).
                                 Scheduling and summation order only. */
  CVR_OPT_WAVE_PAIR = 26,      /* wave-pool scheduler, dense media with cells and bounds: 1 runs two waves
                                 per workgroup whose boundary and collision event lists are shared
                                 (k_wpair: either wave files into them and runs a batch from them; round
                                 5, 4.1x slower: profiles/round5/README.md); 0 (default) one wave per
                                 workgroup, private lists.  Only `make variant-pair` builds k_wpair: the
                                 in-tree libcvr.so refuses 1 with CVR_ERR_UNSUPPORTED.  Scheduling only:
                                 results are unchanged. */
  CVR_OPT_EMPTY_MASK = 28,     /* wave-pool scheduler, sparse media: 1 (default) each workgroup (four
                                 wave-private pools) stages the medium's empty-region mask (one bit per
                                 super-brick of whole leaves, 256 bytes) in LDS once for its waves, which
                                 load the brick word of a Woodcock point only when its super-brick holds
                                 density; 0 loads every point's word.  The words it skips are known
                                 (0): results are unchanged. */
  CVR_OPT_COUNT_WORDS = 29,    /* wave-pool scheduler, sparse media, 5 waves per SIMD: 1 runs the counting
                                 instance, which also counts the brick words its Woodcock points load
                                 into cvr_stats.words (the benchmark's exact algorithmic bytes; one
                                 more VGPR in the track loop, so not the benchmarked kernel); 0
                                 (default) counts nothing.  Results are unchanged. */
  /* 21: unused (a drain-time path migration between waves, measured slower: DESIGN.md §6) */
  CVR_OPT_DRAIN = 22,          /* wave-pool scheduler, once the queues are empty: an event batch runs as
                                 soon as the waiting segments x d >= the tracking ones (d = 0: only when
                                 no lane tracks, or 64 events wait).  -1 (default) = 1.  Scheduling only. */
  CVR_OPT_MK_COMPACTION = 19   /* quirk Q11, naiveMK only: 0 (default) every live path is extended
                                 until it ends; 1 the reference's compaction count end - begin - 1
                                 (RenderKernelLauncher.cu:266-271): after every bounce the live path
                                 with the highest pixel id is dropped, and a bounce that leaves no live
                                 path (the count underflows to 2^32 - 1 in the reference) fails the
                                 launch with CVR_ERR_STATE.  Runs the reference's per-bounce kernel
                                 sequence (one launch and host sync per bounce). */
} cvr_option;

/* HeterogeneousMedium + GGX boundary (Medium.h:110-190, Bsdf.h:17-30). */
typedef struct cvr_medium_desc {
  uint32_t res[3];        /* grid resolution x, y, z */
  const float* density;   /* host, res[0]*res[1]*res[2] fp32, x fastest */
  const float* albedo;    /* host, same grid, 4 floats per voxel (r,g,b,1) */
  float box_min[3];       /* AABB (density_AABB) */
  float box_max[3];
  float scale;            /* density scale (VDB 100, Raw 40) */
  float max_density;      /* majorant / scale */
  float g;                /* HG asymmetry; the reference never uploads it (Q7): 0 */
  float roughness[2];     /* GGX alpha (0.1, 0.1) */
  float eta;              /* int_ior / ext_ior (1.05f / 1.01f) */
} cvr_medium_desc;

/* Sparse medium (extension): the grid of cvr_medium_desc
 * stored as 8^3-voxel leaves (the OpenVDB leaf size).  Voxel (x,y,z) is
 * leaf_density[slot*512 + ((z&7)*8 + (y&7))*8 + (x&7)] with
 * slot = leaf_table[((z>>3)*leaf_dims[1] + (y>>3))*leaf_dims[0] + (x>>3)];
 * a slot of CVR_NO_LEAF means density 0 and albedo albedo_background for
 * all 512 voxels.  Rendering is identical to cvr_set_medium on the densified
 * grid: only the storage differs.  Replaces the reference's dense textures
 * (CudaVolPath.cpp:117-186) where they do not fit (a 2048x1024x2048 cloud is
 * 17 GB of fp32 density + 69 GB of float4 albedo dense). */
#define CVR_NO_LEAF 0xFFFFFFFFu
typedef struct cvr_sparse_medium_desc {
  uint32_t res[3];             /* index-space grid resolution (as cvr_medium_desc.res) */
  uint32_t leaf_dims[3];       /* ceil(res / 8) */
  const uint32_t* leaf_table;  /* host, leaf_dims product entries, x fastest: slot or CVR_NO_LEAF */
  uint32_t n_leaves;           /* slots in the pools */
  const float* leaf_density;   /* host, n_leaves * 512 fp32 */
  const float* leaf_albedo;    /* host, n_leaves * 512 * 4 fp32 (r,g,b,1), or NULL: albedo_background everywhere */
  float albedo_background[4];  /* albedo outside the leaves */
  float box_min[3];
  float box_max[3];
  float scale;
  float max_density;
  float g;
  float roughness[2];
  float eta;
} cvr_sparse_medium_desc;

typedef struct cvr_stats {
  uint64_t paths;      /* paths started */
  uint64_t segments;   /* loop iterations (RAYS_STATISTICS count) */
  uint64_t steps;      /* Woodcock steps drawn */
  uint64_t density;    /* density evaluations (8 fp32 taps each) */
  uint64_t albedo;     /* albedo evaluations (8 float4 taps each) */
  uint64_t escaped;    /* paths that splatted into the framebuffer */
  uint64_t truncated;  /* paths cut by CVR_OPT_MAX_SEGMENTS */
  double kernel_ms;    /* device time of the last launch (HIP events) */
  uint64_t iterations; /* wavefront: events/track kernel pairs of the last launch */
  double track_ms;     /* wavefront: summed device time of the tracking kernels (CVR_OPT_TIMING) */
  double events_ms;    /* wavefront: summed device time of the event kernels (CVR_OPT_TIMING) */
  uint64_t fetches;    /* density cells fetched (evaluations not settled by a brick bound) */
  uint64_t words;      /* sparse media: brick words loaded (the empty-region mask skips the
                          rest); counted only by launches with CVR_OPT_COUNT_WORDS 1, else 0 */
} cvr_stats;

typedef struct cvr_path_record {
  uint32_t image_id;
  uint32_t flags; /* bit0 escaped, bit1 truncated */
  float T[3];
  uint32_t n_segments, n_steps, n_density, n_albedo;
} cvr_path_record;

typedef struct cvr_ctx cvr_ctx;
typedef struct cvr_scene cvr_scene;

/* ---- lifecycle (RenderKernelLauncher.h:20-52) ------------------------- */
int cvr_create(int device, int kernel, cvr_ctx** out);
int cvr_destroy(cvr_ctx* ctx);
const char* cvr_last_error(const cvr_ctx* ctx); /* ctx may be NULL */
int cvr_abi_version(void);

/* setScene + createTextureWithVolume (CudaVolPath.cpp:88-186): copies the
 * host volumes into HBM (the caller keeps ownership of the host arrays). */
int cvr_set_medium(cvr_ctx* ctx, const cvr_medium_desc* medium);
/* Sparse upload: leaf pools go to HBM as they are; the density cells and
 * brick bounds are built on the device for the leaves whose cells can
 * interpolate a non-zero density (a brick-pool instead of dense cells). */
int cvr_set_medium_sparse(cvr_ctx* ctx, const cvr_sparse_medium_desc* medium);
/* Extension: `ctx` renders the medium of `src` (same device) without a copy:
 * its kernels read src's device buffers, which stay owned by src (destroy
 * `ctx` first, or give it a medium of its own, before `src` changes or frees
 * its medium).  For several contexts with renders in flight on one GPU. */
int cvr_share_medium(cvr_ctx* ctx, const cvr_ctx* src);
/* copyInvViewMatrix (12 floats), copyRasterToView, copyPixelIndexRange */
int cvr_set_camera(cvr_ctx* ctx, const float inv_view[12], const float raster_to_view[2],
                   const float full_res[2]);
/* setResolution(tile_dim) */
int cvr_set_resolution(cvr_ctx* ctx, uint32_t tile_w, uint32_t tile_h);
/* The tile resolution the context renders now (set by cvr_set_resolution, or
 * by cvr_render_image / cvr_render_tiles to their tile size): the size of the
 * host image cvr_render_frame writes (tile_w * tile_h float4).  Extension. */
int cvr_get_resolution(const cvr_ctx* ctx, uint32_t* tile_w, uint32_t* tile_h);
/* copyOffset(tile origin) */
int cvr_set_offset(cvr_ctx* ctx, uint32_t x, uint32_t y);
/* setNIterations: n_paths = tile_w * tile_h * iterations */
int cvr_set_iterations(cvr_ctx* ctx, uint32_t iterations);
/* Extension for sharding: launch only path ids [first, first+count) of the
 * tile's n_paths (default: all). */
int cvr_set_path_range(cvr_ctx* ctx, uint64_t first, uint64_t count);
/* Extension for multi-GPU strong scaling: restrict every launch to shard
 * `rank` of `world` of the tile's work.  Launches in the pixel-block work
 * order (whole samples of a tile whose sides are multiples of 8) take the
 * tile's 8x8 pixel blocks rank, rank + world, ... with all their samples, so
 * every shard sees the whole image and costs about the same; other launches
 * take a contiguous 1/world share of their path ids.  Either way the shards of
 * ranks 0..world-1 partition the launch's path ids, and the RNG stays bound
 * to the path id, so their summed images equal the unsharded render up to
 * fp32 summation order.  (0, 1) = no shard (default). */
int cvr_set_block_shard(cvr_ctx* ctx, uint32_t rank, uint32_t world);
/* Extension (scheduling only; results are bound to path ids): the order in
 * which the pixel-block work order hands out its blocks.  `perm` is a
 * permutation of [0, n) with n = the launch's block count (cvr_launch_blocks);
 * block b of the launch is taken as perm[b]'s turn.  Applies to launches with
 * that block count; NULL / n = 0 restores the natural order.  Used to start
 * costly blocks first (cvr_plan_block_order), so a launch does not end on
 * their long paths running on few lanes. */
int cvr_set_block_order(cvr_ctx* ctx, const uint32_t* perm, uint32_t n);
/* The pixel-block work order of the current launch configuration: its block
 * count (0 = not block ordered), its queues and their bands qbeg[0..n_queues]. */
int cvr_launch_blocks(const cvr_ctx* ctx, uint32_t* n_blocks, uint32_t* n_queues, uint32_t qbeg[9]);
/* RNG seed base (RegenerationVolPTsk_kernel.cuh:18 `seed`); path p uses
 * curand_init(seed + p). */
int cvr_set_seed(cvr_ctx* ctx, uint32_t seed);
int cvr_get_seed(const cvr_ctx* ctx, uint32_t* seed);
/* setOutputPtr: device float4 tile buffer; NULL selects a context-owned one. */
int cvr_set_output(cvr_ctx* ctx, void* device_tile_buffer);
void* cvr_output_ptr(cvr_ctx* ctx);
/* Run on a caller stream (hipStream_t), e.g. a framework's current stream;
 * NULL is the device's null stream.  cvr_own_stream() returns the
 * non-blocking stream the context creates for itself (the default). */
int cvr_set_stream(cvr_ctx* ctx, void* hip_stream);
void* cvr_own_stream(cvr_ctx* ctx);
int cvr_set_option(cvr_ctx* ctx, int option, int64_t value);
/* init(): occupancy-based launch sizing (Occupancy.cuh:24-70). */
int cvr_init(cvr_ctx* ctx);
/* launchRender(): asynchronous on the context stream; accumulates into the
 * output buffer. */
int cvr_launch_render(cvr_ctx* ctx);
/* reset(): synchronise, rewind the work queue, advance the seed by n_paths
 * for regenerationSK (RenderKernelLauncher.cu:353-361). */
int cvr_reset(cvr_ctx* ctx);
int cvr_synchronize(cvr_ctx* ctx);
/* memset of the tile buffer (CudaVolPath.cpp:194-209). */
int cvr_clear_output(cvr_ctx* ctx);
/* Counters of the last launch (RAYS_STATISTICS analogue) + its device time. */
int cvr_get_stats(cvr_ctx* ctx, cvr_stats* stats);
/* D->H copy of the tile buffer, every component divided by `scale`. */
int cvr_copy_output(cvr_ctx* ctx, float* host_rgba, float scale);
/* Extension, asynchronous on `stream` (a hipStream_t; NULL = the null
 * stream): host_dst[i] = device_src[i] / scale for n_floats floats, written by
 * a kernel straight into pinned (hipHostMalloc) or registered (hipHostRegister)
 * host memory: the transfer delegate's Scale + D->H copy
 * (ImageBufferTransfer.cu:61-78) in stream order, with no copy engine. */
int cvr_image_to_host(const float* device_src, float* host_dst, size_t n_floats, float scale, void* stream);
/* CudaVolPath::render for one tile (CudaVolPath.cpp:339-347, getImage
 * ImageBufferTransfer.cu:61-78): clear the framebuffer, render the context's
 * launch (resolution, iterations, camera, offset as set) and return once the
 * image, divided by the iteration count, is in `host_image` (width * height
 * float4; pinned memory makes the copy asynchronous).  parts 0 or 1: one
 * launch.  parts 2..3: the launch split into bands of 8-pixel block rows, the
 * largest first, each rendered with its own stream and work queues (helper
 * contexts that share this context's medium and framebuffer), so that a
 * band's normalise + copy runs while the later bands render; measured slower
 * on C2 (5.35 / 5.66 ms for 2 / 3 bands vs 5.37 for one launch: each band
 * adds ~0.15 ms of kernel span, more than its overlapped copy saves;
 * DESIGN.md §6).  Every path renders exactly as in one launch (the RNG is bound
 * to the path id).  Launches that cannot take bands (naive kernels, the
 * thread-bound RNG, sides that are not multiples of 8, partial path ranges,
 * block shards) render as one part.  Afterwards the seed has advanced as the
 * reference's reset() advances it (cvr_reset).  stats (may be NULL, which
 * saves a synchronous counter read per band): the summed counters;
 * kernel_ms = from the clear to the end of the last band.  With one part on
 * the wave-pool scheduler (5 waves per SIMD) and a pinned or registered host
 * image the copy happens inside the launch (CVR_OPT_FRAME_FLUSH, default on):
 * eight flusher waves store
 * each 8x8 block, normalised, as soon as all of its paths have ended, so the
 * image is complete when the kernel ends; if a flusher gives up (no block
 * finished for a second) the call copies the image the usual way instead.
 * host_floats: the floats host_image holds; fewer than tile_w * tile_h * 4
 * (cvr_get_resolution) is CVR_ERR_INVALID and nothing is rendered (ABI 3). */
int cvr_render_frame(cvr_ctx* ctx, float* host_image, size_t host_floats, uint32_t parts, cvr_stats* stats);
/* The last cvr_render_frame's in-launch output: blocks the flushers stored (0
 * if the call copied after the launch) and the number of calls so far that
 * fell back to the copy because a flusher gave up. */
int cvr_frame_flush_info(const cvr_ctx* ctx, uint32_t* blocks, uint32_t* fallbacks);
/* Extension (multi-GPU output): the pixels of block shard (rank, world) of a
 * width x height float4 image (cvr_set_block_shard: 8x8 blocks rank,
 * rank + world, ..., row-major; sides multiples of 8), divided by `scale`,
 * stored by a kernel on `stream` at their places in the full pinned or
 * registered host image `host_dst` (width * height * 4 floats).  The ranks'
 * block shards are pixel-disjoint, so every rank writing its own blocks into
 * one shared host image IS the reference's Scale + D->H copy
 * (ImageBufferTransfer.cu:61-78) of the whole render: no reduction. */
int cvr_blocks_to_host(const float* device_src, float* host_dst, uint32_t width, uint32_t height, uint32_t rank,
                       uint32_t world, float scale, void* stream);
/* Debug/parity: trace path ids [first, first+count) one per work-item and
 * return per-path records (no framebuffer splat). */
int cvr_trace_paths(cvr_ctx* ctx, uint32_t first, uint32_t count, cvr_path_record* host_out);
/* Debug: the production launch (cvr_launch_render on the wave-pool scheduler,
 * regenerationSK / sortingSK) writing every path's final record as it ends:
 * out[p - first] for the path ids p of the launch range [first, first + n_out)
 * (cvr_set_path_range; n_out must equal the range's length).  image_id, flags,
 * T and n_segments are filled (n_steps, n_density, n_albedo stay 0: the wave
 * pool counts those per lane); ids outside a block shard stay zero.
 * Synchronous.  The traced launch splats into a scratch buffer (the context's
 * output is untouched); cvr_get_stats afterwards reports its counters. */
int cvr_trace_launch(cvr_ctx* ctx, cvr_path_record* out, uint64_t n_out);
/* Diagnostic builds (-DCVR_STAMPS=1) only: per-phase cycle counters of the
 * persistent kernel {event cycles, track cycles, event phases, track
 * iterations}, summed over waves; zeros otherwise. */
int cvr_debug_counters(cvr_ctx* ctx, uint64_t out[16]);
/* Device properties used for sizing: CU count, persistent grid. */
int cvr_device_info(cvr_ctx* ctx, int* cu_count, int* persistent_grid);

/* ---- renderer (CudaVolPath::render, CudaVolPath.cpp:339-347) ---------- */
typedef struct cvr_render_desc {
  uint32_t resolution[2]; /* full image W, H */
  uint32_t n_tiles[2];    /* --number-of-tiles (TilingConfig, Config.h:61-78) */
  uint32_t iterations;    /* --iterations */
} cvr_render_desc;
/* Render all tiles: per tile set offset, launch, normalise by iterations
 * into the image, reset.  `device_image` (W*H float4, may be NULL) receives
 * the normalised image on the device, `host_image` (may be NULL) a copy.
 * Pixels outside tile_dim*n_tiles are not written (Q1).  stats->kernel_ms is
 * the sum of the tile launches' HIP-event times; one tile into host memory
 * only (no device_image) runs as cvr_render_frame, whose kernel_ms spans the
 * clear, the launch and its in-launch output. */
int cvr_render_image(cvr_ctx* ctx, const cvr_render_desc* desc, void* device_image, float* host_image,
                     cvr_stats* stats);
/* Tile-sharded variant (tile k -> GPU k): render only the
 * tiles k = first_tile, first_tile + tile_stride, ... of the same tile loop,
 * each with the seed it has in the full loop, so the per-rank images (zero
 * elsewhere when `device_image` starts zeroed) sum to cvr_render_image's.
 * The context's seed ends where the full loop leaves it.  Stats cover the
 * rendered tiles.  cvr_render_image == cvr_render_tiles(ctx, desc, 0, 1, ...). */
int cvr_render_tiles(cvr_ctx* ctx, const cvr_render_desc* desc, uint32_t first_tile, uint32_t tile_stride,
                     void* device_image, float* host_image, cvr_stats* stats);
/* Extension (multi-device renderer; the CLI's --devices): one
 * device's share of a render, stored normalised by a kernel straight into the
 * full pinned host image (cvr_host_alloc, or registered memory; width *
 * height * 4 floats, host_floats checked) at its places, nothing else written:
 *  - more than one tile (desc->n_tiles): tiles first_tile, first_tile +
 *    tile_stride, ... of the tile loop (tile k -> device k mod N,
 *    CudaVolPath.cpp:249-280), each with its sequential-loop seed;
 *  - one tile: the context's block shard (cvr_set_block_shard; sides multiples
 *    of 8; first_tile must be 0).
 * Disjoint shares from N contexts (one host thread each, any devices) leave
 * cvr_render_image's image in the one buffer, with no reduction.  Synchronous;
 * stats cover this share. */
int cvr_render_share_to_host(cvr_ctx* ctx, const cvr_render_desc* desc, uint32_t first_tile, uint32_t tile_stride,
                             float* host_image, size_t host_floats, cvr_stats* stats);
/* Pinned, device-mapped host memory for cvr_render_share_to_host /
 * cvr_render_frame's in-launch output (hipHostMalloc, mapped + portable: every
 * device can store into it), and its release. */
int cvr_host_alloc(size_t bytes, void** out);
int cvr_host_free(void* p);

/* ---- camera / tiling helpers ------------------------------------------ */
/* Default Camera (Camera.h:25-71, MITSUBA_COMPARABLE) after
 * setResolution(w,h), flattened as CudaVolPath::initCamera (CudaVolPath.cpp:67-85). */
int cvr_default_camera(uint32_t width, uint32_t height, float inv_view[12], float raster_to_view[2]);
/* TilingConfig (Config.h:61-78) + initTileArray (CudaVolPath.cpp:13-29). */
int cvr_tiling(uint32_t width, uint32_t height, uint32_t ntx, uint32_t nty, uint32_t tile_dim[2]);
int cvr_tile_origin(uint32_t tile_id, uint32_t ntx, const uint32_t tile_dim[2], uint32_t origin[2]);

/* ---- scenes (SceneBuilder family, Scene.h:56-81) ----------------------- */
/* Load a scene file: Raw (RawSceneBuilder.h), Vdb (VDBSceneBuilder.h), Mhd
 * (convert-mhd semantics), MitsubaXml.  AUTO picks by extension
 * (ConfigParser.cpp:79-97). */
int cvr_scene_load(const char* path, int scene_type, cvr_scene** out);
/* Extension: cvr_scene_load with options.  CVR_LOAD_DEFAULT_ALBEDO (quirk
 * Q17's flag): a VDB file without an "albedo" grid, which the reference
 * refuses (VDBAdapter.cpp:32-37), loads with albedo (r,g,b) everywhere, as
 * the dense grid or, sparse, as leaves without albedo over that background
 * (a wdas_cloud-style density-only file); files with an albedo grid are read
 * as before.  opts may be NULL (= cvr_scene_load). */
enum { CVR_LOAD_DEFAULT_ALBEDO = 1 };
typedef struct cvr_load_options {
  uint32_t flags;
  float default_albedo[3];
} cvr_load_options;
int cvr_scene_load_ex(const char* path, int scene_type, const cvr_load_options* opts, cvr_scene** out);
/* Synthetic proxies for the missing data blobs:
 * "bucky" (32^3 raw), "manix" (256x230x256 VDB-like), "hetvol" (128x128x50),
 * "cloud" (C5: sparse fBm cumulus in a 2048x1024x2048 index box, albedo
 * (1,1,1), stored sparse only).  dims may be NULL (default size). */
int cvr_scene_synthetic(const char* name, uint32_t seed, const uint32_t* dims, cvr_scene** out);
/* Medium description; pointers stay owned by the scene. */
int cvr_scene_medium(const cvr_scene* scene, cvr_medium_desc* out);
/* Sparse view of a scene: sparse scenes (the "cloud" proxy) are stored as
 * leaves; a dense scene is converted once (leaves holding any non-zero
 * density or an albedo other than the voxel (0,0,0)'s, which becomes the
 * background) and the leaves are kept in the scene.  Pointers stay valid
 * while the scene lives.  Dense scenes: cvr_scene_medium; a sparse scene has
 * no dense view (CVR_ERR_UNSUPPORTED). */
int cvr_scene_sparse_medium(cvr_scene* scene, cvr_sparse_medium_desc* out);
/* 1 if the scene is stored sparse only. */
int cvr_scene_is_sparse(const cvr_scene* scene);
/* The scene's camera at a render resolution: the fixed eye and orientation
 * of Camera.h:25-45 with the scene's horizontal fov (0.7 degrees for VDB,
 * Raw and MHD scenes; the XML sensor's fov, default 45, for Mitsuba scenes,
 * XmlSceneBuilder.h:120-150). */
int cvr_scene_camera(const cvr_scene* scene, uint32_t width, uint32_t height, float inv_view[12],
                     float raster_to_view[2]);
int cvr_scene_raw_bytes(const cvr_scene* scene, const uint8_t** bytes, size_t* n);
void cvr_scene_destroy(cvr_scene* scene);
/* Radiance RGBE .hdr of an RGBA float image (Image::saveHDR, Image.cpp:58-62). */
int cvr_write_hdr(const char* path, const float* rgba, uint32_t width, uint32_t height);
/* Kernel name <-> id (Config.h:210-213); unknown -> CVR_KERNEL_UNKNOWN. */
int cvr_kernel_from_name(const char* name);
const char* cvr_kernel_name(int kernel);

#ifdef __cplusplus
}
#endif
#endif /* CVR_H_ */
