// cvr_api.cpp - C ABI implementation: contexts (kernel launchers), device
// volume upload, the CudaVolPath tile loop, camera/tiling helpers.
//
// Reference map:
//   RenderKernelLauncher / VolPTKernelLauncher  RenderKernelLauncher.h:20-174,
//                                                RenderKernelLauncher.cu:86-361
//   CudaVolPath::render / runIterations / getImage / prepareForNextIterations
//                                                CudaVolPath.cpp:189-347
//   Camera + initCamera                          Camera.h:25-71, CudaVolPath.cpp:67-85
//   TilingConfig + initTileArray                 Config.h:61-78, CudaVolPath.cpp:13-29
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cvr.h"
#include "cvr_kernels.h"

namespace {

thread_local std::string g_last_error;

int set_err(std::string* dst, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  if (dst) *dst = buf;
  return code;
}

}  // namespace

namespace cvr {
void set_last_error(const std::string& msg) { g_last_error = msg; }

// Camera(res, fov_x) then setResolution(w, h) -> setFovFromX (Camera.h:25-71),
// and CudaVolPath::initCamera's rows of the model view (CudaVolPath.cpp:67-85).
void camera_for_fov(float fov_x, uint32_t w, uint32_t h, float inv_view[12], float r2v[2]) {
  const float fov_y = ((float)h / (float)w) * fov_x;
  r2v[0] = tanf(fov_x * CVR_PI_F / 360.f);
  r2v[1] = tanf(fov_y * CVR_PI_F / 360.f);
  // glm column-major model view: col0 right (1,0,0,0) [MITSUBA_COMPARABLE],
  // col1 up (0,-1,0,0), col2 view (0,0,-1,0), col3 position (0,0,100,1);
  // initCamera takes rows of its transpose's first three rows.
  const float mv[16] = {1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 0, 0, 0, 100.0f, 1};
  const int idx[12] = {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14};
  for (int i = 0; i < 12; ++i) inv_view[i] = mv[idx[i]];
}
}  // namespace cvr

struct cvr_ctx {
  int device = 0;
  int kernel = CVR_KERNEL_REGENERATION_SK;
  std::string err;

  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  bool timed = false;

  // medium in HBM
  float* d_density = nullptr;
  float4* d_albedo = nullptr;
  float4* d_cells = nullptr;  // corner-replicated density (MediumParams::cells)
  bool use_cells = true;
  bool uniform_albedo = true;  // CVR_OPT_UNIFORM_ALBEDO
  uint8_t* d_bounds = nullptr;  // brick bounds (MediumParams::bounds)
  uint32_t bound_shift = 2;     // log2 brick size, 0 = off
  bool bound_shift_set = false; // CVR_OPT_BOUNDS given (else sparse media use 8^3 bricks)
  size_t n_voxels = 0;
  // sparse medium (cvr_set_medium_sparse)
  uint32_t* d_leaves = nullptr;
  float* d_leaf_density = nullptr;
  float4* d_leaf_albedo = nullptr;
  uint32_t* d_sbounds = nullptr;
  uint32_t* d_emask = nullptr;       // empty-region mask (MediumParams::emask)
  uint32_t* d_block_perm = nullptr;  // cvr_set_block_order
  void* d_rec_active = nullptr;      // cvr_trace_launch: records of the launch in progress
  uint32_t block_perm_n = 0;
  size_t n_cell_leaves = 0;  // cell-leaf pool slots (incl. the zero slot)
  bool have_medium = false;
  cvr::MediumParams m{};

  // launcher state (the reference's __constant__ symbols)
  float inv_view[12] = {1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 100};
  float r2v[2] = {0, 0};
  float full_res[2] = {0, 0};
  bool have_camera = false;
  uint32_t tile_w = 0, tile_h = 0;
  uint32_t off[2] = {0, 0};
  uint32_t iterations = 1;
  uint64_t n_paths = 0;
  uint64_t range_first = 0, range_count = UINT64_MAX;
  uint32_t shard_rank = 0, shard_world = 1;  // cvr_set_block_shard
  uint32_t seed = 0;

  float4* d_out_owned = nullptr;
  size_t out_owned_px = 0;
  float4* d_out = nullptr;  // active output (owned or external)
  bool external_out = false;

  unsigned char* d_work = nullptr;  // queue heads + stats counters (kWork* layout)
  float4* d_pool_T = nullptr;       // wave-pool scheduler: event-only slot part (LaunchParams::pool_T)
  unsigned char* d_smk = nullptr;   // thread-bound streamingMK: slot buffers, flags, RNG states, counters
  size_t smk_n = 0;                 // threads d_smk is carved for
  size_t pool_T_n = 0;
  uint32_t n_queues = 8;            // work-order bands (one per XCD)
  uint32_t subqueues = 8;           // wave pool: queues per band (CVR_OPT_SUBQUEUES)
  int drain = -1;                   // wave pool: drain-mode event trigger (CVR_OPT_DRAIN; -1 = 1)
  int order = 2;                    // 1: pixel-block/sample-inner order when the launch allows it; 2: blocks
                                    // in 2-D Morton order within each band
  // cached Morton permutation of the launch's blocks (order 2), for the block layout in zkey
  uint32_t* d_zperm = nullptr;
  std::vector<uint32_t> h_zperm;
  uint64_t zkey[5] = {0, 0, 0, 0, 0};

  // options
  uint32_t max_segments = 1u << 20;
  uint32_t chunk = 0;  // paths per wave dequeue; 0: auto (wave pool: 64..256 by the launch's size, others 256)
  uint32_t ev_thresh = 56;
  uint32_t grid_override = 0;
  uint32_t inflight = 1;  // CVR_OPT_INFLIGHT: renders the caller keeps in flight (wave-pool grid rule)
  int scatter_eps = -1;
  int rng_binding = 0;  // CVR_OPT_RNG_BINDING
  int world_to_aabb = 0;  // CVR_OPT_WORLD_TO_AABB (Q4)
  int mk_compaction = 0;  // CVR_OPT_MK_COMPACTION (Q11)

  int cu_count = 0;
  int persistent_grid = 0;
  int pool_grid = 0;
  uint32_t pool_tail = 16;
  int wpool_grid = 0, wpool_grid_sparse = 0;
  // wave-pool register/LDS budget in waves per SIMD (CVR_OPT_WAVES: 3, 4, 5);
  // 0 = the default, 5 (dense and sparse, split slots)
  int wpool_waves = 0;
  int morton = 0;  // CVR_OPT_MORTON
  int wave_pair = 0;  // CVR_OPT_WAVE_PAIR
  int sample_order = -1;  // CVR_OPT_SAMPLE_ORDER (-1: the default, 0)
  int empty_mask = 1;     // CVR_OPT_EMPTY_MASK
  int count_words = 0;    // CVR_OPT_COUNT_WORDS
  uint32_t swap_batch = 8;
  int track_grid = 0;
  bool inited = false;
  int scheduler = -1;  // 0 persistent, 1 wavefront pair, 2 workgroup pool, 3 wave-private pool, -1 per kernel id
  int waves = 4;      // persistent kernel register budget (waves per SIMD)

  // wavefront pool (cvr_wavefront.hip)
  unsigned char* d_pool = nullptr;
  size_t pool_bytes = 0;
  uint32_t pool_cap = 0;  // slots the allocation holds
  uint32_t pool_max = 1u << 21;
  cvr::WfPool pool{};
  unsigned int* h_alive = nullptr;  // pinned ring of per-iteration flags
  std::vector<hipEvent_t> it_events;
  uint64_t last_iterations = 0;
  double last_track_ms = 0, last_events_ms = 0;
  bool wf_timing = false;

  cvr_stats last{};

  // cvr_render_frame: this launch's band of block rows (band_count 0: every block), the
  // helper contexts that render the frame's other bands (each with its own stream and work
  // queues, sharing this context's medium and framebuffer), the copy stream, and the
  // normalised device image the bands are copied from
  uint32_t band_first = 0, band_count = 0;
  std::vector<cvr_ctx*> frame_kids;
  hipStream_t frame_copy = nullptr;
  hipEvent_t frame_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // [0] cleared, [1 + k] band k rendered
  float4* d_frame = nullptr;
  size_t frame_px = 0;
  // cvr_render_frame's in-launch output (CVR_OPT_FRAME_FLUSH, wave pool): [FrameFlush
  // header | per-block ended-path counts], the flushers' status words (pinned), the
  // header as last written, and the counts the next launch takes (null: none)
  int frame_flush = 1;
  unsigned char* d_flush = nullptr;
  size_t flush_blocks = 0;
  unsigned int* h_flush_status = nullptr;
  cvr::FrameFlush flush_hdr{};
  bool flush_hdr_valid = false;  // d_flush holds flush_hdr
  unsigned int* frame_done_active = nullptr;
  uint32_t flush_last_blocks = 0, flush_fallbacks = 0;
};

using cvr::kWorkDebug;
using cvr::kWorkQueues;
using cvr::kWorkStats;
// d_work layout: cvr_kernels.h (stats, debug counters, queue heads)
constexpr size_t kWorkBytes = cvr::kWorkBytesBase;

#define HIP_TRY(ctx, expr)                                                                         \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess)                                                                               \
      return set_err((ctx) ? &(ctx)->err : nullptr, CVR_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

namespace {

bool kernel_supported(int k) { return k >= 0 && k < CVR_KERNEL_UNKNOWN; }

// Scheduler that implements each persistent kernel id (results
// depend only on the kernel id's scatter offset and per-tile seed, quirks
// Q2/Q6, so every id may run on any scheduler).  Round 5: every persistent id
// runs the wave-private LDS pool by default, its ballot/prefix compaction of
// finished segments being the streaming kernels' compaction
// (StreamingVolPTsk_kernel.cuh:176-216, StreamingVolPTmk_kernel.cuh:218-252)
// at wave granularity; sortingSK's event batches run sorted by kind; naiveSK
// (one thread per path in the reference, NaiveVolPTsk_kernel.cuh:17-87) runs
// there too: its image is fixed by its Rng(path_id) streams, scatter -eps and
// per-tile seeds, not by the thread mapping (C2: 4.5 vs 26.8 ms as one path
// per work-item).  The structural restatements stay behind CVR_OPT_SCHEDULER:
// 4 one path per work-item (k_naive, naiveSK's own mapping), 2 the workgroup
// pool with bulk compaction phases (StreamingVolPTsk's block streaming, 3-4x
// slower on C2), 1 the multi-kernel wavefront pair (StreamingVolPTmk's
// device-wide compaction), 0 one path per lane of a persistent wave.  naiveMK
// always runs its own kernels (k_naive_mk: per-bounce reseeding, Q12).
constexpr int kSchedPerItem = 4;
int scheduler_for(const cvr_ctx* c) {
  if (c->scheduler >= 0) return c->scheduler;
  return 3;
}

// Scatter origin offset per scheduler: every kernel subtracts
// d*eps at a real collision except single-thread regeneration
// (RegenerationVolPTsk_kernel.cuh:212).
bool scatter_eps_for(const cvr_ctx* c) {
  if (c->scatter_eps >= 0) return c->scatter_eps != 0;
  return c->kernel != CVR_KERNEL_REGENERATION_SK;
}

// streamingSK's default variant sorts its rays by Morton code (Q14,
// StreamingVolPTsk_kernel.cuh:188-216); here the pool scheduler's track order
// does so when CVR_OPT_MORTON is 1.  Off by default: the sort makes the pool
// kernel 8% slower on C2 and 7% on C3.
bool morton_for(const cvr_ctx* c) { return c->morton > 0; }

int wpool_waves_for(const cvr_ctx* c, bool sparse) {
  if (c->wpool_waves) return c->wpool_waves;
  return 5;  // dense and sparse (split slots: DESIGN.md §6)
}

// naiveMK runs the wave pool (k_wpool's kMedMK instances: d_init + d_extend per path, RNG
// re-seeded per bounce; C2 27.5 -> ~4.5 ms) unless another scheduler or budget is asked
// for, the reference's per-bounce compaction (CVR_OPT_MK_COMPACTION 1) or the in-launch
// output (cvr_render_frame then copies after the launch).
bool mk_on_wpool(const cvr_ctx* c) {
  return c->kernel == CVR_KERNEL_NAIVE_MK && scheduler_for(c) == 3 && !c->mk_compaction &&
         wpool_waves_for(c, c->m.leaves != nullptr) == 5;
}

// Wave-pool grid of a launch of n_paths (one wave per workgroup): CVR_OPT_GRID,
// else the occupancy grid, of which a small launch takes a part.  A launch of
// fewer than 64 paths per wave (C1: 262 K paths) ends mostly in ramp-up and
// ramp-down at the full grid: half the grid alone, a quarter with renders in
// flight (the other renders fill the rest; profiles/round2/overlap_c1.log:
// 0.228 vs 0.287 ms alone, 0.094 vs 0.149 ms per render with three in flight).
// With renders in flight (CVR_OPT_INFLIGHT > 1) a launch of fewer than 2048
// paths per wave at the full grid (the 8- and 4-GPU block shards of C2) takes
// half the grid, so each wave gets twice the paths (1/8 shard 0.700 vs 0.735
// ms per render, profiles/round2/overlap_small_shards.log; round 4, three in
// flight: 1/4 shard 1.282 vs 1.320 ms, 1/8 shard 0.724 vs 0.768 at 3/4 grid,
// profiles/round4/shard_grid.log); alone the full grid is faster.
// The grid counts waves, in whole workgroups of the instance (cvr::wpool_wpg).
uint32_t wpool_launch_grid(const cvr_ctx* c, uint64_t n_paths) {
  const uint32_t wpg = cvr::wpool_wpg(wpool_waves_for(c, c->m.leaves != nullptr), c->m.leaves != nullptr);
  auto whole = [wpg](uint32_t g) { return std::max(wpg, g / wpg * wpg); };
  if (c->grid_override) return whole(c->grid_override);
  const uint32_t full = (uint32_t)(c->m.leaves ? c->wpool_grid_sparse : c->wpool_grid);
  const uint32_t half = std::max(1u, full / 2), quarter = std::max(1u, full / 4);
  if (n_paths < 64ull * full) return whole(c->inflight > 1 ? quarter : half);
  if (c->inflight > 1 && n_paths < 2048ull * full) return whole(half);
  return whole(full);
}

int ensure_device(cvr_ctx* c) {
  HIP_TRY(c, hipSetDevice(c->device));
  return CVR_OK;
}

int ensure_output(cvr_ctx* c) {
  if (c->external_out) return CVR_OK;
  const size_t px = (size_t)c->tile_w * c->tile_h;
  if (px == 0) return set_err(&c->err, CVR_ERR_STATE, "resolution not set");
  if (c->out_owned_px < px) {
    // the old framebuffer may still be written by a launch in flight
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->d_out_owned) (void)hipFree(c->d_out_owned);
    c->d_out_owned = nullptr;
    HIP_TRY(c, hipMalloc(&c->d_out_owned, px * sizeof(float4)));
    HIP_TRY(c, hipMemsetAsync(c->d_out_owned, 0, px * sizeof(float4), c->stream));
    c->out_owned_px = px;
  }
  c->d_out = c->d_out_owned;
  return CVR_OK;
}

// FastDiv constants for d >= 1 (cvr_walk.h fastdiv): l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1, s1 = min(l, 1), s2 = max(l - 1, 0) (sh = s1 | s2 << 8).
static cvr::FastDiv make_fastdiv(uint32_t d) {
  if (d == 0) d = 1;
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d) ++l;
  cvr::FastDiv f;
  f.m = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
  f.sh = (l < 1 ? l : 1) | ((l > 1 ? l - 1 : 0) << 8);
  return f;
}

void fill_launch(const cvr_ctx* c, cvr::LaunchParams& L, uint64_t first, uint64_t count, bool sharded = true) {
  const uint32_t shard_world = sharded ? c->shard_world : 1u;
  const uint64_t P0 = (uint64_t)(uint32_t)((float)c->tile_w * (float)c->tile_h);
  // the persistent schedulers take work units through unit_to_path (pixel-block order); naiveSK/MK
  // and the wavefront pair map launch index -> path id directly
  const bool queued = (c->kernel != CVR_KERNEL_NAIVE_MK || mk_on_wpool(c)) && scheduler_for(c) != 1 &&
                      scheduler_for(c) != kSchedPerItem &&
                      c->rng_binding == 0;
  const bool block_order = queued && c->order && P0 && first % P0 == 0 && count % P0 == 0 && count > 0 &&
                           count / P0 <= (1ull << 20) && c->tile_w % 8 == 0 && c->tile_h % 8 == 0;
  if (shard_world > 1 && !block_order) {  // no block order: a contiguous share of the path ids
    const uint64_t base = count / c->shard_world, rem = count % c->shard_world;
    first += c->shard_rank * base + std::min<uint64_t>(c->shard_rank, rem);
    count = base + (c->shard_rank < rem ? 1 : 0);
  }
  memcpy(L.M, c->inv_view, sizeof(L.M));
  L.r2v[0] = c->r2v[0];
  L.r2v[1] = c->r2v[1];
  L.full_res[0] = c->full_res[0];
  L.full_res[1] = c->full_res[1];
  L.tile_res[0] = (float)c->tile_w;  // copyResolution(make_float2(res.x, res.y))
  L.tile_res[1] = (float)c->tile_h;
  L.off[0] = c->off[0];
  L.off[1] = c->off[1];
  L.tile_px = (uint32_t)(L.tile_res[0] * L.tile_res[1]);
  L.tile_w = (uint32_t)L.tile_res[0];
  L.path_first = (uint32_t)first;
  L.path_count = (uint32_t)count;
  L.seed_base = c->seed;
  L.max_segments = c->max_segments;
  L.out = c->d_out;
  L.queue = reinterpret_cast<unsigned int*>(c->d_work + kWorkQueues);
  L.stats = reinterpret_cast<unsigned long long*>(c->d_work + kWorkStats);
  L.chunk = c->chunk ? c->chunk : 256;
  L.ev_thresh = c->ev_thresh ? c->ev_thresh : 1;
  L.tail = c->pool_tail;
  L.batch = c->swap_batch;
  L.naive_mk = (c->kernel == CVR_KERNEL_NAIVE_MK ? 1u : 0u) | (morton_for(c) ? 2u : 0u);
  // work order (see LaunchParams): pixel blocks with samples innermost, one
  // contiguous band of blocks per queue, when the launch covers whole samples
  const uint64_t P = L.tile_px;
  // (at most 2^20 samples: cvr_walk.h unit_to_path's pixel-of-unit division)
  const bool aligned = P && first % P == 0 && count % P == 0 && count > 0 && count / P <= (1ull << 20);
  L.blk_off = 0;
  L.blk_stride = 1;
  if (c->order && aligned && c->tile_w % 8 == 0 && c->tile_h % 8 == 0) {
    L.order = 1;
    L.samples = (uint32_t)(count / P);
    L.blocks_x = c->tile_w / 8;
    L.n_blocks = (uint32_t)(P / 64);
    if (shard_world > 1 && block_order) {  // blocks shard_rank, shard_rank + world, ...
      L.blk_off = c->shard_rank;
      L.blk_stride = c->shard_world;
      L.n_blocks = L.n_blocks > c->shard_rank ? (L.n_blocks - c->shard_rank + c->shard_world - 1) / c->shard_world : 0;
      L.path_count = L.n_blocks * 64u * L.samples;
    } else if (c->band_count && block_order && c->band_first < L.n_blocks) {  // cvr_render_frame's band
      L.blk_off = c->band_first;
      L.n_blocks = std::min(c->band_count, L.n_blocks - c->band_first);
      L.path_count = L.n_blocks * 64u * L.samples;
    }
    uint32_t bands = c->n_queues < L.n_blocks ? c->n_queues : L.n_blocks;
    if (bands == 0) bands = 1;
    // sub-queues per band: the wave pool only, each with at least one block
    // Sub-queues per band (8 by default: C2 5.03 vs 5.07 ms with one, manix 2048^2 28.9 vs
    // 29.2; C3 prefers one, 5.56 vs 5.60; profiles/round3/ab/sub3_*.log, c4sub.log)
    uint32_t sub = scheduler_for(c) == 3 ? c->subqueues : 1u;
    while (sub > 1 && bands * sub > L.n_blocks) --sub;
    L.sub = sub;
    L.n_queues = bands * sub;
  } else {
    L.order = 0;
    L.samples = 0;
    L.blocks_x = 0;
    L.n_blocks = 0;
    L.n_queues = 1;
    L.sub = 1;
  }
  L.div_queues = make_fastdiv(L.n_queues);
  L.block_perm = (L.order == 1 && c->d_block_perm && c->block_perm_n == L.n_blocks) ? c->d_block_perm : nullptr;
  L.div_tile_px = make_fastdiv(L.tile_px);
  L.div_tile_w = make_fastdiv(L.tile_w);
  L.div_block = make_fastdiv(64u * L.samples);
  L.div_blocks_x = make_fastdiv(L.blocks_x);
}

// The medium as the kernels see it for this context's options: with the Q4
// fix (CVR_OPT_WORLD_TO_AABB 1) the Woodcock coordinate is (p - min) scaled by
// (res - 1)/extent instead of p - min/extent (cvr_walk.h MediumParams::gx).
cvr::MediumParams launch_medium(const cvr_ctx* c) {
  cvr::MediumParams m = c->m;
  if (!c->empty_mask) m.emask = nullptr;  // every super-brick loads its words
  if (c->world_to_aabb) {
    const float ex = m.bmax.x - m.bmin.x, ey = m.bmax.y - m.bmin.y, ez = m.bmax.z - m.bmin.z;
    m.shift = m.bmin;
    m.gx = m.agx / ex;
    m.gy = m.agy / ey;
    m.gz = m.agz / ez;
  }
  return m;
}

// First block of queue q of a launch (LaunchParams::n_queues; cvr_walk.h queue_blocks_begin).
uint32_t queue_begin(const cvr::LaunchParams& L, uint32_t q) {
  return (uint32_t)((uint64_t)L.n_blocks * q / L.n_queues);
}
// First block of XCD band b (n_queues / sub bands of sub queues each).
uint32_t band_begin(const cvr::LaunchParams& L, uint32_t b) { return queue_begin(L, b * L.sub); }

int check_ready(cvr_ctx* c) {
  if (!c->have_medium) return set_err(&c->err, CVR_ERR_STATE, "medium not set (cvr_set_medium)");
  if (!c->have_camera) return set_err(&c->err, CVR_ERR_STATE, "camera not set (cvr_set_camera)");
  if (c->tile_w == 0 || c->tile_h == 0) return set_err(&c->err, CVR_ERR_STATE, "resolution not set");
  return CVR_OK;
}

int do_init(cvr_ctx* c) {
  if (c->inited) return CVR_OK;
  int r = ensure_device(c);
  if (r) return r;
  hipDeviceProp_t prop;
  HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
  c->cu_count = prop.multiProcessorCount;
  int bpc = 0;
  HIP_TRY(c, cvr::persistent_occupancy(scatter_eps_for(c), c->waves, &bpc));
  if (bpc < 1) bpc = 1;
  c->persistent_grid = bpc * c->cu_count;
  int pbpc = 0;
  HIP_TRY(c, cvr::pool_occupancy(scatter_eps_for(c), &pbpc));
  if (pbpc < 1) pbpc = 1;
  c->pool_grid = pbpc * c->cu_count;
  int wbpc = 0;
  HIP_TRY(c, cvr::wpool_occupancy(scatter_eps_for(c), wpool_waves_for(c, false), false, &wbpc));
  if (wbpc < 1) wbpc = 1;
  c->wpool_grid = wbpc * c->cu_count;
  HIP_TRY(c, cvr::wpool_occupancy(scatter_eps_for(c), wpool_waves_for(c, true), true, &wbpc));
  if (wbpc < 1) wbpc = 1;
  c->wpool_grid_sparse = wbpc * c->cu_count;
  int tbpc = 0;
  HIP_TRY(c, cvr::wf_track_occupancy(&tbpc));
  if (tbpc < 1) tbpc = 1;
  c->track_grid = tbpc * c->cu_count;
  c->inited = true;
  return CVR_OK;
}

constexpr uint32_t kAliveRing = 8;

// Carve the SoA pool + per-wave cursors/stat rows out of one allocation.
int ensure_pool(cvr_ctx* c, uint32_t n) {
  n = (n + 255u) & ~255u;
  const uint32_t ev_waves = n / 64u;
  const uint32_t tr_waves = (uint32_t)c->track_grid * 4u;
  const size_t slot_bytes = 19 * sizeof(uint32_t);  // 11 floats + 6 rng + img + meta
  const size_t need = (size_t)n * slot_bytes + (size_t)ev_waves * 8 + 256 + kAliveRing * 4 + 256 +
                      (size_t)(ev_waves + tr_waves) * 64 + 4096;
  if (need > c->pool_bytes) {
    if (c->d_pool) (void)hipFree(c->d_pool);
    c->d_pool = nullptr;
    c->pool_bytes = 0;
    HIP_TRY(c, hipMalloc(&c->d_pool, need));
    c->pool_bytes = need;
  }
  if (!c->h_alive) HIP_TRY(c, hipHostMalloc(&c->h_alive, kAliveRing * sizeof(unsigned int), hipHostMallocDefault));
  unsigned char* p = c->d_pool;
  auto take = [&](size_t bytes) {
    unsigned char* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return r;
  };
  cvr::WfPool& P = c->pool;
  float** fl[] = {&P.ox, &P.oy, &P.oz, &P.dx, &P.dy, &P.dz, &P.tx, &P.ty, &P.tz, &P.dist, &P.t};
  for (float** f : fl) *f = reinterpret_cast<float*>(take((size_t)n * 4));
  uint32_t** ui[] = {&P.r0, &P.r1, &P.r2, &P.r3, &P.r4, &P.rd, &P.img, &P.meta};
  for (uint32_t** u : ui) *u = reinterpret_cast<uint32_t*>(take((size_t)n * 4));
  P.cursor = reinterpret_cast<uint32_t*>(take((size_t)ev_waves * 8));
  P.head = reinterpret_cast<unsigned int*>(take(256));
  P.alive = reinterpret_cast<unsigned int*>(take(kAliveRing * 4));
  P.stats_events = reinterpret_cast<unsigned long long*>(take((size_t)ev_waves * 64));
  P.stats_track = reinterpret_cast<unsigned long long*>(take((size_t)tr_waves * 64));
  P.n = n;
  c->pool_cap = n;
  return CVR_OK;
}

// The wavefront render of one launch: events / track alternate until no
// slot is alive.  The host polls the alive flags every few iterations.
int wf_render(cvr_ctx* c, const cvr::LaunchParams& L, bool eps) {
  uint32_t n = L.path_count < c->pool_max ? L.path_count : c->pool_max;
  if (n < 256) n = 256;
  int r = ensure_pool(c, n);
  if (r) return r;
  cvr::WfPool P = c->pool;
  const uint32_t ev_waves = P.n / 64u;
  const uint32_t tr_waves = (uint32_t)c->track_grid * 4u;
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemsetAsync(P.meta, 0, (size_t)P.n * 4, s));  // WF_FREE
  HIP_TRY(c, hipMemsetAsync(P.cursor, 0, (size_t)ev_waves * 8, s));
  HIP_TRY(c, hipMemsetAsync(P.head, 0, 256, s));
  HIP_TRY(c, hipMemsetAsync(P.stats_events, 0, (size_t)ev_waves * 64, s));
  HIP_TRY(c, hipMemsetAsync(P.stats_track, 0, (size_t)tr_waves * 64, s));
  uint32_t it = 0;
  bool done = false;
  if (c->wf_timing && c->it_events.empty()) {
    c->it_events.resize(3 * 512);
    for (auto& e : c->it_events) HIP_TRY(c, hipEventCreate(&e));
  }
  double track_ms = 0, events_ms = 0;
  uint32_t timed_its = 0;
  while (!done) {
    cvr::WfPool Pi = P;
    Pi.alive = P.alive + (it % kAliveRing);
    HIP_TRY(c, hipMemsetAsync(Pi.alive, 0, 4, s));
    const bool tm = c->wf_timing && timed_its < 512;
    if (tm) HIP_TRY(c, hipEventRecord(c->it_events[3 * timed_its], s));
    HIP_TRY(c, cvr::wf_launch_events(launch_medium(c), L, Pi, eps, s));
    if (tm) HIP_TRY(c, hipEventRecord(c->it_events[3 * timed_its + 1], s));
    HIP_TRY(c, cvr::wf_launch_track(launch_medium(c), L, Pi, (uint32_t)c->track_grid, s));
    if (tm) {
      HIP_TRY(c, hipEventRecord(c->it_events[3 * timed_its + 2], s));
      ++timed_its;
    }
    HIP_TRY(c, hipMemcpyAsync(c->h_alive + (it % kAliveRing), Pi.alive, 4, hipMemcpyDeviceToHost, s));
    ++it;
    if (it % 4 == 0) {
      HIP_TRY(c, hipStreamSynchronize(s));
      for (uint32_t k = it - 4; k < it; ++k)
        if (c->h_alive[k % kAliveRing] == 0) done = true;
    }
    if (it > 100000) return set_err(&c->err, CVR_ERR_STATE, "wavefront render did not converge");
  }
  for (uint32_t k = 0; k < timed_its; ++k) {
    float a = 0, b = 0;
    HIP_TRY(c, hipEventElapsedTime(&a, c->it_events[3 * k], c->it_events[3 * k + 1]));
    HIP_TRY(c, hipEventElapsedTime(&b, c->it_events[3 * k + 1], c->it_events[3 * k + 2]));
    events_ms += a;
    track_ms += b;
  }
  // fold the per-wave counters into the context's 8 stats words
  unsigned long long* stats = reinterpret_cast<unsigned long long*>(c->d_work + kWorkStats);
  HIP_TRY(c, cvr::wf_launch_reduce(P.stats_events, ev_waves, stats, s));
  HIP_TRY(c, cvr::wf_launch_reduce(P.stats_track, tr_waves, stats + 8, s));
  c->last_iterations = it;
  c->last_track_ms = track_ms;
  c->last_events_ms = events_ms;
  return CVR_OK;
}

// naiveMK with the reference's compaction count (quirk Q11 reproduced,
// CVR_OPT_MK_COMPACTION 1): NaiveVolPTmk::launchRender / extend
// (RenderKernelLauncher.cu:183-272).  Per iteration: d_init over the tile,
// then bounces while the processed count is non-zero; after each bounce the
// count is (live paths) - 1 and the live path with the highest pixel id (last
// in the stable remove_if's output) is never extended again.  A bounce that
// leaves no live path makes the reference's uint count wrap to 2^32 - 1 (its
// next extend reads stale active-list entries, its remove_if runs off the
// array): reported as CVR_ERR_STATE.  One host sync per bounce, as the
// reference's thrust call.
int mk_reference_render(cvr_ctx* c, const cvr::LaunchParams& L) {
  if (L.path_first != 0 || L.tile_px == 0 || L.path_count % L.tile_px != 0 || c->shard_world != 1)
    return set_err(&c->err, CVR_ERR_UNSUPPORTED,
                   "naiveMK with the reference compaction renders whole tiles only (no path range / shard)");
  const uint32_t iters = L.path_count / L.tile_px;
  const cvr::MediumParams m = launch_medium(c);
  float4* st = nullptr;
  uint32_t* live = nullptr;
  cvr::MkCtl* ctl = nullptr;
  HIP_TRY(c, hipMalloc(&st, (size_t)L.tile_px * 3 * sizeof(float4)));
  hipError_t e = hipMalloc(&live, (size_t)L.tile_px * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&ctl, sizeof(cvr::MkCtl));
  int r = CVR_OK;
  for (uint32_t it = 0; it < iters && e == hipSuccess && r == CVR_OK; ++it) {
    e = cvr::launch_mk_init(m, L, it, st, live, c->stream);
    uint64_t n_processed = L.tile_px;
    for (uint32_t depth = 0; n_processed != 0 && e == hipSuccess; ++depth) {
      if (e == hipSuccess) e = hipMemsetAsync(ctl, 0, sizeof(cvr::MkCtl), c->stream);
      if (e == hipSuccess) e = cvr::launch_mk_extend(m, L, it, depth, st, live, ctl, c->stream);
      cvr::MkCtl h{};
      if (e == hipSuccess) e = hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) break;
      if (h.count == 0) {
        r = set_err(&c->err, CVR_ERR_STATE,
                    "naiveMK reference compaction (Q11): iteration %u bounce %u left no live path, so "
                    "end - begin - 1 underflows (RenderKernelLauncher.cu:271)",
                    it, depth);
        break;
      }
      n_processed = h.count - 1u;
      e = hipMemsetAsync(live + h.max_id, 0, sizeof(uint32_t), c->stream);  // dropped, never extended again
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(st);
  if (live) (void)hipFree(live);
  if (ctl) (void)hipFree(ctl);
  if (r) return r;
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "naiveMK reference compaction: %s", hipGetErrorString(e));
  return CVR_OK;
}

// streamingMK with the thread-bound RNG (CVR_OPT_RNG_BINDING 1):
// StreamingVolPTmk::launchRender (RenderKernelLauncher.cu:435-470).  Per
// iteration d_regenerate fills the slots from n_active on, n_active is reset,
// the slot buffers swap and d_extend runs one segment per active path (all of
// them once the head has passed the last path) and compacts the survivors;
// the host reads n_active and the head back, one sync per iteration as the
// reference.  The RNG states stay with the threads (cvr_kernels.hip
// k_smk_extend).  Buffers: 2 x 3 float4 + 2 flags per slot, 24 bytes of RNG
// state per thread and two counters, carved from one allocation that stays
// with the context (grown only when the grid grows).  Like the reference's
// host loop, a call blocks the host until the render has ended.
int smk_thread_render(cvr_ctx* c, const cvr::LaunchParams& L, uint32_t grid) {
  if (L.path_count == 0) return CVR_OK;
  const size_t n = (size_t)grid * 256u;
  const cvr::MediumParams m = launch_medium(c);
  if (c->smk_n < n) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->d_smk) (void)hipFree(c->d_smk);
    c->d_smk = nullptr;
    c->smk_n = 0;
    // float4 slots | uint4 states | uint2 states | flags | counters (every part 16-byte aligned)
    const size_t bytes = 6 * n * sizeof(float4) + n * sizeof(uint4) + n * sizeof(uint2) + ((2 * n + 15) & ~(size_t)15) + 16;
    HIP_TRY(c, hipMalloc(&c->d_smk, bytes));
    c->smk_n = n;
  }
  unsigned char* p = c->d_smk;
  float4* slots = reinterpret_cast<float4*>(p);
  p += 6 * n * sizeof(float4);
  uint4* st0 = reinterpret_cast<uint4*>(p);
  p += n * sizeof(uint4);
  uint2* st1 = reinterpret_cast<uint2*>(p);
  p += n * sizeof(uint2);
  uint8_t* act = p;
  p += (2 * n + 15) & ~(size_t)15;
  uint32_t* ctl = reinterpret_cast<uint32_t*>(p);
  hipError_t e = hipMemsetAsync(ctl, 0, 2 * sizeof(uint32_t), c->stream);  // d_n_active = head = 0
  cvr::SmkSlots buf[2] = {{slots, slots + n, slots + 2 * n, act}, {slots + 3 * n, slots + 4 * n, slots + 5 * n, act + n}};
  int cur = 0;  // the buffer d_regenerate writes and the next d_extend reads
  uint32_t h[2] = {(uint32_t)n, 0u};
  uint64_t it = 0;
  int r = CVR_OK;
  while (e == hipSuccess && (h[0] > 0u || h[1] < L.path_count)) {
    if (++it > 100000000ull) {
      r = set_err(&c->err, CVR_ERR_STATE, "thread-bound streamingMK did not finish");
      break;
    }
    e = cvr::launch_smk_regen(L, buf[cur], st0, st1, ctl, grid, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(ctl, 0, sizeof(uint32_t), c->stream);  // d_n_active = 0
    if (e == hipSuccess) e = cvr::launch_smk_extend(m, L, buf[cur], buf[cur ^ 1], st0, st1, ctl, grid, c->stream);
    cur ^= 1;
    if (e == hipSuccess) e = hipMemcpyAsync(h, ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  }
  c->last_iterations = (uint32_t)it;
  if (r) return r;
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "thread-bound streamingMK: %s", hipGetErrorString(e));
  return CVR_OK;
}

void compute_range(const cvr_ctx* c, uint64_t* first, uint64_t* count) {
  uint64_t f = c->range_first < c->n_paths ? c->range_first : c->n_paths;
  uint64_t n = c->n_paths - f;
  if (c->range_count < n) n = c->range_count;
  *first = f;
  *count = n;
}

}  // namespace

extern "C" {

int cvr_abi_version(void) { return CVR_ABI_VERSION; }

const char* cvr_last_error(const cvr_ctx* ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return g_last_error.c_str();
}

int cvr_create(int device, int kernel, cvr_ctx** out) {
  if (!out) return set_err(nullptr, CVR_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (kernel < 0 || kernel >= CVR_KERNEL_UNKNOWN)
    return set_err(nullptr, CVR_ERR_INVALID, "unknown kernel id %d", kernel);
  if (!kernel_supported(kernel))
    return set_err(nullptr, CVR_ERR_UNSUPPORTED, "kernel %s is not implemented yet", cvr_kernel_name(kernel));
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return set_err(nullptr, CVR_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= ndev) return set_err(nullptr, CVR_ERR_INVALID, "device %d out of range", device);
  cvr_ctx* c = new cvr_ctx();
  c->device = device;
  c->kernel = kernel;
  auto fail = [&](const char* what, hipError_t err) {
    int r = set_err(nullptr, CVR_ERR_HIP, "%s: %s", what, hipGetErrorString(err));
    cvr_destroy(c);
    return r;
  };
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking)) != hipSuccess)
    return fail("hipStreamCreate", e);
  c->stream = c->own_stream;
  if ((e = hipEventCreate(&c->ev_start)) != hipSuccess) return fail("hipEventCreate", e);
  if ((e = hipEventCreate(&c->ev_stop)) != hipSuccess) return fail("hipEventCreate", e);
  if ((e = hipMalloc(&c->d_work, kWorkBytes)) != hipSuccess) return fail("hipMalloc(work)", e);
  // stats words: [64,128) single-kernel launches / wavefront events, [128,192) wavefront track
  if ((e = hipMemset(c->d_work, 0, kWorkBytes)) != hipSuccess) return fail("hipMemset(work)", e);
  *out = c;
  return CVR_OK;
}

static void free_sparse(cvr_ctx* c);

int cvr_destroy(cvr_ctx* c) {
  if (!c) return CVR_OK;
  (void)hipSetDevice(c->device);
  // the frame helpers first: their launches read this context's medium and framebuffer
  for (cvr_ctx* k : c->frame_kids) cvr_destroy(k);
  c->frame_kids.clear();
  if (c->frame_copy) (void)hipStreamSynchronize(c->frame_copy);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_density) (void)hipFree(c->d_density);
  if (c->d_albedo) (void)hipFree(c->d_albedo);
  if (c->d_cells) (void)hipFree(c->d_cells);
  if (c->d_bounds) (void)hipFree(c->d_bounds);
  free_sparse(c);
  if (c->d_out_owned) (void)hipFree(c->d_out_owned);
  if (c->d_work) (void)hipFree(c->d_work);
  if (c->d_pool_T) (void)hipFree(c->d_pool_T);
  if (c->d_smk) (void)hipFree(c->d_smk);
  if (c->d_block_perm) (void)hipFree(c->d_block_perm);
  if (c->d_zperm) (void)hipFree(c->d_zperm);
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->d_pool) (void)hipFree(c->d_pool);
  if (c->h_alive) (void)hipHostFree(c->h_alive);
  for (auto& e : c->it_events) (void)hipEventDestroy(e);
  for (auto& e : c->frame_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->frame_copy) (void)hipStreamDestroy(c->frame_copy);
  if (c->d_frame) (void)hipFree(c->d_frame);
  if (c->d_flush) (void)hipFree(c->d_flush);
  if (c->h_flush_status) (void)hipHostFree(c->h_flush_status);
  delete c;
  return CVR_OK;
}

static void free_sparse(cvr_ctx* c) {
  if (c->d_leaves) (void)hipFree(c->d_leaves);
  if (c->d_leaf_density) (void)hipFree(c->d_leaf_density);
  if (c->d_leaf_albedo) (void)hipFree(c->d_leaf_albedo);
  if (c->d_sbounds) (void)hipFree(c->d_sbounds);
  if (c->d_emask) (void)hipFree(c->d_emask);
  c->d_emask = nullptr;
  c->d_leaves = nullptr;
  c->d_leaf_density = nullptr;
  c->d_leaf_albedo = nullptr;
  c->d_sbounds = nullptr;
  c->n_cell_leaves = 0;
}

// Geometry, scale and BSDF parameters shared by the dense and sparse uploads
// (HeterogeneousMedium + GGX, Medium.h:110-190).
static void fill_medium_common(cvr::MediumParams& m, const uint32_t res[3], const float box_min[3],
                               const float box_max[3], float scale, float max_density, float g,
                               const float roughness[2], float eta) {
  m.rx = res[0];
  m.ry = res[1];
  m.rz = res[2];
  m.rxy = res[0] * res[1];  // only used by dense media, where it is < 2^24
  m.fres_x = (float)res[0];
  m.fres_y = (float)res[1];
  m.fres_z = (float)res[2];
  m.gx = m.agx = (float)(res[0] - 1u);
  m.gy = m.agy = (float)(res[1] - 1u);
  m.gz = m.agz = (float)(res[2] - 1u);
  m.bmin = cvr::V3{box_min[0], box_min[1], box_min[2]};
  m.bmax = cvr::V3{box_max[0], box_max[1], box_max[2]};
  const float ex = box_max[0] - box_min[0], ey = box_max[1] - box_min[1], ez = box_max[2] - box_min[2];
  m.shift = cvr::V3{box_min[0] / ex, box_min[1] / ey, box_min[2] / ez};
  m.scale = scale;
  m.inv_sigma = 1.0f / (scale * max_density);
  m.g = g;
  m.ax = roughness[0];
  m.ay = roughness[1];
  m.eta = eta;
  m.inv_eta = 1.0f / eta;
}

int cvr_set_medium(cvr_ctx* c, const cvr_medium_desc* md) {
  if (!c || !md) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  if (!md->density || !md->albedo) return set_err(&c->err, CVR_ERR_INVALID, "density/albedo is NULL");
  if (md->res[0] == 0 || md->res[1] == 0 || md->res[2] == 0)
    return set_err(&c->err, CVR_ERR_INVALID, "empty grid");
  const size_t n = (size_t)md->res[0] * md->res[1] * md->res[2];
  if (n > 0xFFFFFFFFull) return set_err(&c->err, CVR_ERR_INVALID, "grid exceeds 2^32 voxels");
  // the kernels index cells and bricks with 24-bit multiplies
  if ((uint64_t)md->res[1] * md->res[2] >= (1ull << 24) || (uint64_t)md->res[0] * md->res[1] >= (1ull << 24))
    return set_err(&c->err, CVR_ERR_UNSUPPORTED, "dense grid with y*z or x*y >= 2^24: use cvr_set_medium_sparse");
  int r = ensure_device(c);
  if (r) return r;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  free_sparse(c);
  if (n != c->n_voxels || !c->d_density) {
    if (c->d_density) (void)hipFree(c->d_density);
    if (c->d_albedo) (void)hipFree(c->d_albedo);
    c->d_density = nullptr;
    c->d_albedo = nullptr;
    HIP_TRY(c, hipMalloc(&c->d_density, n * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->d_albedo, n * sizeof(float4)));
    c->n_voxels = n;
  }
  HIP_TRY(c, hipMemcpy(c->d_density, md->density, n * sizeof(float), hipMemcpyHostToDevice));
  HIP_TRY(c, hipMemcpy(c->d_albedo, md->albedo, n * sizeof(float4), hipMemcpyHostToDevice));
  if (c->d_cells) (void)hipFree(c->d_cells);
  c->d_cells = nullptr;
  if (c->use_cells) {
    HIP_TRY(c, hipMalloc(&c->d_cells, 2 * n * sizeof(float4)));
    HIP_TRY(c, cvr::launch_build_cells(c->d_density, md->res[0], md->res[1], md->res[2], c->d_cells, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  if (c->d_bounds) (void)hipFree(c->d_bounds);
  c->d_bounds = nullptr;
  const float sigma = md->scale * md->max_density;
  uint32_t bnx = 0, bny = 0, bsentinel = 0;
  if (c->bound_shift && sigma > 0.0f && std::isfinite(sigma) && md->scale > 0.0f) {
    const uint32_t B = 1u << c->bound_shift;
    bnx = (md->res[0] + B - 1) / B;
    bny = (md->res[1] + B - 1) / B;
    const size_t nb = (size_t)bnx * bny * ((md->res[2] + B - 1) / B);
    bsentinel = (uint32_t)nb;  // the no-bound entry past the last brick (k_build_bounds writes it)
    HIP_TRY(c, hipMalloc(&c->d_bounds, nb + 1));
    HIP_TRY(c, cvr::launch_build_bounds(c->d_density, md->res[0], md->res[1], md->res[2], c->bound_shift,
                                        md->max_density, c->d_bounds, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  cvr::MediumParams& m = c->m;
  m = cvr::MediumParams{};
  m.bounds = c->d_bounds;
  m.bshift = c->bound_shift;
  m.bnx = bnx;
  m.bny = bny;
  m.bnxy = bnx * bny;
  m.bsentinel = bsentinel;
  m.cells = c->d_cells;
  m.density = c->d_density;
  m.albedo = c->d_albedo;
  fill_medium_common(m, md->res, md->box_min, md->box_max, md->scale, md->max_density, md->g, md->roughness,
                     md->eta);
  if (c->uniform_albedo) {
    // every voxel's rgb bit-identical to the first (the XML smoke scene's constant albedo)
    bool same = true;
    for (size_t i = 1; i < n && same; ++i) same = memcmp(md->albedo + 4 * i, md->albedo, 3 * sizeof(float)) == 0;
    if (same) {
      m.albedo_uniform = 1u;
      m.albedo_bg = cvr::V3{md->albedo[0], md->albedo[1], md->albedo[2]};
    }
  }
  c->have_medium = true;
  return CVR_OK;
}

int cvr_set_medium_sparse(cvr_ctx* c, const cvr_sparse_medium_desc* sd) {
  if (!c || !sd) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  const uint32_t* res = sd->res;
  if (res[0] == 0 || res[1] == 0 || res[2] == 0) return set_err(&c->err, CVR_ERR_INVALID, "empty grid");
  for (int k = 0; k < 3; ++k)
    if (sd->leaf_dims[k] != (res[k] + 7u) / 8u)
      return set_err(&c->err, CVR_ERR_INVALID, "leaf_dims[%d] = %u, expected ceil(res/8) = %u", k, sd->leaf_dims[k],
                     (res[k] + 7u) / 8u);
  const uint32_t lnx = sd->leaf_dims[0], lny = sd->leaf_dims[1], lnz = sd->leaf_dims[2];
  const size_t nleaf = (size_t)lnx * lny * lnz;
  if (nleaf > 0xFFFFFFFFull) return set_err(&c->err, CVR_ERR_INVALID, "leaf table exceeds 2^32 entries");
  if (!sd->leaf_table || (sd->n_leaves && !sd->leaf_density))
    return set_err(&c->err, CVR_ERR_INVALID, "leaf table / density pool is NULL");
  // cell leaves: a leaf's cells read the corners in it and its forward
  // neighbours, so it needs a slot iff one of those 8 leaves exists
  std::vector<uint32_t> cell_slot(nleaf, 0u), coords{0u, 0u, 0u};  // slot 0: the zero leaf
  for (uint32_t z = 0; z < lnz; ++z)
    for (uint32_t y = 0; y < lny; ++y)
      for (uint32_t x = 0; x < lnx; ++x) {
        const size_t i = ((size_t)z * lny + y) * lnx + x;
        const uint32_t v = sd->leaf_table[i];
        if (v != CVR_NO_LEAF && v >= sd->n_leaves)
          return set_err(&c->err, CVR_ERR_INVALID, "leaf table entry %u >= n_leaves %u", v, sd->n_leaves);
        bool any = false;
        for (uint32_t dz = 0; dz < 2 && !any; ++dz)
          for (uint32_t dy = 0; dy < 2 && !any; ++dy)
            for (uint32_t dx = 0; dx < 2 && !any; ++dx)
              if (x + dx < lnx && y + dy < lny && z + dz < lnz)
                any = sd->leaf_table[((size_t)(z + dz) * lny + (y + dy)) * lnx + (x + dx)] != CVR_NO_LEAF;
        if (any) {
          cell_slot[i] = (uint32_t)(coords.size() / 3);
          coords.insert(coords.end(), {x, y, z});
        }
      }
  const size_t ncl = coords.size() / 3;
  if (ncl > (1u << 24))
    return set_err(&c->err, CVR_ERR_UNSUPPORTED, "sparse medium needs %zu cell leaves (> 2^24)", ncl);
  int r = ensure_device(c);
  if (r) return r;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // drop the previous medium (dense or sparse)
  if (c->d_density) (void)hipFree(c->d_density);
  if (c->d_albedo) (void)hipFree(c->d_albedo);
  if (c->d_cells) (void)hipFree(c->d_cells);
  if (c->d_bounds) (void)hipFree(c->d_bounds);
  c->d_density = nullptr;
  c->d_albedo = nullptr;
  c->d_cells = nullptr;
  c->d_bounds = nullptr;
  c->n_voxels = 0;
  c->have_medium = false;
  free_sparse(c);
  const size_t np = (size_t)sd->n_leaves * 512;
  HIP_TRY(c, hipMalloc(&c->d_leaves, nleaf * sizeof(uint32_t)));
  HIP_TRY(c, hipMemcpy(c->d_leaves, sd->leaf_table, nleaf * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(&c->d_leaf_density, (np ? np : 1) * sizeof(float)));
  if (np) HIP_TRY(c, hipMemcpy(c->d_leaf_density, sd->leaf_density, np * sizeof(float), hipMemcpyHostToDevice));
  if (sd->leaf_albedo && np) {
    HIP_TRY(c, hipMalloc(&c->d_leaf_albedo, np * sizeof(float4)));
    HIP_TRY(c, hipMemcpy(c->d_leaf_albedo, sd->leaf_albedo, np * sizeof(float4), hipMemcpyHostToDevice));
  }
  cvr::MediumParams& m = c->m;
  m = cvr::MediumParams{};
  fill_medium_common(m, res, sd->box_min, sd->box_max, sd->scale, sd->max_density, sd->g, sd->roughness, sd->eta);
  m.leaves = c->d_leaves;
  m.leaf_density = c->d_leaf_density;
  m.leaf_albedo = c->d_leaf_albedo;
  m.lnx = lnx;
  m.lny = lny;
  m.albedo_bg = cvr::V3{sd->albedo_background[0], sd->albedo_background[1], sd->albedo_background[2]};
  // bricks of 2^bshift <= 8 cells (within one leaf); bounds off -> q = 255
  const float sigma = sd->scale * sd->max_density;
  const int unbounded = !(c->bound_shift && sigma > 0.0f && std::isfinite(sigma) && sd->scale > 0.0f);
  // Default 8^3 cells per brick: one brick word per leaf's cells (C5: 33.6 MB
  // of words instead of 268 MB at 4^3, so they stay in L2 / Infinity Cache;
  // 12% faster at an unchanged fetch rate, clouds being empty or dense).
  m.bshift = !c->bound_shift_set ? 3u : c->bound_shift == 0 ? 2u : std::min(c->bound_shift, 3u);
  const uint32_t B = 1u << m.bshift;
  m.bnx = (res[0] + B - 1) / B;
  m.bny = (res[1] + B - 1) / B;
  const uint32_t bnz = (res[2] + B - 1) / B;
  const size_t nb = (size_t)m.bnx * m.bny * bnz;
  m.bnxy = m.bnx * m.bny;
  if ((uint64_t)m.bnx * m.bny >= (1ull << 24) || nb >= 0xFFFFFFFFull)
    return set_err(&c->err, CVR_ERR_UNSUPPORTED, "sparse grid has too many bricks (%zu)", nb);
  m.bsentinel = (uint32_t)nb;  // the no-bound word past the last brick (k_build_sparse_bounds writes it)
  HIP_TRY(c, hipMalloc(&c->d_sbounds, (nb + 1) * sizeof(uint32_t)));
  if (c->use_cells) HIP_TRY(c, hipMalloc(&c->d_cells, ncl * 1024 * sizeof(float4)));
  uint32_t *d_coords = nullptr, *d_slot = nullptr;
  hipError_t e = hipMalloc(&d_coords, coords.size() * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&d_slot, nleaf * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(d_coords, coords.data(), coords.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_slot, cell_slot.data(), nleaf * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = cvr::launch_build_sparse(m, d_coords, c->use_cells ? ncl : 0, d_slot, bnz, sd->max_density, unbounded,
                                 c->d_cells, c->d_sbounds, c->stream);
  // Empty-region mask (MediumParams::emask): the smallest super-brick of 2^es
  // cells per axis whose grid, each axis padded to a power of two, fits 32
  // kEmaskWords bits; bit set iff a leaf in it has a cell leaf.  Clear
  // super-bricks' brick words are 0 only when bounded.
  if (e == hipSuccess && !unbounded) {
    auto log2up = [](uint32_t v) {
      uint32_t l = 0;
      while ((1u << l) < v) ++l;
      return l;
    };
    uint32_t es = 3, lx = log2up(lnx), ly = log2up(lny), lz = log2up(lnz);
    while (lx + ly + lz > log2up(32u * cvr::kEmaskWords)) {
      ++es;
      lx -= lx > 0;
      ly -= ly > 0;
      lz -= lz > 0;
    }
    std::vector<uint32_t> em(cvr::kEmaskWords, 0u);
    const uint32_t k = es - 3;
    for (uint32_t z = 0; z < lnz; ++z)
      for (uint32_t y = 0; y < lny; ++y)
        for (uint32_t x = 0; x < lnx; ++x)
          if (cell_slot[((size_t)z * lny + y) * lnx + x] != 0u) {
            const uint32_t b = (z >> k) << (lx + ly) | (y >> k) << lx | (x >> k);
            em[b >> 5] |= 1u << (b & 31u);
          }
    e = hipMalloc(&c->d_emask, em.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpy(c->d_emask, em.data(), em.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    m.eshift = es;
    m.eshy = lx;
    m.eshz = lx + ly;
    m.emask = c->d_emask;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (d_coords) (void)hipFree(d_coords);
  if (d_slot) (void)hipFree(d_slot);
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "sparse medium build: %s", hipGetErrorString(e));
  m.cells = c->d_cells;
  m.sbounds = c->d_sbounds;
  c->n_cell_leaves = ncl;
  c->have_medium = true;
  return CVR_OK;
}

int cvr_share_medium(cvr_ctx* c, const cvr_ctx* src) {
  if (!c || !src) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  if (c == src) return CVR_OK;
  if (!src->have_medium) return set_err(&c->err, CVR_ERR_STATE, "source context has no medium");
  if (src->device != c->device)
    return set_err(&c->err, CVR_ERR_INVALID, "source context is on device %d, not %d", src->device, c->device);
  int r = ensure_device(c);
  if (r) return r;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // drop this context's own medium; the kernels read the source's buffers
  if (c->d_density) (void)hipFree(c->d_density);
  if (c->d_albedo) (void)hipFree(c->d_albedo);
  if (c->d_cells) (void)hipFree(c->d_cells);
  if (c->d_bounds) (void)hipFree(c->d_bounds);
  c->d_density = nullptr;
  c->d_albedo = nullptr;
  c->d_cells = nullptr;
  c->d_bounds = nullptr;
  c->n_voxels = 0;
  free_sparse(c);
  c->m = src->m;
  c->n_cell_leaves = src->n_cell_leaves;
  c->have_medium = true;
  c->inited = false;
  return CVR_OK;
}

int cvr_set_camera(cvr_ctx* c, const float inv_view[12], const float r2v[2], const float full_res[2]) {
  if (!c || !inv_view || !r2v || !full_res) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  memcpy(c->inv_view, inv_view, sizeof(c->inv_view));
  c->r2v[0] = r2v[0];
  c->r2v[1] = r2v[1];
  c->full_res[0] = full_res[0];
  c->full_res[1] = full_res[1];
  c->have_camera = true;
  return CVR_OK;
}

int cvr_set_resolution(cvr_ctx* c, uint32_t w, uint32_t h) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (w == 0 || h == 0) return set_err(&c->err, CVR_ERR_INVALID, "zero tile resolution");
  if ((uint64_t)w * h > (1ull << 24))
    return set_err(&c->err, CVR_ERR_INVALID, "tile of %ux%u exceeds 2^24 pixels (float pixel indexing)", w, h);
  if ((uint64_t)w * h * c->iterations > 0xFFFFFFFFull)
    return set_err(&c->err, CVR_ERR_INVALID, "n_paths = %llu exceeds the reference's uint32 path ids",
                   (unsigned long long)((uint64_t)w * h * c->iterations));
  c->tile_w = w;
  c->tile_h = h;
  c->n_paths = (uint64_t)w * h * c->iterations;
  return ensure_output(c);
}

int cvr_get_resolution(const cvr_ctx* c, uint32_t* w, uint32_t* h) {
  if (!c || !w || !h) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  *w = c->tile_w;
  *h = c->tile_h;
  return CVR_OK;
}

int cvr_set_offset(cvr_ctx* c, uint32_t x, uint32_t y) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  c->off[0] = x;
  c->off[1] = y;
  return CVR_OK;
}

int cvr_set_iterations(cvr_ctx* c, uint32_t it) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  const uint64_t np = (uint64_t)c->tile_w * c->tile_h * it;
  if (np > 0xFFFFFFFFull)
    return set_err(&c->err, CVR_ERR_INVALID, "n_paths = %llu exceeds the reference's uint32 path ids",
                   (unsigned long long)np);
  c->iterations = it;
  c->n_paths = np;
  return CVR_OK;
}

int cvr_set_path_range(cvr_ctx* c, uint64_t first, uint64_t count) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  c->range_first = first;
  c->range_count = count;
  return CVR_OK;
}

int cvr_set_block_shard(cvr_ctx* c, uint32_t rank, uint32_t world) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (world == 0 || rank >= world) return set_err(&c->err, CVR_ERR_INVALID, "bad shard %u of %u", rank, world);
  c->shard_rank = rank;
  c->shard_world = world;
  return CVR_OK;
}

int cvr_set_block_order(cvr_ctx* c, const uint32_t* perm, uint32_t n) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (c->d_block_perm) (void)hipFree(c->d_block_perm);
  c->d_block_perm = nullptr;
  c->block_perm_n = 0;
  if (!perm || n == 0) return CVR_OK;  // natural order
  std::vector<uint8_t> seen(n, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (perm[i] >= n || seen[perm[i]])
      return set_err(&c->err, CVR_ERR_INVALID, "block order is not a permutation of [0, %u)", n);
    seen[perm[i]] = 1;
  }
  int r = ensure_device(c);
  if (r) return r;
  HIP_TRY(c, hipMalloc(&c->d_block_perm, (size_t)n * sizeof(uint32_t)));
  HIP_TRY(c, hipMemcpy(c->d_block_perm, perm, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice));
  c->block_perm_n = n;
  return CVR_OK;
}

int cvr_launch_blocks(const cvr_ctx* c, uint32_t* n_blocks, uint32_t* n_queues, uint32_t qbeg[9]) {
  if (!c || !n_blocks || !n_queues || !qbeg) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  cvr::LaunchParams L{};
  uint64_t first = 0, count = 0;
  compute_range(c, &first, &count);
  fill_launch(c, L, first, count);
  *n_blocks = L.order == 1 ? L.n_blocks : 0;
  const uint32_t bands = L.n_queues / L.sub;
  *n_queues = bands;
  for (uint32_t q = 0; q < 9; ++q) qbeg[q] = q <= bands ? band_begin(L, q) : L.n_blocks;
  return CVR_OK;
}

int cvr_set_seed(cvr_ctx* c, uint32_t seed) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  c->seed = seed;
  return CVR_OK;
}

int cvr_get_seed(const cvr_ctx* c, uint32_t* seed) {
  if (!c || !seed) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  *seed = c->seed;
  return CVR_OK;
}

int cvr_set_output(cvr_ctx* c, void* p) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (p) {
    c->d_out = static_cast<float4*>(p);
    c->external_out = true;
    return CVR_OK;
  }
  c->external_out = false;
  if (c->tile_w && c->tile_h) return ensure_output(c);
  c->d_out = nullptr;
  return CVR_OK;
}

void* cvr_output_ptr(cvr_ctx* c) { return c ? c->d_out : nullptr; }

int cvr_set_stream(cvr_ctx* c, void* s) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  c->stream = static_cast<hipStream_t>(s);  // NULL = the device's null stream
  return CVR_OK;
}

void* cvr_own_stream(cvr_ctx* c) { return c ? (void*)c->own_stream : nullptr; }

int cvr_set_option(cvr_ctx* c, int opt, int64_t v) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  switch (opt) {
    case CVR_OPT_MAX_SEGMENTS:
      if (v < 0) return set_err(&c->err, CVR_ERR_INVALID, "max_segments < 0");
      c->max_segments = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_CHUNK:
      if (v < 1 || v > (1 << 20)) return set_err(&c->err, CVR_ERR_INVALID, "chunk out of range");
      c->chunk = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_EVENT_THRESHOLD:
      if (v < 1 || v > 64) return set_err(&c->err, CVR_ERR_INVALID, "event threshold must be 1..64");
      c->ev_thresh = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_GRID:
      if (v < 0) return set_err(&c->err, CVR_ERR_INVALID, "grid < 0");
      c->grid_override = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_SCHEDULER:
      if (v < 0 || v > kSchedPerItem) return set_err(&c->err, CVR_ERR_INVALID, "scheduler must be 0..4");
      c->scheduler = (int)v;
      return CVR_OK;
    case CVR_OPT_POOL:
      if (v < 256 || v > (1 << 26)) return set_err(&c->err, CVR_ERR_INVALID, "pool size out of range");
      c->pool_max = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_TIMING:
      c->wf_timing = v != 0;
      return CVR_OK;
    case CVR_OPT_ORDER:
      if (v < 0 || v > 2) return set_err(&c->err, CVR_ERR_INVALID, "order must be 0, 1 or 2");
      c->order = (int)v;
      return CVR_OK;
    case CVR_OPT_QUEUES:
      if (v < 1 || v > 8) return set_err(&c->err, CVR_ERR_INVALID, "queues must be 1..8");
      c->n_queues = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_SUBQUEUES:
      if (v < 1 || v > 8) return set_err(&c->err, CVR_ERR_INVALID, "subqueues must be 1..8");
      c->subqueues = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_INFLIGHT:
      if (v < 1 || v > 64) return set_err(&c->err, CVR_ERR_INVALID, "inflight must be 1..64");
      c->inflight = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_FRAME_FLUSH:
      if (v < 0 || v > 2) return set_err(&c->err, CVR_ERR_INVALID, "frame flush must be 0, 1 or 2");
      c->frame_flush = (int)v;
      return CVR_OK;
    case CVR_OPT_DRAIN:
      if (v < -1 || v > 64) return set_err(&c->err, CVR_ERR_INVALID, "drain must be -1..64");
      c->drain = (int)v;
      return CVR_OK;
    case CVR_OPT_WAVES:
      if (v != 3 && v != 4 && v != 5 && v != 6 && v != 8)
        return set_err(&c->err, CVR_ERR_INVALID, "waves must be 3, 4, 5, 6 or 8");
      c->waves = (int)v;
      c->wpool_waves = (v == 5 || v == 3 || v == 6) ? (int)v : 4;
      c->inited = false;
      return CVR_OK;
    case CVR_OPT_MORTON:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "morton must be 0 or 1");
      c->morton = (int)v;
      return CVR_OK;
    case CVR_OPT_BATCH:
      if (v < 1 || v > 64) return set_err(&c->err, CVR_ERR_INVALID, "batch must be 1..64");
      c->swap_batch = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_TAIL:
      if (v < 0 || v > 64) return set_err(&c->err, CVR_ERR_INVALID, "tail must be 0..64");
      c->pool_tail = (uint32_t)v;
      return CVR_OK;
    case CVR_OPT_BOUNDS:
      // takes effect at the next cvr_set_medium
      if (v < 0 || v > 5) return set_err(&c->err, CVR_ERR_INVALID, "bounds must be 0 (off) or log2 brick size 1..5");
      c->bound_shift = (uint32_t)v;
      c->bound_shift_set = true;
      return CVR_OK;
    case CVR_OPT_CELLS:
      // takes effect at the next cvr_set_medium
      c->use_cells = v != 0;
      return CVR_OK;
    case CVR_OPT_SAMPLE_ORDER:
      if (v < -1 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "sample order must be -1, 0 or 1");
      c->sample_order = (int)v;
      return CVR_OK;
    case CVR_OPT_EMPTY_MASK:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "empty mask must be 0 or 1");
      c->empty_mask = (int)v;
      return CVR_OK;
    case CVR_OPT_COUNT_WORDS:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "count words must be 0 or 1");
      c->count_words = (int)v;
      return CVR_OK;
    case CVR_OPT_WAVE_PAIR:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "wave pair must be 0 or 1");
      if (v == 1 && !cvr::wpool_pair_built())
        return set_err(&c->err, CVR_ERR_UNSUPPORTED,
                       "wave pair (k_wpair) is an experiment built only into `make variant-pair`");
      c->wave_pair = (int)v;
      return CVR_OK;
    case CVR_OPT_UNIFORM_ALBEDO:
      // takes effect at the next cvr_set_medium
      c->uniform_albedo = v != 0;
      return CVR_OK;
    case CVR_OPT_RNG_BINDING:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "rng binding must be 0 (path) or 1 (thread)");
      c->rng_binding = (int)v;
      return CVR_OK;
    case CVR_OPT_WORLD_TO_AABB:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "world_to_aabb must be 0 (reference) or 1 (fixed)");
      c->world_to_aabb = (int)v;
      return CVR_OK;
    case CVR_OPT_MK_COMPACTION:
      if (v < 0 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "mk_compaction must be 0 (fixed) or 1 (reference)");
      c->mk_compaction = (int)v;
      return CVR_OK;
    case CVR_OPT_SCATTER_EPS:
      if (v < -1 || v > 1) return set_err(&c->err, CVR_ERR_INVALID, "scatter_eps must be -1, 0 or 1");
      c->scatter_eps = (int)v;
      c->inited = false;
      return CVR_OK;
    default:
      return set_err(&c->err, CVR_ERR_INVALID, "unknown option %d", opt);
  }
}

int cvr_init(cvr_ctx* c) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  return do_init(c);
}

int cvr_device_info(cvr_ctx* c, int* cu_count, int* grid) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  int r = do_init(c);
  if (r) return r;
  if (cu_count) *cu_count = c->cu_count;
  if (grid) *grid = c->persistent_grid;
  return CVR_OK;
}

static uint32_t spread_bits16(uint32_t v) {  // bit i -> bit 2i
  v &= 0xFFFFu;
  v = (v | (v << 8)) & 0x00FF00FFu;
  v = (v | (v << 4)) & 0x0F0F0F0Fu;
  v = (v | (v << 2)) & 0x33333333u;
  v = (v | (v << 1)) & 0x55555555u;
  return v;
}

// Order 2: within each queue's band, the launch's blocks in 2-D Morton order
// of their (x, y) in the tile, so the blocks in flight on an XCD cover a
// compact patch of the image (and so of the volume) instead of a strip of a
// block row.  C5 (4096^2, sparse cloud): 149.3 vs 155.3 ms row-major; C2
// unchanged (tools/block_order.py).  Computed on the host once per block
// layout, kept on the device.
static int ensure_zorder(cvr_ctx* c, cvr::LaunchParams& L) {
  if (L.order != 1 || L.block_perm || c->order != 2 || L.n_blocks == 0) return CVR_OK;
  const uint64_t key[5] = {L.n_blocks, (uint64_t)L.n_queues / L.sub, L.blk_off, L.blk_stride, L.blocks_x};
  if (!c->d_zperm || memcmp(key, c->zkey, sizeof(key)) != 0) {
    const uint32_t nb = L.n_blocks;
    std::vector<uint32_t>& perm = c->h_zperm;
    perm.resize(nb);
    std::vector<std::pair<uint32_t, uint32_t>> code(nb);
    for (uint32_t q = 0; q < L.n_queues / L.sub; ++q) {  // Morton order within each XCD band
      const uint32_t a = band_begin(L, q), e = band_begin(L, q + 1);
      for (uint32_t b = a; b < e; ++b) {
        const uint32_t tb = L.blk_off + b * L.blk_stride;
        const uint32_t bx = tb % L.blocks_x, by = tb / L.blocks_x;
        code[b] = {spread_bits16(bx) | (spread_bits16(by) << 1), b};
      }
      std::sort(code.begin() + a, code.begin() + e);
      for (uint32_t b = a; b < e; ++b) perm[b] = code[b].second;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // the previous table may still be in use
    if (c->d_zperm) (void)hipFree(c->d_zperm);
    c->d_zperm = nullptr;
    HIP_TRY(c, hipMalloc(&c->d_zperm, (size_t)nb * sizeof(uint32_t)));
    HIP_TRY(c, hipMemcpy(c->d_zperm, perm.data(), (size_t)nb * sizeof(uint32_t), hipMemcpyHostToDevice));
    memcpy(c->zkey, key, sizeof(key));
  }
  L.block_perm = c->d_zperm;
  return CVR_OK;
}

int cvr_launch_render(cvr_ctx* c) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  int r = check_ready(c);
  if (r) return r;
  if (!c->d_out) return set_err(&c->err, CVR_ERR_STATE, "no output buffer");
  if ((r = do_init(c))) return r;
  uint64_t first, count;
  compute_range(c, &first, &count);
  cvr::LaunchParams L{};
  fill_launch(c, L, first, count);
  if ((r = ensure_zorder(c, L))) return r;
  const bool eps = scatter_eps_for(c);
  if (!c->chunk && scheduler_for(c) == 3) {
    // Wave-pool dequeue chunk by the paths each wave gets: about 8 chunks per
    // wave, 64..256 paths.  Small launches (block shards of a multi-GPU render)
    // then end with the waves' last chunks evenly spread (C2 shard 1/8 on one
    // GPU: 1.09 ms at 64 vs 1.18 at 256; the whole C2 launch keeps 256).
    const uint64_t grid = wpool_launch_grid(c, L.path_count);
    const uint64_t per_wave = grid ? (uint64_t)L.path_count / grid : 0;
    L.chunk = per_wave >= 2048 ? 256u : per_wave >= 1024 ? 128u : 64u;
  }
  if (scheduler_for(c) == 3) {
    L.wflags = (uint32_t)(c->drain < 0 ? 1 : c->drain) & cvr::kDrainMask;
    // samples innermost + combined splats (CVR_OPT_SAMPLE_ORDER 1): dense C2 / C3 +2.7% / +3.6%
    // (profiles/round5/ab/call6_sample_order_ab.log); C5 -1.4% before the sparse empty-region
    // mask, +2.2% with it (116.4-116.8 vs 118.9-119.7 ms, profiles/round5/ab/
    // c5_sample_order_emask.log): off by default.  The in-launch output instance
    // (cvr_render_frame) splats per lane (combining cost its dense instance two VGPR spills), and
    // per-lane splats with samples innermost put the same pixel on several lanes of one atomic
    // instruction, which the memory side serialises (C5 one render 2086 vs 2666 Msamples/s):
    // that launch always keeps the sample-major order.
    int so = c->sample_order >= 0 ? c->sample_order : 0;
    if (c->frame_done_active) so = 0;
    if (so == 1) L.wflags |= cvr::kUnitSampleInner | cvr::kSplatCombine;
  }
  // The persistent schedulers' u32 queue heads run past a queue's end by at
  // most one chunk per wave before every wave sees the queue exhausted
  // (waves: at most 4 per block of any scheduler).
  const uint64_t waves_max =
      4ull * (c->grid_override ? c->grid_override
                               : (uint64_t)std::max({c->persistent_grid, c->pool_grid, c->wpool_grid,
                                                      c->wpool_grid_sparse}));
  uint64_t units_max = L.order ? 0 : count;
  for (uint32_t q = 0; L.order && q < L.n_queues; ++q)
    units_max = std::max<uint64_t>(units_max, (uint64_t)(queue_begin(L, q + 1) - queue_begin(L, q)) * 64u * L.samples);
  if (first + count > 0xFFFFFFFFull || units_max + waves_max * L.chunk > 0xFFFFFFFFull)
    return set_err(&c->err, CVR_ERR_INVALID, "path range [%llu, +%llu) overflows the 32-bit path ids / queue heads",
                   (unsigned long long)first, (unsigned long long)count);
  HIP_TRY(c, hipMemsetAsync(c->d_work, 0, kWorkBytes, c->stream));
  HIP_TRY(c, hipEventRecord(c->ev_start, c->stream));
  c->last_iterations = 0;
  c->last_track_ms = c->last_events_ms = 0;
  if (c->rng_binding == 1) {
    if (c->kernel != CVR_KERNEL_REGENERATION_SK && c->kernel != CVR_KERNEL_STREAMING_SK &&
        c->kernel != CVR_KERNEL_SORTING_SK && c->kernel != CVR_KERNEL_STREAMING_MK)
      return set_err(&c->err, CVR_ERR_UNSUPPORTED,
                     "thread-bound RNG (CVR_OPT_RNG_BINDING 1) is regenerationSK, streamingSK, sortingSK or "
                     "streamingMK only");
    if (L.order) {  // one queue of path ids in order: the thread-bound kernels have no work bands
      L.order = 0;
      L.n_queues = 1;
    }
    if (c->kernel == CVR_KERNEL_REGENERATION_SK) {
      const uint32_t grid = c->grid_override ? c->grid_override : (uint32_t)c->cu_count * 16u;
      HIP_TRY(c, cvr::launch_regen_thread(launch_medium(c), L, eps, grid, c->stream));
    } else if (c->kernel == CVR_KERNEL_STREAMING_MK) {
      // 256-thread blocks, the occupancy grid of d_extend (RenderKernelLauncher.cu:366-392)
      const uint32_t grid = c->grid_override ? c->grid_override : (uint32_t)c->cu_count * 2u;
      if ((r = smk_thread_render(c, L, grid))) return r;
    } else {
      // StreamingVolPTsk / SortingVolPTsk: 256-thread blocks, the occupancy grid (maxOccupancyGrid,
      // RenderKernelLauncher.cu:501-508) of 2 blocks per CU unless CVR_OPT_GRID says otherwise
      const uint32_t grid = c->grid_override ? c->grid_override : (uint32_t)c->cu_count * 2u;
      HIP_TRY(c, cvr::launch_stream_thread(launch_medium(c), L, c->kernel == CVR_KERNEL_SORTING_SK, grid, c->stream));
    }
  } else if (c->kernel == CVR_KERNEL_NAIVE_MK && c->mk_compaction) {
    if ((r = mk_reference_render(c, L))) return r;
  } else if (c->kernel == CVR_KERNEL_NAIVE_MK && !mk_on_wpool(c)) {
    HIP_TRY(c, cvr::launch_naive_mk(launch_medium(c), L, c->stream));
  } else if (scheduler_for(c) == kSchedPerItem) {
    HIP_TRY(c, cvr::launch_naive(launch_medium(c), L, eps, c->stream));
  } else if (scheduler_for(c) == 0) {
    const uint32_t grid = c->grid_override ? c->grid_override : (uint32_t)c->persistent_grid;
    HIP_TRY(c, cvr::launch_persistent(launch_medium(c), L, eps, c->waves, grid, c->stream));
  } else if (scheduler_for(c) == 2) {
    const uint32_t grid = c->grid_override ? c->grid_override : (uint32_t)c->pool_grid;
    HIP_TRY(c, cvr::launch_pool(launch_medium(c), L, eps, grid, c->stream));
  } else if (scheduler_for(c) == 3) {
    const bool sparse = c->m.leaves != nullptr;
    const int waves = wpool_waves_for(c, sparse);
    const uint32_t grid = wpool_launch_grid(c, L.path_count);
    const size_t need = (size_t)grid * cvr::wpool_slots(waves, sparse);
    if (need > c->pool_T_n) {
      if (c->d_pool_T) (void)hipFree(c->d_pool_T);
      c->d_pool_T = nullptr;
      c->pool_T_n = 0;
      HIP_TRY(c, hipMalloc(&c->d_pool_T, need * sizeof(float4)));
      c->pool_T_n = need;
    }
    L.pool_T = c->d_pool_T;
    L.rec = c->d_rec_active;
    if (c->frame_done_active) {
      // in-launch output: the first kFrameFlushers workgroups flush, the rest render
      if (L.rec || L.order != 1 || grid <= 4 * cvr::kFrameFlushers)
        return set_err(&c->err, CVR_ERR_STATE, "in-launch output needs a pixel-block launch of > %u waves",
                       4 * cvr::kFrameFlushers);
      L.frame_done = c->frame_done_active;
    }
    HIP_TRY(c, cvr::launch_wpool(launch_medium(c), L, eps, waves, grid, c->stream, c->wave_pair != 0,
                                 c->kernel == CVR_KERNEL_NAIVE_MK, c->count_words != 0));
  } else if (L.path_count > 0) {
    if ((r = wf_render(c, L, eps))) return r;
  }
  HIP_TRY(c, hipEventRecord(c->ev_stop, c->stream));
  c->timed = true;
  return CVR_OK;
}

int cvr_synchronize(cvr_ctx* c) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return CVR_OK;
}

// Per-tile seed advance (RenderKernelLauncher.cu): RegenerationVolPTsk and
// StreamingVolPTmk add n_paths per reset (:359, :480), StreamingVolPTsk and
// SortingVolPTsk add 1 (:573, :664), NaiveVolPTsk and NaiveVolPTmk keep it.
// Returns the seed after `resets` resets starting from `seed` (u32 wrap).
static uint32_t seed_after_resets(const cvr_ctx* c, uint32_t seed, uint32_t resets) {
  if (c->kernel == CVR_KERNEL_REGENERATION_SK || c->kernel == CVR_KERNEL_STREAMING_MK)
    return seed + (uint32_t)c->n_paths * resets;
  if (c->kernel == CVR_KERNEL_STREAMING_SK || c->kernel == CVR_KERNEL_SORTING_SK) return seed + resets;
  return seed;
}

int cvr_reset(cvr_ctx* c) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // Queue heads are re-zeroed per launch; only the seed carries over.
  c->seed = seed_after_resets(c, c->seed, 1);
  return CVR_OK;
}

int cvr_clear_output(cvr_ctx* c) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (!c->d_out) return set_err(&c->err, CVR_ERR_STATE, "no output buffer");
  HIP_TRY(c, hipMemsetAsync(c->d_out, 0, (size_t)c->tile_w * c->tile_h * sizeof(float4), c->stream));
  return CVR_OK;
}

int cvr_blocks_to_host(const float* device_src, float* host_dst, uint32_t width, uint32_t height, uint32_t rank,
                       uint32_t world, float scale, void* stream) {
  if (!device_src || !host_dst) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  if (width % 8 || height % 8 || world == 0 || rank >= world)
    return set_err(nullptr, CVR_ERR_INVALID, "block shards need sides that are multiples of 8 and rank < world");
  if ((((uintptr_t)device_src) | ((uintptr_t)host_dst)) & 15u)
    return set_err(nullptr, CVR_ERR_INVALID, "image buffers must be 16-byte aligned");
  if (width == 0 || height == 0) return CVR_OK;
  void* dptr = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dptr, host_dst, 0);
  if (e != hipSuccess || !dptr)
    return set_err(nullptr, CVR_ERR_INVALID, "host buffer is not pinned or registered: %s", hipGetErrorString(e));
  e = cvr::launch_blocks_to_host(device_src, static_cast<float*>(dptr), width, height, rank, world, scale,
                                 static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_err(nullptr, CVR_ERR_HIP, "blocks_to_host: %s", hipGetErrorString(e));
  return CVR_OK;
}

int cvr_image_to_host(const float* device_src, float* host_dst, size_t n_floats, float scale, void* stream) {
  if (!device_src || !host_dst) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  if (n_floats == 0) return CVR_OK;
  void* dptr = nullptr;  // the host buffer's device address (pinned / registered memory)
  hipError_t e = hipHostGetDevicePointer(&dptr, host_dst, 0);
  if (e != hipSuccess || !dptr)
    return set_err(nullptr, CVR_ERR_INVALID, "host buffer is not pinned or registered: %s", hipGetErrorString(e));
  e = cvr::launch_image_to_host(device_src, static_cast<float*>(dptr), n_floats, scale, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return set_err(nullptr, CVR_ERR_HIP, "image to host: %s", hipGetErrorString(e));
  return CVR_OK;
}

int cvr_get_stats(cvr_ctx* c, cvr_stats* st) {
  if (!c || !st) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  unsigned long long w[32] = {0};  // 16 stats (two rows of 8) and the diagnostic row
  static_assert(cvr::kStatWordsSlot < 32 && kWorkDebug == kWorkStats + 16 * sizeof(unsigned long long), "work area layout");
  HIP_TRY(c, hipMemcpy(w, c->d_work + kWorkStats, sizeof(w), hipMemcpyDeviceToHost));
  unsigned long long v[8];
  for (int k = 0; k < 8; ++k) v[k] = w[k] + w[8 + k];  // wavefront: events + track rows
  cvr_stats s{};
  s.paths = v[cvr::STAT_PATHS];
  s.segments = v[cvr::STAT_SEGMENTS];
  s.steps = v[cvr::STAT_STEPS];
  s.density = v[cvr::STAT_DENSITY];
  s.albedo = v[cvr::STAT_ALBEDO];
  s.escaped = v[cvr::STAT_ESCAPED];
  s.truncated = v[cvr::STAT_TRUNCATED];
  s.fetches = v[cvr::STAT_FETCH];
  s.words = w[cvr::kStatWordsSlot];  // counting launches only (CVR_OPT_COUNT_WORDS)
  s.kernel_ms = 0.0;
  if (c->timed) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_start, c->ev_stop));
    s.kernel_ms = ms;
  }
  s.iterations = c->last_iterations;
  s.track_ms = c->last_track_ms;
  s.events_ms = c->last_events_ms;
  *st = s;
  c->last = s;
  return CVR_OK;
}

int cvr_debug_counters(cvr_ctx* c, uint64_t out[16]) {
  if (!c || !out) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(out, c->d_work + kWorkDebug, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return CVR_OK;
}


int cvr_copy_output(cvr_ctx* c, float* host, float scale) {
  if (!c || !host) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  if (!c->d_out) return set_err(&c->err, CVR_ERR_STATE, "no output buffer");
  const size_t n = (size_t)c->tile_w * c->tile_h * 4;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(host, c->d_out, n * sizeof(float), hipMemcpyDeviceToHost));
  if (scale != 1.0f)
    for (size_t i = 0; i < n; ++i) host[i] = host[i] / scale;
  return CVR_OK;
}

int cvr_trace_launch(cvr_ctx* c, cvr_path_record* out, uint64_t n_out) {
  if (!c || !out) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  int r = check_ready(c);
  if (r) return r;
  if ((r = do_init(c))) return r;
  if (scheduler_for(c) != 3 || c->rng_binding || c->kernel == CVR_KERNEL_NAIVE_MK)
    return set_err(&c->err, CVR_ERR_UNSUPPORTED, "cvr_trace_launch traces the wave-pool scheduler only");
  uint64_t first, count;
  compute_range(c, &first, &count);
  if (n_out != count)
    return set_err(&c->err, CVR_ERR_INVALID, "record buffer holds %llu records, the launch range %llu",
                   (unsigned long long)n_out, (unsigned long long)count);
  const bool sparse = c->m.leaves != nullptr;
  cvr::LaunchParams Lq{};
  fill_launch(c, Lq, first, count);
  const uint64_t grid = wpool_launch_grid(c, Lq.path_count);
  const size_t pid_bytes = (size_t)grid * cvr::wpool_slots(wpool_waves_for(c, sparse), sparse) * sizeof(uint32_t);
  const size_t rec_bytes = (size_t)count * sizeof(cvr_path_record);
  // the traced launch splats into a scratch framebuffer, not the context's
  const size_t out_bytes = (size_t)c->tile_w * c->tile_h * sizeof(float4);
  const size_t out_at = (pid_bytes + rec_bytes + 16 + 255) & ~(size_t)255;
  char* d = nullptr;
  HIP_TRY(c, hipMalloc(&d, out_at + out_bytes));
  hipError_t e = hipMemsetAsync(d, 0, out_at + out_bytes, c->stream);
  if (e == hipSuccess) {
    float4* saved_out = c->d_out;
    c->d_out = reinterpret_cast<float4*>(d + out_at);
    c->d_rec_active = d + pid_bytes;
    r = cvr_launch_render(c);
    c->d_rec_active = nullptr;
    c->d_out = saved_out;
    if (!r) {
      // the kernel writes path p's record at p - L.path_first: a contiguous
      // shard (no block order) moved path_first to the shard's first id
      cvr::LaunchParams Ls{};
      fill_launch(c, Ls, first, count);
      const uint64_t shift = Ls.path_first - first;
      e = hipStreamSynchronize(c->stream);
      if (e == hipSuccess && shift) {
        memset(out, 0, rec_bytes);
        e = hipMemcpy(out + shift, d + pid_bytes, (size_t)Ls.path_count * sizeof(cvr_path_record),
                      hipMemcpyDeviceToHost);
      } else if (e == hipSuccess) {
        e = hipMemcpy(out, d + pid_bytes, rec_bytes, hipMemcpyDeviceToHost);
      }
    }
  }
  (void)hipFree(d);
  if (r) return r;
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "trace launch: %s", hipGetErrorString(e));
  return CVR_OK;
}

int cvr_trace_paths(cvr_ctx* c, uint32_t first, uint32_t count, cvr_path_record* out) {
  if (!c || !out) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  int r = check_ready(c);
  if (r) return r;
  if (count == 0) return CVR_OK;
  cvr::LaunchParams L{};
  fill_launch(c, L, first, count, /*sharded=*/false);
  cvr::PathRecord* d_rec = nullptr;
  HIP_TRY(c, hipMalloc(&d_rec, (size_t)count * sizeof(cvr::PathRecord)));
  hipError_t e = cvr::launch_trace(launch_medium(c), L, scatter_eps_for(c), d_rec, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess)
    e = hipMemcpy(out, d_rec, (size_t)count * sizeof(cvr::PathRecord), hipMemcpyDeviceToHost);
  (void)hipFree(d_rec);
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "trace: %s", hipGetErrorString(e));
  return CVR_OK;
}

// ------------------------------------------------------------ renderer ----
int cvr_render_image(cvr_ctx* c, const cvr_render_desc* d, void* device_image, float* host_image, cvr_stats* stats) {
  return cvr_render_tiles(c, d, 0, 1, device_image, host_image, stats);
}

int cvr_render_tiles(cvr_ctx* c, const cvr_render_desc* d, uint32_t first_tile, uint32_t tile_stride,
                     void* device_image, float* host_image, cvr_stats* stats) {
  if (!c || !d) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  if (tile_stride == 0) return set_err(&c->err, CVR_ERR_INVALID, "tile stride 0");
  uint32_t tile_dim[2];
  int r = cvr_tiling(d->resolution[0], d->resolution[1], d->n_tiles[0], d->n_tiles[1], tile_dim);
  if (r) return set_err(&c->err, r, "%s", g_last_error.c_str());
  if ((r = cvr_set_resolution(c, tile_dim[0], tile_dim[1]))) return r;
  if ((r = cvr_set_iterations(c, d->iterations))) return r;  // setNIterations
  if ((r = check_ready(c))) return r;
  const uint32_t W = d->resolution[0], H = d->resolution[1];
  const uint32_t ntiles = d->n_tiles[0] * d->n_tiles[1];
  if (ntiles == 1 && first_tile == 0 && !device_image && host_image && !c->external_out) {
    // one tile into host memory: cvr_render_frame (no scratch image per call; the same
    // clear, launch, Scale + copy and seed advance as the loop below)
    if ((r = cvr_set_offset(c, 0, 0))) return r;
    if ((r = ensure_output(c))) return r;
    return cvr_render_frame(c, host_image, (size_t)W * H * 4u, 1, stats);
  }
  float4* dimg = static_cast<float4*>(device_image);
  float4* tmp_img = nullptr;
  if (!dimg && host_image) {
    HIP_TRY(c, hipMalloc(&tmp_img, (size_t)W * H * sizeof(float4)));
    const hipError_t e = hipMemsetAsync(tmp_img, 0, (size_t)W * H * sizeof(float4), c->stream);
    if (e != hipSuccess) {
      (void)hipFree(tmp_img);
      return set_err(&c->err, CVR_ERR_HIP, "image buffer: %s", hipGetErrorString(e));
    }
    dimg = tmp_img;
  }
  const uint32_t seed0 = c->seed;
  cvr_stats acc{};
  // initRenderState: memset the accumulator
  if ((r = cvr_clear_output(c))) goto done;
  for (uint32_t k = first_tile; k < ntiles; k += tile_stride) {
    // the seed tile k has in the sequential tile loop (k resets after seed0)
    c->seed = seed_after_resets(c, seed0, k);
    uint32_t org[2];
    cvr_tile_origin(k, d->n_tiles[0], tile_dim, org);
    if ((r = cvr_set_offset(c, org[0], org[1]))) goto done;  // copyOffset
    if ((r = cvr_launch_render(c))) goto done;               // launchRender
    if (dimg) {  // getImage: scale by 1/current_iteration_ into the image
      hipError_t e = cvr::launch_tile_to_image(c->d_out, tile_dim[0], tile_dim[1], dimg, W, org[0], org[1],
                                               (float)d->iterations, c->stream);
      if (e != hipSuccess) {
        r = set_err(&c->err, CVR_ERR_HIP, "tile transfer: %s", hipGetErrorString(e));
        goto done;
      }
    }
    cvr_stats s{};
    if ((r = cvr_get_stats(c, &s))) goto done;  // synchronises (reset() does too)
    acc.paths += s.paths;
    acc.segments += s.segments;
    acc.steps += s.steps;
    acc.density += s.density;
    acc.albedo += s.albedo;
    acc.escaped += s.escaped;
    acc.truncated += s.truncated;
    acc.fetches += s.fetches;
    acc.words += s.words;
    acc.kernel_ms += s.kernel_ms;
    if ((r = cvr_reset(c))) goto done;  // prepareForNextIterations
    if (ntiles != 1 && (r = cvr_clear_output(c))) goto done;
  }
  c->seed = seed_after_resets(c, seed0, ntiles);  // as after the whole tile loop
  if (host_image) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(host_image, dimg, (size_t)W * H * sizeof(float4), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      r = set_err(&c->err, CVR_ERR_HIP, "image copy: %s", hipGetErrorString(e));
      goto done;
    }
  }
  if (stats) *stats = acc;
done:
  if (tmp_img) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(tmp_img);
  }
  return r;
}

// One device's share of a multi-device render (cvr --devices):
// its tiles of the tile loop (tile k -> device k mod N, CudaVolPath.cpp:249-280
// split over devices) or its block shard of the one tile, normalised and stored
// by a kernel straight into the shared pinned host image at their places.  The
// shares are pixel-disjoint, so N of these calls (one host thread per device)
// leave cvr_render_image's image in the one host buffer: no reduction.
int cvr_render_share_to_host(cvr_ctx* c, const cvr_render_desc* d, uint32_t first_tile, uint32_t tile_stride,
                             float* host_image, size_t host_floats, cvr_stats* stats) {
  if (!c || !d || !host_image) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  if (tile_stride == 0) return set_err(&c->err, CVR_ERR_INVALID, "tile stride 0");
  const uint32_t W = d->resolution[0], H = d->resolution[1];
  if (host_floats < (size_t)W * H * 4u)
    return set_err(&c->err, CVR_ERR_INVALID, "host image holds %zu floats, the %ux%u image needs %zu", host_floats, W,
                   H, (size_t)W * H * 4u);
  if ((uintptr_t)host_image & 15u) return set_err(&c->err, CVR_ERR_INVALID, "host image must be 16-byte aligned");
  int r = ensure_device(c);
  if (r) return r;
  void* dhost = nullptr;  // the host image's device address (pinned / registered memory)
  hipError_t e = hipHostGetDevicePointer(&dhost, host_image, 0);
  if (e != hipSuccess || !dhost) {
    (void)hipGetLastError();
    return set_err(&c->err, CVR_ERR_INVALID, "host image is not pinned or registered (cvr_host_alloc)");
  }
  const uint32_t ntiles = d->n_tiles[0] * d->n_tiles[1];
  if (ntiles != 1 || c->shard_world == 1) {
    // tiles k = first_tile, first_tile + stride, ...: each tile's pixels only (k_tile_to_image
    // into the mapped host image), each tile with its sequential-loop seed
    if (ntiles != 1 && c->shard_world != 1)
      return set_err(&c->err, CVR_ERR_INVALID, "a tile share and a block shard at once");
    return cvr_render_tiles(c, d, first_tile, tile_stride, dhost, nullptr, stats);
  }
  // one tile, this context's block shard: launch, then its 8x8 blocks into the host image
  if (first_tile != 0) return set_err(&c->err, CVR_ERR_INVALID, "one tile: the share is the block shard");
  if (W % 8 || H % 8) return set_err(&c->err, CVR_ERR_INVALID, "block shards need sides that are multiples of 8");
  if ((r = cvr_set_resolution(c, W, H)) || (r = cvr_set_iterations(c, d->iterations)) || (r = cvr_set_offset(c, 0, 0)))
    return r;
  if ((r = check_ready(c)) || (r = ensure_output(c))) return r;
  {
    // the launch must really be this context's 8x8-block shard: fill_launch falls back to a
    // contiguous slice of path ids (part-sums of other pixels) without the block work order
    // (thread-bound RNG, CVR_OPT_ORDER 0, the per-item / wavefront schedulers, > 2^20 samples)
    uint64_t first = 0, count = 0;
    compute_range(c, &first, &count);
    cvr::LaunchParams Lc{};
    fill_launch(c, Lc, first, count);
    if (c->shard_world > 1 && (Lc.order != 1 || Lc.blk_stride != c->shard_world || c->rng_binding != 0))
      return set_err(&c->err, CVR_ERR_UNSUPPORTED,
                     "this launch has no 8x8-block work order (thread-bound RNG, CVR_OPT_ORDER 0, a per-item or "
                     "wavefront scheduler, or more than 2^20 samples), so it cannot be block-sharded over devices");
  }
  if ((r = cvr_clear_output(c)) || (r = cvr_launch_render(c))) return r;
  e = cvr::launch_blocks_to_host(reinterpret_cast<const float*>(c->d_out), static_cast<float*>(dhost), W, H,
                                 c->shard_rank, c->shard_world, (float)d->iterations, c->stream);
  if (e != hipSuccess) return set_err(&c->err, CVR_ERR_HIP, "blocks to host: %s", hipGetErrorString(e));
  cvr_stats s{};
  if ((r = cvr_get_stats(c, &s))) return r;  // synchronises: the blocks are in the host image
  if (stats) *stats = s;
  return cvr_reset(c);  // prepareForNextIterations
}

int cvr_host_alloc(size_t bytes, void** out) {
  if (!out) return set_err(nullptr, CVR_ERR_INVALID, "NULL argument");
  *out = nullptr;
  const hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable);
  if (e != hipSuccess) return set_err(nullptr, CVR_ERR_HIP, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  return CVR_OK;
}

int cvr_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) return set_err(nullptr, CVR_ERR_HIP, "hipHostFree failed");
  return CVR_OK;
}

// The launcher settings a helper context of cvr_render_frame takes from its
// parent: everything but its own resources (stream, work queues, scratch).
static void copy_settings(cvr_ctx* d, const cvr_ctx* s) {
  d->m = s->m;  // the parent's medium (re-shared every frame: the parent may have loaded another)
  d->n_cell_leaves = s->n_cell_leaves;
  d->have_medium = s->have_medium;
  memcpy(d->inv_view, s->inv_view, sizeof(d->inv_view));
  d->r2v[0] = s->r2v[0];
  d->r2v[1] = s->r2v[1];
  d->full_res[0] = s->full_res[0];
  d->full_res[1] = s->full_res[1];
  d->have_camera = s->have_camera;
  d->tile_w = s->tile_w;
  d->tile_h = s->tile_h;
  d->off[0] = s->off[0];
  d->off[1] = s->off[1];
  d->iterations = s->iterations;
  d->n_paths = s->n_paths;
  d->range_first = s->range_first;
  d->range_count = s->range_count;
  d->shard_rank = s->shard_rank;
  d->shard_world = s->shard_world;
  d->seed = s->seed;
  d->n_queues = s->n_queues;
  d->subqueues = s->subqueues;
  d->drain = s->drain;
  d->sample_order = s->sample_order;
  d->empty_mask = s->empty_mask;
  d->count_words = s->count_words;
  d->order = s->order;
  d->max_segments = s->max_segments;
  d->chunk = s->chunk;
  d->ev_thresh = s->ev_thresh;
  d->grid_override = s->grid_override;
  d->inflight = s->inflight;
  d->scatter_eps = s->scatter_eps;
  d->rng_binding = s->rng_binding;
  d->world_to_aabb = s->world_to_aabb;
  d->mk_compaction = s->mk_compaction;
  d->pool_tail = s->pool_tail;
  d->wpool_waves = s->wpool_waves;
  d->morton = s->morton;
  d->wave_pair = s->wave_pair;
  d->swap_batch = s->swap_batch;
  d->scheduler = s->scheduler;
  d->waves = s->waves;
  d->pool_max = s->pool_max;
}

// cvr_render_frame with the in-launch output: the clear, the header and the block
// counts, one launch whose flusher waves store the normalised blocks into the host
// image (device address dhost), and the copy after the launch only if a flusher gave up.
static int render_frame_flush(cvr_ctx* c, void* dhost, cvr_stats* stats) {
  const uint32_t W = c->tile_w, H = c->tile_h;
  const size_t px = (size_t)W * H, nb = (size_t)(W / 8u) * (H / 8u);
  if (c->flush_blocks < nb) {
    if (c->d_flush) (void)hipFree(c->d_flush);
    c->d_flush = nullptr;
    c->flush_blocks = 0;
    HIP_TRY(c, hipMalloc(&c->d_flush, sizeof(cvr::FrameFlush) + nb * cvr::kDoneStride * sizeof(unsigned int)));
    c->flush_blocks = nb;
    c->flush_hdr_valid = false;
  }
  if (!c->h_flush_status) {
    HIP_TRY(c, hipHostMalloc(&c->h_flush_status, 64, hipHostMallocDefault));
  }
  if (!c->frame_ev[0])
    for (auto& e : c->frame_ev) HIP_TRY(c, hipEventCreate(&e));
  unsigned int* dstatus = nullptr;
  HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&dstatus), c->h_flush_status, 0));
  memset(c->h_flush_status, 0, 64);  // the previous frame has ended (its call synchronised)
  cvr::FrameFlush hdr{};
  hdr.host = static_cast<float4*>(dhost);
  hdr.status = dstatus;
  hdr.host_w = W;
  hdr.scale = (float)c->iterations;
  hdr.give_up = c->frame_flush == 2 ? 1u : 0u;
  // the header only travels when it changed (the same host image frame after frame: none)
  const bool send_hdr = !c->flush_hdr_valid || memcmp(&hdr, &c->flush_hdr, sizeof(hdr)) != 0;
  c->flush_hdr = hdr;
  unsigned int* done = reinterpret_cast<unsigned int*>(c->d_flush + sizeof(cvr::FrameFlush));
  HIP_TRY(c, hipMemsetAsync(c->d_out, 0, px * sizeof(float4), c->stream));  // initRenderState
  if (send_hdr) {
    c->flush_hdr_valid = false;
    HIP_TRY(c, hipMemcpyAsync(c->d_flush, &c->flush_hdr, sizeof(cvr::FrameFlush), hipMemcpyHostToDevice, c->stream));
    c->flush_hdr_valid = true;
  }
  HIP_TRY(c, hipMemsetAsync(done, 0, nb * cvr::kDoneStride * sizeof(unsigned int), c->stream));
  HIP_TRY(c, hipEventRecord(c->frame_ev[0], c->stream));
  c->frame_done_active = done;
  int r = cvr_launch_render(c);
  c->frame_done_active = nullptr;
  if (r) return r;
  HIP_TRY(c, hipEventRecord(c->frame_ev[1], c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  uint64_t stored = 0;
  for (uint32_t f = 0; f < cvr::kFrameFlushers; ++f) stored += c->h_flush_status[f];
  if (c->h_flush_status[cvr::kFrameFlushers] != 0 || stored != nb) {
    // a flusher gave up: getImage the usual way (the framebuffer is complete)
    ++c->flush_fallbacks;
    c->flush_last_blocks = 0;
    HIP_TRY(c, cvr::launch_image_to_host(reinterpret_cast<const float*>(c->d_out), static_cast<float*>(dhost),
                                         px * 4, (float)c->iterations, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  } else {
    c->flush_last_blocks = (uint32_t)stored;
  }
  c->seed = seed_after_resets(c, c->seed, 1);  // reset(): prepareForNextIterations
  if (!stats) return CVR_OK;
  cvr_stats acc{};
  if ((r = cvr_get_stats(c, &acc))) return r;
  float ms = 0.f;  // clear to the end of the launch
  HIP_TRY(c, hipEventElapsedTime(&ms, c->frame_ev[0], c->frame_ev[1]));
  acc.kernel_ms = ms;
  c->last = acc;
  *stats = acc;
  return CVR_OK;
}

int cvr_frame_flush_info(const cvr_ctx* c, uint32_t* blocks, uint32_t* fallbacks) {
  if (!c) return set_err(nullptr, CVR_ERR_INVALID, "NULL ctx");
  if (blocks) *blocks = c->flush_last_blocks;
  if (fallbacks) *fallbacks = c->flush_fallbacks;
  return CVR_OK;
}

int cvr_render_frame(cvr_ctx* c, float* host_image, size_t host_floats, uint32_t parts, cvr_stats* stats) {
  if (!c || !host_image) return set_err(c ? &c->err : nullptr, CVR_ERR_INVALID, "NULL argument");
  int r = check_ready(c);
  if (r) return r;
  if (host_floats < (size_t)c->tile_w * c->tile_h * 4u)
    return set_err(&c->err, CVR_ERR_INVALID, "host image holds %zu floats, the %ux%u tile needs %zu", host_floats,
                   c->tile_w, c->tile_h, (size_t)c->tile_w * c->tile_h * 4u);
  if (!c->d_out) return set_err(&c->err, CVR_ERR_STATE, "no output buffer");
  if ((r = do_init(c))) return r;
  const uint32_t W = c->tile_w, H = c->tile_h;
  const size_t px = (size_t)W * H;
  // bands need the pixel-block work order of a whole-sample, unsharded, queued launch
  uint64_t first, count;
  compute_range(c, &first, &count);
  cvr::LaunchParams L0{};
  fill_launch(c, L0, first, count);
  const bool queued = (c->kernel != CVR_KERNEL_NAIVE_MK || mk_on_wpool(c)) && scheduler_for(c) != 1 &&
                      scheduler_for(c) != kSchedPerItem &&
                      c->rng_binding == 0;
  const uint32_t brows = (L0.order == 1 && queued && c->shard_world == 1) ? H / 8u : 0u;
  if (parts == 0) parts = 1;
  parts = std::min<uint32_t>(parts, 3u);
  if (brows < parts) parts = brows ? brows : 1u;
  // band k takes (parts - k) shares of the block rows: the last band, whose copy
  // the frame waits for, is the smallest
  uint32_t row0[4] = {0, 0, 0, 0};
  {
    const uint32_t shares = parts * (parts + 1) / 2;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < parts; ++k) {
      acc += parts - k;
      row0[k + 1] = k + 1 == parts ? brows : (uint32_t)((uint64_t)brows * acc / shares);
    }
  }
  // in-launch output (CVR_OPT_FRAME_FLUSH): one part on the wave pool, and a host image
  // the GPU can store into
  void* dhost = nullptr;
  if (c->frame_flush && parts == 1 && brows && scheduler_for(c) == 3 && !c->d_rec_active &&
      c->kernel != CVR_KERNEL_NAIVE_MK &&  // (no in-launch output instance of naiveMK's walk)
      wpool_waves_for(c, c->m.leaves != nullptr) == 5 && wpool_launch_grid(c, L0.path_count) > 4 * cvr::kFrameFlushers) {
    if (hipHostGetDevicePointer(&dhost, host_image, 0) != hipSuccess) {
      (void)hipGetLastError();  // pageable memory: not an error, the copy path below
      dhost = nullptr;
    }
  }
  if (dhost) return render_frame_flush(c, dhost, stats);
  c->flush_last_blocks = 0;
  while (c->frame_kids.size() + 1 < parts) {
    cvr_ctx* k = nullptr;
    if ((r = cvr_create(c->device, c->kernel, &k))) return set_err(&c->err, r, "frame helper: %s", g_last_error.c_str());
    c->frame_kids.push_back(k);
  }
  if (!c->frame_copy) {
    int lo = 0, hi = 0;
    HIP_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(c, hipStreamCreateWithPriority(&c->frame_copy, hipStreamNonBlocking, hi));
  }
  // the same events as render_frame_flush's (created once, whichever path comes first)
  if (!c->frame_ev[0])
    for (auto& e : c->frame_ev) HIP_TRY(c, hipEventCreate(&e));
  if (c->frame_px < px) {
    HIP_TRY(c, hipStreamSynchronize(c->frame_copy));
    if (c->d_frame) (void)hipFree(c->d_frame);
    c->d_frame = nullptr;
    c->frame_px = 0;
    HIP_TRY(c, hipMalloc(&c->d_frame, px * sizeof(float4)));
    c->frame_px = px;
  }
  // clear (initRenderState), then every band on its own stream
  HIP_TRY(c, hipMemsetAsync(c->d_out, 0, px * sizeof(float4), c->stream));
  HIP_TRY(c, hipEventRecord(c->frame_ev[0], c->stream));
  cvr_ctx* who[3] = {c, nullptr, nullptr};
  for (uint32_t k = 1; k < parts; ++k) {
    cvr_ctx* kid = c->frame_kids[k - 1];
    copy_settings(kid, c);
    kid->d_out = c->d_out;
    kid->external_out = true;
    if ((r = do_init(kid))) return set_err(&c->err, r, "frame helper: %s", kid->err.c_str());
    HIP_TRY(c, hipStreamWaitEvent(kid->stream, c->frame_ev[0], 0));
    who[k] = kid;
  }
  const float scale = (float)c->iterations;
  for (uint32_t k = 0; k < parts; ++k) {
    cvr_ctx* x = who[k];
    x->band_first = brows ? row0[k] * (W / 8u) : 0u;
    x->band_count = brows ? (row0[k + 1] - row0[k]) * (W / 8u) : 0u;
    r = cvr_launch_render(x);
    x->band_first = x->band_count = 0;
    if (r) return x == c ? r : set_err(&c->err, r, "frame band %u: %s", k, x->err.c_str());
    HIP_TRY(c, hipEventRecord(c->frame_ev[1 + k], x->stream));
    // getImage of the band's rows (ImageBufferTransfer.cu:61-78: Scale, then the D->H
    // copy) on the copy stream, while the later bands render
    const uint32_t y0 = brows ? row0[k] * 8u : 0u, y1 = brows ? row0[k + 1] * 8u : H;
    HIP_TRY(c, hipStreamWaitEvent(c->frame_copy, c->frame_ev[1 + k], 0));
    HIP_TRY(c, cvr::launch_tile_to_image(c->d_out + (size_t)y0 * W, W, y1 - y0, c->d_frame, W, 0, y0, scale,
                                         c->frame_copy));
    HIP_TRY(c, hipMemcpyAsync(host_image + (size_t)y0 * W * 4, c->d_frame + (size_t)y0 * W,
                              (size_t)(y1 - y0) * W * sizeof(float4), hipMemcpyDeviceToHost, c->frame_copy));
  }
  HIP_TRY(c, hipStreamSynchronize(c->frame_copy));
  c->seed = seed_after_resets(c, c->seed, 1);  // reset(): prepareForNextIterations
  if (!stats) return CVR_OK;  // the counters cost a synchronous read per band
  cvr_stats acc{};
  for (uint32_t k = 0; k < parts; ++k) {
    cvr_stats s{};
    if ((r = cvr_get_stats(who[k], &s))) return who[k] == c ? r : set_err(&c->err, r, "%s", who[k]->err.c_str());
    acc.paths += s.paths;
    acc.segments += s.segments;
    acc.steps += s.steps;
    acc.density += s.density;
    acc.albedo += s.albedo;
    acc.escaped += s.escaped;
    acc.truncated += s.truncated;
    acc.fetches += s.fetches;
    acc.words += s.words;
  }
  float ms = 0.f;  // clear to the end of the band that ends last
  for (uint32_t k = 0; k < parts; ++k) {
    float t = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&t, c->frame_ev[0], c->frame_ev[1 + k]));
    ms = std::max(ms, t);
  }
  acc.kernel_ms = ms;
  c->last = acc;
  *stats = acc;
  return CVR_OK;
}

// ------------------------------------------------------------- helpers ----
int cvr_default_camera(uint32_t w, uint32_t h, float inv_view[12], float r2v[2]) {
  if (!inv_view || !r2v || w == 0 || h == 0) return set_err(nullptr, CVR_ERR_INVALID, "bad camera arguments");
  cvr::camera_for_fov(0.7f, w, h, inv_view, r2v);  // Camera(400, 400, 0.7), Camera.h:25
  return CVR_OK;
}

int cvr_tiling(uint32_t w, uint32_t h, uint32_t ntx, uint32_t nty, uint32_t tile_dim[2]) {
  if (!tile_dim || ntx == 0 || nty == 0) return set_err(nullptr, CVR_ERR_INVALID, "bad tiling arguments");
  // tile_dim = (int)ceil(resolution / n_tiles) with integer division inside
  // ceil: the remainder is never rendered (Q1).
  tile_dim[0] = w / ntx;
  tile_dim[1] = h / nty;
  if (tile_dim[0] == 0 || tile_dim[1] == 0) return set_err(nullptr, CVR_ERR_INVALID, "more tiles than pixels");
  return CVR_OK;
}

int cvr_tile_origin(uint32_t id, uint32_t ntx, const uint32_t tile_dim[2], uint32_t org[2]) {
  if (!tile_dim || !org || ntx == 0) return set_err(nullptr, CVR_ERR_INVALID, "bad tile arguments");
  org[0] = tile_dim[0] * (id % ntx);
  org[1] = tile_dim[1] * (uint32_t)(int)((float)id / (float)ntx);
  return CVR_OK;
}

int cvr_kernel_from_name(const char* name) {
  static const char* names[] = {"naiveSK", "naiveMK", "regenerationSK", "streamingMK", "streamingSK", "sortingSK"};
  if (!name) return CVR_KERNEL_UNKNOWN;
  for (int i = 0; i < 6; ++i)
    if (strcmp(name, names[i]) == 0) return i;
  return CVR_KERNEL_UNKNOWN;
}

const char* cvr_kernel_name(int k) {
  static const char* names[] = {"naiveSK", "naiveMK", "regenerationSK", "streamingMK", "streamingSK", "sortingSK"};
  if (k < 0 || k > 5) return "unknown";
  return names[k];
}

}  // extern "C"
