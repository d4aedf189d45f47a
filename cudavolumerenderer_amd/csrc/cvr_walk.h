// cvr_walk.h - device building blocks of the volumetric random walk (gfx950).
//
// Each function restates one piece of the reference hot path
// (Fe0437/CudaVolumeRenderer implementation/src, cited per function) with the
// exact operation order of oracle/cvr_oracle.c, so that one path traced here
// is bit-identical to the same path traced by the CPU oracle.  Compiled with
// -ffp-contract=off; the only fused multiply-adds are the explicit det_fmaf
// calls (Woodcock step, Woodcock position, trilinear lerps, RNG mapping).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cvr_detmath.h"

namespace cvr {

#define CVR_DEV __device__ __forceinline__

// A pointer to global memory as the global address space.  The wave-pool
// kernel keeps its launch parameters in LDS, so their pointers reach the code
// as generic (flat) pointers, and flat loads, stores and atomics count in
// lgkmcnt as well as vmcnt: every later LDS wait then also waits for them (a
// batch's slot stores and framebuffer atomics stalled its LDS list updates).
// Global instructions count in vmcnt only.
template <class T>
using gptr_t = __attribute__((address_space(1))) T*;
template <class T>
CVR_DEV gptr_t<T> gmem(T* p) {
  return (gptr_t<T>)p;
}
typedef float cvr_f4v __attribute__((ext_vector_type(4)));
CVR_DEV void gstore4(float4* p, float4 v) { *(gptr_t<cvr_f4v>)p = cvr_f4v{v.x, v.y, v.z, v.w}; }
CVR_DEV float4 gload4(const float4* p) {
  const cvr_f4v v = *(__attribute__((address_space(1))) const cvr_f4v*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}

// ------------------------------------------------------------- vectors ----
struct V3 {
  float x, y, z;
};
CVR_DEV V3 mk3(float x, float y, float z) { return V3{x, y, z}; }
CVR_DEV V3 add3(V3 a, V3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
CVR_DEV V3 sub3(V3 a, V3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
CVR_DEV V3 mul3(V3 a, V3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
CVR_DEV V3 div3(V3 a, V3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
CVR_DEV V3 scl3(V3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
CVR_DEV V3 neg3(V3 a) { return mk3(-a.x, -a.y, -a.z); }
CVR_DEV float dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
CVR_DEV V3 cross3(V3 a, V3 b) {
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// helper_math.h:1055 normalize(v) = v*rsqrtf(dot); restated with a correctly
// rounded 1/sqrtf so host and device agree.
CVR_DEV V3 normalize3(V3 v) { return scl3(v, 1.0f / det_sqrtf(dot3(v, v))); }

// ----------------------------------------------------------------- RNG ----
// cuRAND XORWOW, curand_init(seed, 0, 0) + curand_uniform (Rng.h:22-30).
struct Rng {
  uint32_t v0, v1, v2, v3, v4, d;
};
CVR_DEV void rng_init(Rng& s, int32_t seed) {
  // Rng(int) -> unsigned long long: sign extension
  const unsigned long long sd = (unsigned long long)(long long)seed;
  const uint32_t s0 = ((uint32_t)sd) ^ 0xaad26b49u;
  const uint32_t s1 = ((uint32_t)(sd >> 32)) ^ 0xf7dcefddu;
  const uint32_t t0 = 1099087573u * s0;
  const uint32_t t1 = 2591861531u * s1;
  s.d = 6615241u + t1 + t0;
  s.v0 = 123456789u + t0;
  s.v1 = 362436069u ^ t0;
  s.v2 = 521288629u + t1;
  s.v3 = 88675123u ^ t1;
  s.v4 = 5783321u + t0;
}
// Three-input xor as gfx950's v_bitop3_b32 (truth table 0x96 = a ^ b ^ c):
// hipcc 7.2 does not form it from a ^ b ^ c (it emits two v_xor_b32).
CVR_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
CVR_DEV uint32_t rng_next(Rng& s) {
  const uint32_t t = s.v0 ^ (s.v0 >> 2);
  s.v0 = s.v1;
  s.v1 = s.v2;
  s.v2 = s.v3;
  s.v3 = s.v4;
  // (v4 ^ (v4 << 4)) ^ (t ^ (t << 1)): xor is associative, so the same word
  // with one v_bitop3 and one v_xor instead of three v_xor (6 VALU per word, was 7)
  s.v4 = xor3(s.v4, s.v4 << 4, t) ^ (t << 1);
  s.d += 362437u;
  return s.v4 + s.d;
}
// Inverse of rng_next's state transition (takes back the last draw).  The
// new word is n = (v4 ^ (v4 << 4)) ^ (u ^ (u << 1)) with u = v0 ^ (v0 >> 2);
// both xorshifts are invertible by prefix xors.
CVR_DEV void rng_undo(Rng& s) {
  uint32_t u = xor3(s.v4, s.v3, s.v3 << 4);  // = u ^ (u << 1)
  u ^= u << 1;
  u ^= u << 2;
  u ^= u << 4;
  u ^= u << 8;
  u ^= u << 16;  // u
  u ^= u >> 2;
  u ^= u >> 4;
  u ^= u >> 8;
  u ^= u >> 16;  // v0
  s.v4 = s.v3;
  s.v3 = s.v2;
  s.v2 = s.v1;
  s.v1 = s.v0;
  s.v0 = u;
  s.d -= 362437u;
}
CVR_DEV float rng_float(Rng& s) {
  return det_fmaf((float)rng_next(s), 2.3283064e-10f, 1.1641532e-10f);
}

// ------------------------------------------------------ kernel params -----
struct MediumParams {
  const float* __restrict__ density;  // rx*ry*rz fp32, x fastest
  // Corner-replicated copy of the density for the Woodcock gathers: cell
  // (x,y,z) holds its 8 trilinear corners (texel-clamped as the reference's
  // point-sampled texture) in two float4 = 32 contiguous bytes, z planes
  // interleaved for the packed lerps (trilerp_cell), so one
  // evaluation is 2 x 16-byte loads from one cache line instead of 8 scattered
  // dword gathers.  Cells exist for 0 <= x1 < rx etc.; other corners (the Q5
  // uint wrap at -1, far out-of-range taps) use `density`.
  const float4* __restrict__ cells;   // 2 * rx*ry*rz float4, may be null
  const float4* __restrict__ albedo;  // rx*ry*rz float4 (rgb, w=1)
  // Brick bounds (DESIGN.md §Brick bounds): for each brick of 2^bshift cells
  // per axis, a u8 code c of an upper bound of every Woodcock test value
  // fl(fl(scale*rho)*inv_sigma) the brick's cells can give, as a minifloat
  // (bound_value: 4 exponent, 4 mantissa bits; 255 = 1.9375 = no bound, as
  // every test draw is <= 1).  A Woodcock tentative point whose brick bound is
  // below its test draw is a null collision whatever the exact density is, so
  // the cell is not fetched.  Entry bsentinel (one past the last brick) holds
  // 255: points off the cell grid read it.  May be null (every point is fetched).
  const uint8_t* __restrict__ bounds;
  uint32_t bshift, bnx, bny;  // brick size log2, bricks per x / y row
  uint32_t bnxy;              // bnx * bny (< 2^24)
  uint32_t bsentinel;         // index of the no-bound entry of bounds / sbounds
  // Sparse storage (cvr_set_medium_sparse; all null for a dense medium):
  // 8^3-voxel leaves, slot = leaves[leaf index] or CVR_NO_LEAF (density 0,
  // albedo albedo_bg).  `density`/`albedo` are then null, `cells` is the
  // cell-leaf pool (512 cells of 2 float4 per slot, slot 0 all zero) and
  // `sbounds` replaces `bounds`: per brick, c << 24 | cell-leaf slot.
  const uint32_t* __restrict__ leaves;
  const float* __restrict__ leaf_density;  // slot * 512 + local
  const float4* __restrict__ leaf_albedo;  // may be null: albedo_bg everywhere
  const uint32_t* __restrict__ sbounds;
  uint32_t lnx, lny;                       // leaves per x / y row
  V3 albedo_bg;
  uint32_t rx, ry, rz;
  uint32_t rxy;                  // rx * ry (< 2^24 for a dense medium)
  float fres_x, fres_y, fres_z;  // (float)res
  // Woodcock density coordinate -> grid: cx = (p - shift) * gx.  Default
  // (quirk Q4 reproduced): shift = box_min / extent (worldToAABB's operator
  // precedence, Utilities.cuh:129-132) and gx = res - 1 (volumeToGrid).
  // CVR_OPT_WORLD_TO_AABB 1: shift = box_min, gx = (res - 1) / extent, the
  // intended (p - min)/extent folded into the grid scale (no extra step code).
  float gx, gy, gz;
  float agx, agy, agz;  // (float)(res-1): the albedo lookup's volumeToGrid (AABB::transform coordinates)
  V3 bmin, bmax;
  V3 shift;
  float scale;
  float inv_sigma;   // 1 / (scale * max_density)
  float g;           // HG asymmetry (0 in the reference, Q7)
  float ax, ay;      // GGX roughness
  float eta;         // int_ior / ext_ior
  float inv_eta;     // 1.0f / eta
  // Dense media: every albedo voxel holds the same rgb (detected at cvr_set_medium,
  // CVR_OPT_UNIFORM_ALBEDO), stored in albedo_bg: the 8 taps of a collision's albedo
  // lookup are that constant, interpolated with the same operations, and nothing is
  // loaded (the same values, so the same result).  Last, so that the other fields
  // keep their kernel-argument offsets.
  uint32_t albedo_uniform;
  // Sparse media, the empty-region mask (round 5, cvr_set_medium_sparse): one bit
  // per super-brick of 2^eshift cells per axis (eshift >= 3, whole leaves), the
  // super-brick grid padded to powers of two per axis, bit sz << eshz | sy << eshy
  // | sx, set iff some leaf in it has a cell leaf, in kEmaskWords words.  Every brick word of a clear super-brick is 0 (bound code
  // 0, the zero cell leaf: k_build_sparse_bounds), so the wave pool, which stages
  // the mask in LDS, knows such a point's word without loading it
  // (woodcock_point_em).  Null: no mask (every bit set; also when the bricks are
  // unbounded, whose words are not 0).
  const uint32_t* emask;
  uint32_t eshift, eshy, eshz;
};
// Words of the empty-region mask (a power of two): 64 (2048 super-bricks, C5's
// cloud at 128^3 cells each), staged once per workgroup of the sparse instances,
// whose workgroups hold four wave-private pools (cvr_wpool.hip, kWpgSparse).  A
// finer mask costs the pools slots: 512 words (64^3 cells, 27% fewer word loads
// on C5) ran 114.4 ms against 112.9 with 64 (profiles/round6/ab/c5_wpg_mask_ab.log).
#ifndef CVR_WPOOL_EMASK_WORDS
#define CVR_WPOOL_EMASK_WORDS 64
#endif
constexpr int kEmaskWords = CVR_WPOOL_EMASK_WORDS;
// u64 index in the work area's counters (the diagnostic row, cvr_kernels.h kWorkDebug)
// of the brick words a counting launch loaded (CVR_OPT_COUNT_WORDS, cvr_stats.words)
constexpr uint32_t kStatWordsSlot = 24;
static_assert(kEmaskWords >= 64 && (kEmaskWords & (kEmaskWords - 1)) == 0, "mask words: a power of two >= 64");

// Brick-bound code -> bound (MediumParams::bounds): the float with bits
// (c << 19) + (112 << 23), one v_lshl_add_u32.  c = 16 e + m stands for
// 2^(e - 15) (1 + m / 16): 0 is 2^-15 (below every test draw but 2^-15 of
// them), 255 is 1.9375 (above every test draw: no bound).
constexpr uint32_t kBoundBias = 112u << 23;
CVR_DEV float bound_value(uint32_t c) { return __uint_as_float((c << 19) + kBoundBias); }

// u32 division by a launch-invariant divisor: q = (t + ((u - t) >> s1)) >> s2
// with t = mulhi(u, m) (round-up method, exact for every u32 and d >= 1;
// host side: cvr_api.cpp make_fastdiv).
struct FastDiv {
  uint32_t m, sh;  // sh = s1 | s2 << 8
};
CVR_DEV uint32_t fastdiv(uint32_t u, const FastDiv& f) {
  const uint32_t t = __umulhi(u, f.m);
  return (t + ((u - t) >> (f.sh & 0xFFu))) >> (f.sh >> 8);
}

struct LaunchParams {
  float M[12];            // c_inv_view_mat
  float r2v[2];           // c_raster_to_view
  float full_res[2];      // c_pixel_index_range
  float tile_res[2];      // c_resolution
  uint32_t off[2];        // c_offset
  uint32_t tile_px;       // (uint)(c_resolution.x * c_resolution.y)
  uint32_t tile_w;        // (uint)c_resolution.x
  uint32_t path_first;    // first path id of this launch
  uint32_t path_count;    // number of path ids
  uint32_t seed_base;     // RNG seed = seed_base + path_id
  uint32_t max_segments;  // safety cap (0 = none)
  float4* out;            // tile accumulator, tile_px float4
  unsigned int* queue;    // work-queue heads, one per 64-byte line (zeroed per launch)
  unsigned long long* stats;  // CVR_STAT_* counters (zeroed per launch)
  float4* pool_T;         // wave-pool scheduler: event-only slot part, grid * slots float4 (cvr_api wpool_slots)
  // Debug (cvr_trace_launch): the wave pool writes each path's final record
  // (cvr_path_record) at rec[path_id - path_first]; a u32 path-id array of
  // grid * slots entries sits just below rec.  Null in production.
  void* rec;
  uint32_t chunk;         // paths per wave dequeue
  uint16_t ev_thresh;     // persistent kernel: event batch threshold (lanes, <= 64)
  uint16_t tail;          // pool kernel: a wave leaves TRACK when the pool is dry and fewer lanes track
  uint32_t batch;         // wave-pool kernel: idle lanes that trigger a swap
  uint32_t naive_mk;      // bit 0: trace kernel runs naiveMK paths (walk_mk) instead of path_begin + loop;
                          // bit 1: pool kernel sorts each track phase's paths by Morton code (streamingSK)
  // Wave pool: bits 0-15 the drain rule (once the queues are empty, the launch's drain, an
  // event batch runs when waiting x drain >= tracking paths; 0: only when no lane tracks or
  // 64 events wait); kUnitSampleInner, kSplatCombine: see unit_to_path / splat_wave.
  uint32_t wflags;
  // Work order (scheduling only; results are bound to path ids).  order 0:
  // path ids in sample-major order from one queue.  order 1: 8x8-pixel
  // blocks with all their samples back to back (path_first must be a
  // multiple of tile_px, path_count = samples * tile_px, tile dims multiples
  // of 8); the block range is split into n_queues / sub contiguous bands, one
  // per XCD, so that the waves of one XCD share one band (its L2), and each
  // band into `sub` contiguous sub-queues (the wave pool: more queue heads,
  // so that small dequeue chunks do not contend on one atomic per XCD).
  // Queue q holds blocks [n_blocks q / n_queues, n_blocks (q+1) / n_queues).
  uint32_t order;
  uint32_t samples;       // path_count / tile_px (order 1)
  uint32_t blocks_x;      // tile_w / 8
  uint32_t n_blocks;      // blocks of this launch: tile_px / 64 (or the block shard's share)
  uint32_t n_queues;      // queues in all: bands (1..8) * sub
  uint32_t sub;           // sub-queues per band (1..8)
  // Block shard (cvr_set_block_shard): this launch's blocks are the tile's
  // blocks blk_off, blk_off + blk_stride, ...; local block b is tile block
  // blk_off + b * blk_stride (0 / 1: the whole tile).
  uint32_t blk_off, blk_stride;
  // Block order (cvr_set_block_order; null = natural): the b-th block of the
  // launch is block_perm[b] (a permutation of [0, n_blocks)), e.g. costly
  // blocks first so that the launch does not end on their long paths.
  const uint32_t* block_perm;
  // by tile_px, tile_w, 64*samples, blocks_x, n_queues
  FastDiv div_tile_px, div_tile_w, div_block, div_blocks_x, div_queues;
  // cvr_render_frame's in-launch output (wave pool, order 1, whole samples; null
  // otherwise): per tile block the number of its paths that have ended (block b at
  // frame_done[kDoneStride * b]), preceded by the FrameFlush header (frame_header()).
  // See cvr_wpool.hip, frame_flusher.
  unsigned int* frame_done;
};

// Header of the in-launch output (64 bytes just below LaunchParams::frame_done).
struct FrameFlush {
  float4* host;          // device address of the pinned host image (the tile's pixels)
  unsigned int* status;  // device address of pinned host words: [f] blocks flusher f stored,
                         // [kFrameFlushers] flushers that gave up waiting
  uint32_t host_w;       // host image row length in pixels
  float scale;           // the Scale functor's divisor (iterations)
  uint32_t give_up;      // test mode (CVR_OPT_FRAME_FLUSH 2): the flushers give up at once
  uint32_t pad[9];
};
static_assert(sizeof(FrameFlush) == 64, "FrameFlush is the 64-byte header below frame_done");
constexpr uint32_t kFrameFlushers = 8;  // the first workgroups of a flushing launch
// one count per 64-byte line: blocks dequeued together are counted by different
// waves at the same time, and atomics on one line serialise at the memory side
constexpr uint32_t kDoneStride = 16;
CVR_DEV const FrameFlush* frame_header(const unsigned int* done) {
  return reinterpret_cast<const FrameFlush*>(done) - 1;
}

// Map the u-th work unit of queue q to a path id (order 1), see LaunchParams.
// n_blocks * q < 2^24 (n_blocks <= 2^18, q <= 64).
CVR_DEV uint32_t queue_blocks_begin(const LaunchParams& L, uint32_t q) {
  return fastdiv(L.n_blocks * q, L.div_queues);  // n_blocks * q / n_queues
}
CVR_DEV uint32_t queue_units(const LaunchParams& L, uint32_t q) {
  if (L.order == 0) return q == 0 ? L.path_count : 0u;
  return (queue_blocks_begin(L, q + 1) - queue_blocks_begin(L, q)) * 64u * L.samples;
}
// Within a block the units run sample by sample, the block's 64 pixels
// innermost.  With kUnitSampleInner (round 5, CVR_OPT_SAMPLE_ORDER 1) they run
// pixel by pixel with the pixel's samples innermost instead, so the paths a
// wave holds at once belong to a few pixels and the escapes of one event batch
// mostly share pixels, whose framebuffer adds the batch then combines
// (splat_wave, kSplatCombine).  The pixel of unit rem of a block is then
// rem / samples = (rem << 6) / (64 samples), one fastdiv by the block divisor
// (exact while 64 * 64 * samples <= 2^32: the host keeps launches with more
// than 2^20 samples in path-id order).  Scheduling only: the same path ids.
constexpr uint32_t kDrainMask = 0xFFFFu, kUnitSampleInner = 1u << 16, kSplatCombine = 1u << 17;
CVR_DEV uint32_t unit_to_path(const LaunchParams& L, uint32_t q, uint32_t u) {
  if (L.order == 0) return L.path_first + u;
  const uint32_t per_block = 64u * L.samples;
  const uint32_t bq = fastdiv(u, L.div_block);
  uint32_t bl = queue_blocks_begin(L, q) + bq;
  if (L.block_perm) bl = gmem(L.block_perm)[bl];
  const uint32_t b = L.blk_off + __umul24(bl, L.blk_stride);
  const uint32_t rem = u - bq * per_block;
  uint32_t s, lane;
  if (L.wflags & kUnitSampleInner) {
    lane = fastdiv(rem << 6, L.div_block);
    s = rem - lane * L.samples;
  } else {
    s = rem >> 6;
    lane = rem & 63u;
  }
  const uint32_t by = fastdiv(b, L.div_blocks_x);
  const uint32_t px = (b - by * L.blocks_x) * 8u + (lane & 7u), py = by * 8u + (lane >> 3);
  return L.path_first + s * L.tile_px + py * L.tile_w + px;
}
// Tile block of the launch's bl-th block (order 1), as unit_to_path maps it.
CVR_DEV uint32_t launch_block_tile(const LaunchParams& L, uint32_t bl) {
  if (L.block_perm) bl = gmem(L.block_perm)[bl];
  return L.blk_off + __umul24(bl, L.blk_stride);
}
// Tile block (8x8 pixels, row-major) of a pixel of the tile.
CVR_DEV uint32_t tile_block_of(const LaunchParams& L, uint32_t image_id) {
  const uint32_t py = fastdiv(image_id, L.div_tile_w), px = image_id - py * L.tile_w;
  return (py >> 3) * L.blocks_x + (px >> 3);
}

enum {
  STAT_PATHS = 0,
  STAT_SEGMENTS,
  STAT_STEPS,
  STAT_DENSITY,
  STAT_ALBEDO,
  STAT_ESCAPED,
  STAT_TRUNCATED,
  STAT_FETCH,  // density cells actually fetched (the rest were bounded out)
  STAT_COUNT
};

// -------------------------------------------------------- grid lookup -----
// Volume.h:47-69 + RenderKernelLauncher.cu:20-25: point taps, clamp, the int
// index goes through uint so -1 clamps to res-1 (Q5).
CVR_DEV uint32_t texel(int i, uint32_t res) {
  const uint32_t u = (uint32_t)i;
  return u < res - 1u ? u : res - 1u;
}
CVR_DEV float lerpf(float a, float b, float f, float fi) { return det_fmaf(b, f, a * fi); }

struct Tri {
  uint32_t xa, xb, ya, yb, za, zb;
  float fx, fy, fz;
};
CVR_DEV Tri tri_setup(const MediumParams& m, V3 p, float gx, float gy, float gz) {
  const float cx = p.x * gx, cy = p.y * gy, cz = p.z * gz;
  const int x1 = det_floor_i32(cx), y1 = det_floor_i32(cy), z1 = det_floor_i32(cz);
  Tri t;
  t.fx = cx - (float)x1;
  t.fy = cy - (float)y1;
  t.fz = cz - (float)z1;
  t.xa = texel(x1, m.rx);
  t.xb = texel(x1 + 1, m.rx);
  t.ya = texel(y1, m.ry);
  t.yb = texel(y1 + 1, m.ry);
  t.za = texel(z1, m.rz);
  t.zb = texel(z1 + 1, m.rz);
  return t;
}
// Trilinear of one corner-replicated cell, the two z planes side by side so
// the x and y lerps run as packed pairs (v_pk_mul_f32 / v_pk_fma_f32): cell
// lo = (d000, d100, d001, d101), hi = (d010, d110, d011, d111), d{z}{y}{x}.
// Per value the operations are trilerp8's (x, then y, then z).
typedef float cvr_f2 __attribute__((ext_vector_type(2)));
CVR_DEV float trilerp_cell(float4 lo, float4 hi, float fx, float fy, float fz) {
  const cvr_f2 fx2 = {fx, fx}, fxi2 = {1.0f - fx, 1.0f - fx};
  const cvr_f2 fy2 = {fy, fy}, fyi2 = {1.0f - fy, 1.0f - fy};
  const cvr_f2 a0 = {lo.x, lo.y}, b0 = {lo.z, lo.w}, a1 = {hi.x, hi.y}, b1 = {hi.z, hi.w};
  const cvr_f2 x0 = __builtin_elementwise_fma(b0, fx2, a0 * fxi2);  // (z0 y0, z1 y0)
  const cvr_f2 x1 = __builtin_elementwise_fma(b1, fx2, a1 * fxi2);  // (z0 y1, z1 y1)
  const cvr_f2 y = __builtin_elementwise_fma(x1, fy2, x0 * fyi2);   // (z0, z1)
  return lerpf(y.x, y.y, fz, 1.0f - fz);
}
CVR_DEV float trilerp8(float d000, float d001, float d010, float d011, float d100, float d101, float d110,
                       float d111, float fx, float fy, float fz) {
  const float _fx = 1.0f - fx, _fy = 1.0f - fy, _fz = 1.0f - fz;
  const float a = lerpf(lerpf(d000, d001, fx, _fx), lerpf(d010, d011, fx, _fx), fy, _fy);
  const float b = lerpf(lerpf(d100, d101, fx, _fx), lerpf(d110, d111, fx, _fx), fy, _fy);
  return lerpf(a, b, fz, _fz);
}

// Texel fetch from the dense grid or the sparse leaves (same value).
CVR_DEV uint32_t leaf_local(uint32_t x, uint32_t y, uint32_t z) {
  return ((z & 7u) << 6) | ((y & 7u) << 3) | (x & 7u);
}
CVR_DEV float texel_density(const MediumParams& m, uint32_t x, uint32_t y, uint32_t z) {
  if (m.leaves) {
    const uint32_t slot = m.leaves[(__umul24(z >> 3, m.lny) + (y >> 3)) * m.lnx + (x >> 3)];
    return slot == 0xFFFFFFFFu ? 0.0f : m.leaf_density[((size_t)slot << 9) | leaf_local(x, y, z)];
  }
  return m.density[(z * m.ry + y) * m.rx + x];
}
CVR_DEV float4 texel_albedo(const MediumParams& m, uint32_t x, uint32_t y, uint32_t z) {
  if (m.leaves) {
    const uint32_t slot = m.leaf_albedo ? m.leaves[(__umul24(z >> 3, m.lny) + (y >> 3)) * m.lnx + (x >> 3)]
                                        : 0xFFFFFFFFu;
    return slot == 0xFFFFFFFFu ? make_float4(m.albedo_bg.x, m.albedo_bg.y, m.albedo_bg.z, 1.0f)
                               : m.leaf_albedo[((size_t)slot << 9) | leaf_local(x, y, z)];
  }
  if (m.albedo_uniform) return make_float4(m.albedo_bg.x, m.albedo_bg.y, m.albedo_bg.z, 1.0f);
  return m.albedo[(z * m.ry + y) * m.rx + x];
}

// The reference's 8-tap trilinear (Volume.h:47-69), used where no cell
// applies (the Q5 wrap, points outside the grid).
CVR_DEV float density_lookup_gather(const MediumParams& m, V3 p) {
  const Tri t = tri_setup(m, p, m.gx, m.gy, m.gz);
  const float d000 = texel_density(m, t.xa, t.ya, t.za), d001 = texel_density(m, t.xb, t.ya, t.za);
  const float d010 = texel_density(m, t.xa, t.yb, t.za), d011 = texel_density(m, t.xb, t.yb, t.za);
  const float d100 = texel_density(m, t.xa, t.ya, t.zb), d101 = texel_density(m, t.xb, t.ya, t.zb);
  const float d110 = texel_density(m, t.xa, t.yb, t.zb), d111 = texel_density(m, t.xb, t.yb, t.zb);
  const float _fx = 1.0f - t.fx, _fy = 1.0f - t.fy, _fz = 1.0f - t.fz;
  const float a = lerpf(lerpf(d000, d001, t.fx, _fx), lerpf(d010, d011, t.fx, _fx), t.fy, _fy);
  const float b = lerpf(lerpf(d100, d101, t.fx, _fx), lerpf(d110, d111, t.fx, _fx), t.fy, _fy);
  return lerpf(a, b, t.fz, _fz);
}
CVR_DEV V3 albedo_lookup(const MediumParams& m, V3 p) {
  const Tri t = tri_setup(m, p, m.agx, m.agy, m.agz);
  const float _fx = 1.0f - t.fx, _fy = 1.0f - t.fy, _fz = 1.0f - t.fz;
  // one z plane at a time (same operations as the 8-tap form: x, then y
  // lerps per plane, then z), so at most 4 texels are live
  V3 a, b;
  {
    const float4 d000 = texel_albedo(m, t.xa, t.ya, t.za), d001 = texel_albedo(m, t.xb, t.ya, t.za);
    const float4 d010 = texel_albedo(m, t.xa, t.yb, t.za), d011 = texel_albedo(m, t.xb, t.yb, t.za);
    a = mk3(lerpf(lerpf(d000.x, d001.x, t.fx, _fx), lerpf(d010.x, d011.x, t.fx, _fx), t.fy, _fy),
            lerpf(lerpf(d000.y, d001.y, t.fx, _fx), lerpf(d010.y, d011.y, t.fx, _fx), t.fy, _fy),
            lerpf(lerpf(d000.z, d001.z, t.fx, _fx), lerpf(d010.z, d011.z, t.fx, _fx), t.fy, _fy));
  }
  // keep the second plane's loads after the first plane's lerps (otherwise
  // the scheduler issues all 8 loads first: 32 live VGPRs at the peak)
  __builtin_amdgcn_sched_barrier(0);
  {
    const float4 d100 = texel_albedo(m, t.xa, t.ya, t.zb), d101 = texel_albedo(m, t.xb, t.ya, t.zb);
    const float4 d110 = texel_albedo(m, t.xa, t.yb, t.zb), d111 = texel_albedo(m, t.xb, t.yb, t.zb);
    b = mk3(lerpf(lerpf(d100.x, d101.x, t.fx, _fx), lerpf(d110.x, d111.x, t.fx, _fx), t.fy, _fy),
            lerpf(lerpf(d100.y, d101.y, t.fx, _fx), lerpf(d110.y, d111.y, t.fx, _fx), t.fy, _fy),
            lerpf(lerpf(d100.z, d101.z, t.fx, _fx), lerpf(d110.z, d111.z, t.fx, _fx), t.fy, _fy));
  }
  return mk3(lerpf(a.x, b.x, t.fz, _fz), lerpf(a.y, b.y, t.fz, _fz), lerpf(a.z, b.z, t.fz, _fz));
}

// ---------------------------------------------------------------- AABB ----
// Geometry.h:55-92.  `normal` persists when no plane matches.
struct Isect {
  float dist;
  V3 normal;
  bool inside;
};
CVR_DEV bool aabb_intersect(const MediumParams& m, V3 o, V3 d, Isect& is) {
  const V3 invR = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const V3 tbot = mul3(invR, sub3(m.bmin, o));
  const V3 ttop = mul3(invR, sub3(m.bmax, o));
  const V3 tmin = mk3(det_fminf(ttop.x, tbot.x), det_fminf(ttop.y, tbot.y), det_fminf(ttop.z, tbot.z));
  const V3 tmax = mk3(det_fmaxf(ttop.x, tbot.x), det_fmaxf(ttop.y, tbot.y), det_fmaxf(ttop.z, tbot.z));
  const float largest_tmin = det_fmaxf(det_fmaxf(tmin.x, tmin.y), det_fmaxf(tmin.x, tmin.z));
  const float smallest_tmax = det_fminf(det_fminf(tmax.x, tmax.y), det_fminf(tmax.x, tmax.z));
  is.dist = (largest_tmin > CVR_EPSILON_F) ? largest_tmin : smallest_tmax;
  if (is.dist == ttop.x) is.normal = mk3(1, 0, 0);
  else if (is.dist == ttop.y) is.normal = mk3(0, 1, 0);
  else if (is.dist == ttop.z) is.normal = mk3(0, 0, 1);
  else if (is.dist == tbot.x) is.normal = mk3(-1, 0, 0);
  else if (is.dist == tbot.y) is.normal = mk3(0, -1, 0);
  else if (is.dist == tbot.z) is.normal = mk3(0, 0, -1);
  is.inside = dot3(is.normal, d) > 0.0f;
  return (smallest_tmax > largest_tmin) && (is.dist > 0.0f);
}

// ---------------------------------------------------------- Woodcock ------
// One Woodcock step (Utilities.cuh:134-136,148-152).  Returns 0 = keep
// tracking, 1 = tentative t beyond max_t (no collision), 2 = accepted.
//
// The test value is drawn before the density is looked up: the reference
// draws it right after the lookup and nothing in between consumes the RNG,
// so the stream is the same.  Brick bounds (MediumParams::bounds): the exact
// test is !(fl(fl(scale*rho)*inv_sigma) < xi) with rho the trilinear density
// of the cell, and rho <= mx*(1 + 9u) for mx the brick's largest density
// (three fma lerps of values <= mx), so fl(fl(scale*rho)*inv_sigma) <=
// mx/max_density*(1 + 14u) <= bound_value(c) (k_build_bounds' bound_code):
// when that bound is below xi the point is a null collision whatever rho is,
// and the cell is not fetched.  Points whose lower corner lies outside the
// grid (quirk Q5 taps, NaN) read the sentinel entry (no bound) and the 8-tap
// gather.
//
// Result: 0 null collision (continue), 1 t > max_t (no density evaluation),
// 2 real collision with t < max_t, 3 real collision at t == max_t (the
// reference scatters iff t < max_t, so this ends the segment at the box).
// Every step but a 1 evaluates the density once.
// Tentative point of a Woodcock step: its cell, brick bound and cell pointer.
struct WoodcockPoint {
  V3 c;                 // worldToAABB coordinate (Q4)
  float cx, cy, cz;     // grid coordinate (DeviceVolume::volumeToGrid)
  bool in;              // lower corner inside the grid (cell path), else the 8-tap gather
  float qb;             // brick bound (bound_value; 1.9375: no bound)
  const float4* cp;     // the cell's two float4 (valid when in && m.cells)
};
CVR_DEV void woodcock_coords(const MediumParams& m, V3 o, V3 d, float t, WoodcockPoint& P) {
  P.c = sub3(mk3(det_fmaf(t, d.x, o.x), det_fmaf(t, d.y, o.y), det_fmaf(t, d.z, o.z)), m.shift);
  // fma(c, g, +0) is the product c*g rounded once, except that a -0 product
  // becomes +0 (-0 + +0 = +0); the trilinear weights cx - floor(cx) and the
  // cell index are the same for both zeros.
  P.cx = det_fmaf(P.c.x, m.gx, 0.0f);
  P.cy = det_fmaf(P.c.y, m.gy, 0.0f);
  P.cz = det_fmaf(P.c.z, m.gz, 0.0f);
  // floor(cx) >= 0 && floor(cx) < res  <=>  0 <= cx < res (res an integer)
  // <=>  bits(cx) < bits(res) as unsigned: non-negative floats order as
  // their bit patterns, negatives and -NaN have the sign bit set, +NaN lies
  // above +inf, and cx is never -0 (above).  One compare per axis, one mask.
  P.in = ((int)(det_f2u(P.cx) < det_f2u(m.fres_x)) & (int)(det_f2u(P.cy) < det_f2u(m.fres_y)) &
          (int)(det_f2u(P.cz) < det_f2u(m.fres_z))) != 0;
}
CVR_DEV WoodcockPoint woodcock_point(const MediumParams& m, V3 o, V3 d, float t) {
  WoodcockPoint P;
  woodcock_coords(m, o, d, t, P);
  // The cell and brick indices only mean something when in: off the grid the
  // brick index is replaced by the sentinel entry (no bound) and the cell
  // pointer is never used (the 8-tap gather).  In the grid 0 <= cx < 2^24, so
  // the truncating conversion is floor(cx) (Volume.h:52, (int)floorf) with no
  // v_floor.  24-bit multiplies: the host keeps bnx*bny, rx*ry and ry*rz below 2^24.
  const uint32_t x1 = (uint32_t)P.cx, y1 = (uint32_t)P.cy, z1 = (uint32_t)P.cz;
  const uint32_t bx = x1 >> m.bshift, by = y1 >> m.bshift, bz = z1 >> m.bshift;
  const uint32_t bi = P.in ? __umul24(bz, m.bnxy) + __umul24(by, m.bnx) + bx : m.bsentinel;
  if (m.sbounds) {  // sparse: bound and cell-leaf slot in one word
    const uint32_t sw = m.sbounds[bi];
    P.qb = bound_value(sw >> 24);
    P.cp = m.cells + ((((size_t)(sw & 0xFFFFFFu)) << 9 | leaf_local(x1, y1, z1)) << 1);
  } else {
    uint32_t q = 255u;
    if (m.bounds) q = m.bounds[bi];
    P.qb = bound_value(q);
    P.cp = m.cells + 2 * (__umul24(z1, m.rxy) + __umul24(y1, m.rx) + x1);
  }
  return P;
}
// woodcock_point on a sparse medium with the empty-region mask staged in LDS
// (em: MediumParams::emask's kWords words).  The same point, bound and cell
// pointer; the brick word is loaded only when the point's super-brick has a
// cell leaf: in a clear one it is 0 (bound code 0, the zero cell leaf), and off
// the grid the sentinel's (255 << 24, slot 0), both known without a load.
// n_words (counting instances only, CVR_OPT_COUNT_WORDS): += 1 per brick word loaded.
template <int kWords, class EmWords>
CVR_DEV WoodcockPoint woodcock_point_em(const MediumParams& m, V3 o, V3 d, float t, const EmWords& em,
                                        uint32_t* n_words = nullptr) {
  WoodcockPoint P;
  woodcock_coords(m, o, d, t, P);
  const uint32_t x1 = (uint32_t)P.cx, y1 = (uint32_t)P.cy, z1 = (uint32_t)P.cz;
  // (off the grid x1.. are meaningless: the word index is masked into the array,
  // so the LDS read needs no branch; shifts and v_lshl_or, no multiplies)
  const uint32_t sb = ((z1 >> m.eshift) << m.eshz) | ((y1 >> m.eshift) << m.eshy) | (x1 >> m.eshift);
  const uint32_t word = em[(sb >> 5) & (uint32_t)(kWords - 1)];
  const bool load = P.in & (__builtin_amdgcn_ubfe(word, sb & 31u, 1u) != 0u);
  uint32_t sw = P.in ? 0u : 255u << 24;
  if (load) sw = m.sbounds[__umul24(z1 >> m.bshift, m.bnxy) + __umul24(y1 >> m.bshift, m.bnx) + (x1 >> m.bshift)];
  if (n_words) *n_words += load ? 1u : 0u;
  P.qb = bound_value(sw >> 24);
  P.cp = m.cells + ((((size_t)(sw & 0xFFFFFFu)) << 9 | leaf_local(x1, y1, z1)) << 1);
  return P;
}

// The exact density at the point (cell trilinear or the 8-tap gather).
CVR_DEV float woodcock_density(const MediumParams& m, const WoodcockPoint& P) {
  if (P.in && m.cells) {
    const float4 lo = P.cp[0], hi = P.cp[1];
    // cx - floorf(cx) (Volume.h:56-58): exact for 0 <= cx, which is what v_fract_f32 returns
    return trilerp_cell(lo, hi, __builtin_amdgcn_fractf(P.cx), __builtin_amdgcn_fractf(P.cy),
                        __builtin_amdgcn_fractf(P.cz));
  }
  return density_lookup_gather(m, P.c);
}
// == det_logf(det_fmaxf(xi, EPSILON)) * -inv_sigma + t: xi is never NaN and
// the clamped argument is a normal float, so the NaN and subnormal paths are
// dropped, and the clamp is one v_max_f32 (maxnum, which equals det_fmaxf
// for a non-NaN xi).
CVR_DEV float woodcock_advance(const MediumParams& m, float xi, float t) {
  return det_fmaf(-det_logf_normal(__builtin_fmaxf(xi, CVR_EPSILON_F)), m.inv_sigma, t);
}

CVR_DEV int woodcock_step_core(const MediumParams& m, V3 o, V3 d, float max_t, float& t, Rng& rng,
                               uint32_t& n_fetch) {
  t = woodcock_advance(m, rng_float(rng), t);
  if (!(t <= max_t)) return 1;
  WoodcockPoint P = woodcock_point(m, o, d, t);
  const float xi_test = rng_float(rng);
  if (P.qb < xi_test) return 0;  // bounded out (brick bound)
  ++n_fetch;
  const float rho = m.scale * woodcock_density(m, P);
  if (!(rho * m.inv_sigma < xi_test)) return t < max_t ? 2 : 3;
  return 0;
}
// Per-lane counting wrapper: 0 continue, 1 t > max_t, 2 real collision
// (the caller scatters iff also t < max_t).
CVR_DEV int woodcock_step(const MediumParams& m, V3 o, V3 d, float max_t, float& t, Rng& rng,
                          uint32_t& n_steps, uint32_t& n_density, uint32_t& n_fetch) {
  ++n_steps;
  const int r = woodcock_step_core(m, o, d, max_t, t, rng, n_fetch);
  n_density += r != 1;
  return r == 3 ? 2 : r;
}

// --------------------------------------------------------------- HG -------
// HG.h:11-63
CVR_DEV V3 hg_sample(V3 v, float g, float e1, float e2) {
  float cosT;
  if (det_fabsf(g) > CVR_EPSILON_F) {
    const float sq = (1.0f - g * g) / ((1.0f - g) + (2.0f * g) * e1);
    cosT = ((1.0f + g * g) - sq * sq) / (2.0f * det_fabsf(g));
  } else {
    cosT = 1.0f - 2.0f * e1;
  }
  const float sinT = det_sqrtf(det_fmaxf(0.0f, 1.0f - cosT * cosT));
  const float phi = CVR_TWOPI_F * e2;
  const float invN = 1.0f / det_sqrtf(v.x * v.x + v.z * v.z);
  const V3 v1 = mk3(v.z * invN, 0.0f, (-v.x) * invN);
  const V3 v2 = cross3(v, v1);
  float sp, cp;
  det_sincosf(phi, &sp, &cp);
  return add3(add3(scl3(v1, sinT * cp), scl3(v2, sinT * sp)), scl3(v, cosT));
}

// -------------------------------------------------------------- GGX -------
// GGX.h:13-38
CVR_DEV float fresnel_dielectric(float eta, float inv_eta, float ndotwi, float& ndotwt) {
  if (eta == 1.0f) {
    ndotwt = -ndotwi;
    return 0.0f;
  }
  const float scale = (ndotwi > 0.0f) ? inv_eta : eta;  // inv_eta = 1.0f / eta (host, same IEEE quotient)
  const float sin_sqr = 1.0f - ndotwi * ndotwi;
  const float ndotwt_sqr = 1.0f - (sin_sqr * scale) * scale;
  if (ndotwt_sqr <= 0.0f) {
    ndotwt = 0.0f;
    return 1.0f;
  }
  const float a_wi = det_fabsf(ndotwi);
  const float a_wt = det_sqrtf(ndotwt_sqr);
  const float Rs = (a_wi - eta * a_wt) / (a_wi + eta * a_wt);
  const float Rp = (eta * a_wi - a_wt) / (eta * a_wi + a_wt);
  ndotwt = (ndotwi > 0.0f) ? -a_wt : a_wt;
  return 0.5f * (Rs * Rs + Rp * Rp);
}
// GGX.h:85-144
CVR_DEV void sample_visible11(float thetaI, float sx, float sy, float& ox, float& oy) {
  const float phi = (2.0f * CVR_PI_F) * sy;
  if (thetaI < 1e-4f) {
    const float r = det_sqrtf(det_fmaxf(0.0f, sx / (1.0f - sx)));
    float sp, cp;
    det_sincosf(phi, &sp, &cp);
    ox = r * cp;
    oy = r * sp;
    return;
  }
  const float tanThetaI = det_tanf(thetaI);
  float a = 1.0f / tanThetaI;
  a = 1.0f + (1.0f / (a * a));
  const float G1 = 2.0f / (1.0f + det_sqrtf(a));
  float A = ((2.0f * sx) / G1) - 1.0f;
  if (det_fabsf(A) == 1.0f) A -= (A < 0.0f ? -1.0f : 1.0f) * CVR_EPSILON_F;
  const float tmp = 1.0f / (A * A - 1.0f);
  const float B = tanThetaI;
  const float D = det_sqrtf(det_fmaxf(0.0f, ((B * B) * tmp) * tmp - (A * A - B * B) * tmp));
  const float s1 = B * tmp - D, s2 = B * tmp + D;
  const float slope_x = (A < 0.0f || s2 > 1.0f / tanThetaI) ? s1 : s2;
  float S;
  if (sy > 0.5f) {
    S = 1.0f;
    sy = 2.0f * (sy - 0.5f);
  } else {
    S = -1.0f;
    sy = 2.0f * (0.5f - sy);
  }
  const float z =
      (sy * (sy * (sy * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) +
       0.000152998850436920f) /
      (sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) +
             1.0f) -
       0.539825872510702f);
  ox = slope_x;
  oy = (S * z) * det_sqrtf(1.0f + slope_x * slope_x);
}
// GGX.h:146-181
CVR_DEV V3 ggx_sample_vndf(V3 wi_, float ax, float ay, float sx, float sy) {
  const V3 wi = normalize3(mk3(ax * wi_.x, ay * wi_.y, wi_.z));
  float theta = 0.0f, phi = 0.0f;
  if (wi.z < 0.999999f) {
    theta = det_acosf(wi.z);
    phi = det_atan2f(wi.y, wi.x);
  }
  float sinPhi, cosPhi;
  det_sincosf(phi, &sinPhi, &cosPhi);
  float slx, sly;
  sample_visible11(theta, sx, sy, slx, sly);
  float rx = cosPhi * slx - sinPhi * sly;
  float ry = sinPhi * slx + cosPhi * sly;
  rx *= ax;
  ry *= ay;
  const float n = 1.0f / det_sqrtf(rx * rx + ry * ry + 1.0f);
  return mk3(-rx * n, -ry * n, n);
}
// GGX.h:213-255
CVR_DEV float project_roughness(V3 v, float ax, float ay) {
  if (ax == ay) return ax;  // isotropic (the reference's 0.1, 0.1): no division needed
  const float invSinTheta2 = 1.0f / (1.0f - v.z * v.z);
  if (invSinTheta2 <= 0.0f) return ax;
  const float cosPhi2 = v.x * v.x * invSinTheta2;
  const float sinPhi2 = v.y * v.y * invSinTheta2;
  return det_sqrtf(cosPhi2 * ax * ax + sinPhi2 * ay * ay);
}
CVR_DEV float ggx_g1(float ax, float ay, V3 v, V3 m) {
  if (dot3(v, m) * v.z <= 0.0f) return 0.0f;
  const float temp = 1.0f - v.z * v.z;
  if (temp <= 0.0f) return 0.0f;
  const float tn = det_fabsf(det_sqrtf(temp) / v.z);
  if (tn == 0.0f) return 1.0f;
  const float root = project_roughness(v, ax, ay) * tn;
  return 2.0f / (1.0f + det_sqrtf(1.0f + root * root));
}
// GGX.h:265-326; `wo` aliases the path direction (Q8).
CVR_DEV bool ggx_sample(const MediumParams& m, V3 wi, Rng& rng, V3& wo, float& weight) {
  const float ndotwi = wi.z;
  if (ndotwi == 0.0f) {
    weight = 0.0f;
    return false;
  }
  weight = 1.0f;
  // wi.z / |wi.z| is +-1 exactly for a finite wi.z (!= 0 here); the
  // division itself runs only for inf/NaN (same NaN as before)
  float sign;
  if (det_fabsf(wi.z) <= 3.40282347e38f) sign = wi.z > 0.0f ? 1.0f : -1.0f;
  else sign = wi.z / det_fabsf(wi.z);
  const float s0 = rng_float(rng);
  const float s1 = rng_float(rng);
  const V3 wh = ggx_sample_vndf(scl3(wi, sign), m.ax, m.ay, s0, s1);
  float whdotwt = __builtin_nanf("");
  const float whdotwi = dot3(wh, wi);
  const float F = fresnel_dielectric(m.eta, m.inv_eta, whdotwi, whdotwt);
  if (rng_float(rng) <= F) {
    wo = sub3(scl3(wh, 2.0f * whdotwi), wi);
    if (wi.z * wo.z <= 0.0f) {
      weight = 0.0f;
      return false;
    }
  } else {
    if (whdotwt == 0.0f) {
      weight = 0.0f;
      return false;
    }
    float eta = m.eta;
    if (whdotwt < 0.0f) eta = m.inv_eta;
    wo = sub3(scl3(wh, whdotwi * eta + whdotwt), scl3(wi, eta));
    if (wi.z * wo.z >= 0.0f) {
      weight = 0.0f;
      return false;
    }
  }
  weight *= ggx_g1(m.ax, m.ay, wo, wh);
  return true;
}

// ------------------------------------------------------------- frame ------
// CVRMath.h:58-91
struct Frame {
  V3 x, y, z;
};
// normalize3(v) is v itself, bit for bit, when dot(v, v) == 1 exactly
// (sqrt(1) = 1, 1/1 = 1, v*1 = v): the AABB normals and their cross
// products with the frame's helper axis take this branch and skip the
// square root and the division.
CVR_DEV V3 normalize3_unit_fast(V3 v) {
  if (dot3(v, v) == 1.0f) return v;
  return normalize3(v);
}
CVR_DEV Frame frame_from_z(V3 n) {
  Frame f;
  f.z = normalize3_unit_fast(n);
  const V3 tx = (det_fabsf(f.z.x) > 0.99f) ? mk3(0, 1, 0) : mk3(1, 0, 0);
  f.y = normalize3_unit_fast(cross3(f.z, tx));
  f.x = cross3(f.y, f.z);
  return f;
}
CVR_DEV V3 frame_to_local(const Frame& f, V3 a) { return mk3(dot3(a, f.x), dot3(a, f.y), dot3(a, f.z)); }
CVR_DEV V3 frame_to_world(const Frame& f, V3 a) {
  return add3(add3(scl3(f.x, a.x), scl3(f.y, a.y)), scl3(f.z, a.z));
}

// ------------------------------------------------------------ camera ------
// NaiveVolPTsk_kernel.cuh:22-31 / RegenerationVolPTsk_kernel.cuh:169-177 and
// Utilities.cuh:180-213: path_id -> (image_id, seeded RNG, camera ray).
struct PathState {
  Rng rng;
  V3 o, d, T;
  uint32_t image_id;
};
// Camera ray of pixel ps.image_id drawn from ps.rng (indexToCameraRay,
// Utilities.cuh:180-213).
CVR_DEV void camera_ray(const LaunchParams& L, PathState& ps);
CVR_DEV void path_begin(const LaunchParams& L, uint32_t path_id, PathState& ps) {
  ps.image_id = path_id - fastdiv(path_id, L.div_tile_px) * L.tile_px;  // path_id % tile_px
  rng_init(ps.rng, (int32_t)(L.seed_base + path_id));
  camera_ray(L, ps);
}
CVR_DEV void camera_ray(const LaunchParams& L, PathState& ps) {
  const float px = (float)(ps.image_id - fastdiv(ps.image_id, L.div_tile_w) * L.tile_w) + (float)L.off[0];
  const float py = det_floorf((float)ps.image_id / L.tile_res[0]) + (float)L.off[1];
  const float r0 = rng_float(ps.rng);
  const float r1 = rng_float(ps.rng);
  float rx = ((px + r0) * 2.0f) / L.full_res[0] - 1.0f;
  float ry = ((py + r1) * 2.0f) / L.full_res[1] - 1.0f;
  rx = L.r2v[0] * rx;
  ry = L.r2v[1] * ry;
  const float* M = L.M;
  ps.o = mk3(0.0f * M[0] + 0.0f * M[1] + 0.0f * M[2] + 1.0f * M[3],
             0.0f * M[4] + 0.0f * M[5] + 0.0f * M[6] + 1.0f * M[7],
             0.0f * M[8] + 0.0f * M[9] + 0.0f * M[10] + 1.0f * M[11]);
  const V3 v = normalize3(mk3(rx, ry, 1.0f));
  ps.d = mk3(dot3(v, mk3(M[0], M[1], M[2])), dot3(v, mk3(M[4], M[5], M[6])),
             dot3(v, mk3(M[8], M[9], M[10])));
  ps.T = mk3(1.0f, 1.0f, 1.0f);
}

// Boundary event (NaiveVolPTsk_kernel.cuh:53-65): GGX at the AABB surface.
CVR_DEV void boundary_event(const MediumParams& m, PathState& ps, const Isect& is) {
  const Frame fr = frame_from_z(is.normal);
  const V3 dir = frame_to_local(fr, normalize3(neg3(ps.d)));
  ps.o = add3(ps.o, scl3(ps.d, is.dist));
  float weight = 1.0f;
  if (ggx_sample(m, dir, ps.rng, ps.d, weight)) {
    ps.T = scl3(ps.T, weight);
    ps.d = frame_to_world(fr, ps.d);
    ps.o = add3(ps.o, scl3(ps.d, CVR_EPSILON_F));
  }
}
// Real collision (NaiveVolPTsk_kernel.cuh:66-72; regeneration :212 has no -eps).
template <bool kScatterEps>
CVR_DEV void scatter_event(const MediumParams& m, PathState& ps, float t) {
  ps.o = add3(ps.o, scl3(ps.d, t));
  if (kScatterEps) ps.o = sub3(ps.o, scl3(ps.d, CVR_EPSILON_F));
  const V3 a = albedo_lookup(m, div3(sub3(ps.o, m.bmin), sub3(m.bmax, m.bmin)));
  ps.T = mul3(ps.T, a);
  const float e1 = rng_float(ps.rng);
  const float e2 = rng_float(ps.rng);
  ps.d = hg_sample(ps.d, m.g, e1, e2);
}
// Russian roulette (NaiveVolPTsk_kernel.cuh:75-84).  Returns false = path dies.
CVR_DEV bool roulette(PathState& ps) {
  const float p = det_fminf(1.0f, det_fmaxf(det_fmaxf(ps.T.x, ps.T.y), ps.T.z));
  if (rng_float(ps.rng) > p) return false;
  ps.T = mk3(ps.T.x / p, ps.T.y / p, ps.T.z / p);
  return true;
}
// atomicVectorAdd (Utilities.cuh:15-22) with Le = 1.
CVR_DEV void splat(const LaunchParams& L, const PathState& ps) {
  gptr_t<float> px = gmem(reinterpret_cast<float*>(L.out + ps.image_id));
  // A zero component is not added: a pixel is never -0 (cleared to +0, and every
  // contribution is >= +0 or NaN: albedo and G1 factors are >= 0, roulette divides by
  // p > 0), so x + 0 == x and the sum is the same.  After one collision in a medium
  // with albedo (d, 0, 0) (the MHD converter's, mhd_to_vdb.py:62-64) two of the
  // three atomics go.
  if (ps.T.x != 0.0f) __hip_atomic_fetch_add(px + 0, ps.T.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ps.T.y != 0.0f) __hip_atomic_fetch_add(px + 1, ps.T.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ps.T.z != 0.0f) __hip_atomic_fetch_add(px + 2, ps.T.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // w = 1 (Utilities.cuh:21, a plain store there) as a memory-side atomic swap: a plain
  // store leaves the pixel's line dirty in this XCD's L2 while the rgb atomics are
  // performed at the memory side, and the mix cost C2 1.3% and C3 1.5% of kernel time
  // (profiles/round3/ab/splat_w/).  Same value, same image.
  (void)__hip_atomic_exchange(reinterpret_cast<gptr_t<unsigned int>>(px + 3), 0x3F800000u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ naiveMK -----
// utilhash / makeSeededRng (Utilities.cuh:157-178): naiveMK re-seeds the RNG
// from (iteration, pixel, depth) at every kernel launch.
CVR_DEV uint32_t utilhash(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}
CVR_DEV void rng_seeded(Rng& s, uint32_t iteration, uint32_t index, uint32_t depth) {
  rng_init(s, (int32_t)(utilhash(0x80000000u | (depth << 22) | iteration) ^ utilhash(index)));
}

// NaiveVolPTmk_kernel::d_init (NaiveVolPTmk_kernel.cuh:20-77) for path id
// = iteration * tile_px + image_id: camera ray on the (iteration, pixel, 0)
// stream, AABB test, then the GGX sample at the box before any medium test
// (Q12).  Returns MK_ALIVE (ps holds the path for the first d_extend),
// MK_MISSED (the box was missed: the pixel gets (1,1,1)) or MK_DROPPED (a
// failed GGX sample: no contribution).
enum : uint32_t { MK_ALIVE = 0, MK_MISSED = 1, MK_DROPPED = 2, MK_ESCAPED = 3, MK_DIED = 4, MK_TRUNCATED = 5 };
CVR_DEV uint32_t mk_init(const MediumParams& m, const LaunchParams& L, uint32_t iteration, uint32_t image_id,
                         PathState& ps) {
  ps.image_id = image_id;
  rng_seeded(ps.rng, iteration, image_id, 0u);
  {
    // camera ray as path_begin, on the (iteration, pixel, 0) stream
    const float px = (float)(image_id % L.tile_w) + (float)L.off[0];
    const float py = det_floorf((float)image_id / L.tile_res[0]) + (float)L.off[1];
    const float r0 = rng_float(ps.rng);
    const float r1 = rng_float(ps.rng);
    float rx = ((px + r0) * 2.0f) / L.full_res[0] - 1.0f;
    float ry = ((py + r1) * 2.0f) / L.full_res[1] - 1.0f;
    rx = L.r2v[0] * rx;
    ry = L.r2v[1] * ry;
    const float* M = L.M;
    ps.o = mk3(0.0f * M[0] + 0.0f * M[1] + 0.0f * M[2] + 1.0f * M[3],
               0.0f * M[4] + 0.0f * M[5] + 0.0f * M[6] + 1.0f * M[7],
               0.0f * M[8] + 0.0f * M[9] + 0.0f * M[10] + 1.0f * M[11]);
    const V3 v = normalize3(mk3(rx, ry, 1.0f));
    ps.d = mk3(dot3(v, mk3(M[0], M[1], M[2])), dot3(v, mk3(M[4], M[5], M[6])), dot3(v, mk3(M[8], M[9], M[10])));
  }
  ps.T = mk3(1.0f, 1.0f, 1.0f);
  Isect is;
  is.dist = 0.0f;
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  if (!aabb_intersect(m, ps.o, ps.d, is)) return MK_MISSED;
  if (is.dist < 0.0f) is.dist = 0.0f;  // clamp to near plane
  ps.o = add3(ps.o, scl3(ps.d, is.dist));
  const Frame fr = frame_from_z(is.normal);
  const V3 dir = frame_to_local(fr, normalize3(neg3(ps.d)));
  float weight = 1.0f;
  if (!ggx_sample(m, dir, ps.rng, ps.d, weight)) return MK_DROPPED;
  ps.T = scl3(ps.T, weight);
  ps.d = frame_to_world(fr, ps.d);
  ps.o = add3(ps.o, scl3(ps.d, CVR_EPSILON_F));
  return MK_ALIVE;
}

// One NaiveVolPTmk_kernel::d_extend bounce (NaiveVolPTmk_kernel.cuh:79-151)
// of a live path at `depth`: re-seed from (iteration, pixel, depth), three
// unused draws (Q12), one naiveSK segment (scatter with -eps), roulette.
// Returns MK_ALIVE, MK_ESCAPED (splat ps.T) or MK_DIED (roulette).
CVR_DEV uint32_t mk_extend(const MediumParams& m, uint32_t iteration, uint32_t depth, PathState& ps,
                           uint32_t& n_steps, uint32_t& n_density, uint32_t& n_fetch, uint32_t& n_albedo) {
  rng_seeded(ps.rng, iteration, ps.image_id, depth);
  (void)rng_float(ps.rng);  // float3 e = rng.getFloat3(), unused (Q12)
  (void)rng_float(ps.rng);
  (void)rng_float(ps.rng);
  Isect is;
  is.dist = 0.0f;  // a fresh SimpleIsect per d_extend
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  if (!aabb_intersect(m, ps.o, ps.d, is)) return MK_ESCAPED;
  float t = 0.0f;
  bool collided = false;
  if (is.inside) {
    int s;
    do {
      s = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, n_steps, n_density, n_fetch);
    } while (s == 0);
    collided = t < is.dist;
  }
  if (!collided) {
    boundary_event(m, ps, is);
  } else {
    scatter_event<true>(m, ps, t);
    ++n_albedo;
  }
  return roulette(ps) ? MK_ALIVE : MK_DIED;
}

// Outcome of one naiveMK path (flags as PathRecord: bit0 contributed T,
// bit1 truncated, bit2 missed the box at init (T = 1), bit3 dropped by a
// failed GGX sample at init).
struct MkResult {
  uint32_t flags;
  V3 T;
  uint32_t n_segments, n_steps, n_density, n_fetch, n_albedo;
};

// NaiveVolPTmk_kernel::d_init + the d_extend bounce loop (NaiveVolPTmk_kernel.cuh:20-151,
// RenderKernelLauncher.cu:183-272) for path id = iteration * tile_px + pixel.
// Per path the multi-kernel wavefront reduces to this loop: every live path
// is extended once per launch, and compaction keeps every live path (quirk
// Q11 fixed; CVR_OPT_MK_COMPACTION 1 runs the reference's per-bounce launches,
// k_mk_extend).  Same operation order as the oracle's trace_path_mk.
CVR_DEV MkResult walk_mk(const MediumParams& m, const LaunchParams& L, uint32_t path_id) {
  MkResult r{0u, mk3(1.0f, 1.0f, 1.0f), 1u, 0u, 0u, 0u, 0u};
  const uint32_t image_id = path_id % L.tile_px, iteration = path_id / L.tile_px;
  PathState ps;
  const uint32_t s0 = mk_init(m, L, iteration, image_id, ps);
  if (s0 == MK_MISSED) {
    r.flags = 1u | 4u;
    return r;
  }
  if (s0 == MK_DROPPED) {
    r.flags = 8u;  // dropped: no contribution, T recorded as 0 (as the oracle)
    r.T = mk3(0.0f, 0.0f, 0.0f);
    return r;
  }
  for (uint32_t depth = 0;; ++depth) {
    if (L.max_segments && r.n_segments >= L.max_segments) {
      r.flags |= 2u;
      break;
    }
    ++r.n_segments;
    const uint32_t e = mk_extend(m, iteration, depth, ps, r.n_steps, r.n_density, r.n_fetch, r.n_albedo);
    if (e == MK_ESCAPED) r.flags |= 1u;
    if (e != MK_ALIVE) break;
  }
  r.T = ps.T;
  return r;
}

}  // namespace cvr
