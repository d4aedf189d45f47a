// cvr_kernels.hip - reference-shaped kernels and helpers (gfx950).
//
//   k_naive        NaiveVolPTsk_kernel::d_render (NaiveVolPTsk_kernel.cuh:17-87):
//                  one work-item per path, the whole walk in one loop.
//   k_trace        debug: one work-item per path, writes a per-path record
//                  instead of splatting (bit-exact parity vs the oracle).
//   k_tile_to_image, k_build_cells: output transfer and the density cell table.
// The production regenerationSK scheduler is cvr_persistent.hip.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cvr_kernels.h"
#include "cvr_walk.h"

namespace cvr {

__device__ __forceinline__ void flush_stats(const LaunchParams& L, const uint32_t (&c)[STAT_COUNT]) {
#pragma unroll
  for (int k = 0; k < STAT_COUNT; ++k) {
    unsigned long long v = c[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(L.stats + k, v);
  }
}

// ------------------------------------------------------------- naiveSK ----
template <bool kScatterEps>
__global__ __launch_bounds__(256) void k_naive(MediumParams m, LaunchParams L) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0};
  if (tid < L.path_count) {
    PathState ps;
    path_begin(L, L.path_first + tid, ps);
    Isect is;
    is.dist = 0.0f;
    is.normal = mk3(0, 0, 0);
    is.inside = false;
    uint32_t nseg = 0;
    c[STAT_PATHS] = 1;
    for (;;) {
      if (L.max_segments && nseg >= L.max_segments) {
        c[STAT_TRUNCATED]++;
        break;
      }
      ++nseg;
      if (!aabb_intersect(m, ps.o, ps.d, is)) {
        splat(L, ps);
        c[STAT_ESCAPED]++;
        break;
      }
      float t = 0.0f;
      bool collided = false;
      if (is.inside) {
        int r;
        do {
          r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
        } while (r == 0);
        collided = t < is.dist;
      }
      if (!collided) {
        boundary_event(m, ps, is);
      } else {
        scatter_event<kScatterEps>(m, ps, t);
        c[STAT_ALBEDO]++;
      }
      if (!roulette(ps)) break;
    }
    c[STAT_SEGMENTS] = nseg;
  }
  flush_stats(L, c);
}

// ------------------------------------------------------------- naiveMK ----
// One work-item per (iteration, pixel) path; walk_mk restates the reference's
// init + extend kernels for one path (cvr_walk.h).
__global__ __launch_bounds__(256) void k_naive_mk(MediumParams m, LaunchParams L) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (tid < L.path_count) {
    const uint32_t pid = L.path_first + tid;
    const MkResult r = walk_mk(m, L, pid);
    c[STAT_PATHS] = 1;
    c[STAT_SEGMENTS] = r.n_segments;
    c[STAT_STEPS] = r.n_steps;
    c[STAT_DENSITY] = r.n_density;
    c[STAT_FETCH] = r.n_fetch;
    c[STAT_ALBEDO] = r.n_albedo;
    c[STAT_TRUNCATED] = (r.flags >> 1) & 1u;
    if (r.flags & 1u) {
      PathState ps;
      ps.image_id = pid % L.tile_px;
      ps.T = r.T;
      splat(L, ps);
      c[STAT_ESCAPED] = 1;
    }
  }
  flush_stats(L, c);
}

// ------------------------------------------ naiveMK, reference compaction --
// CVR_OPT_MK_COMPACTION 1 (quirk Q11 reproduced): the reference's per-bounce
// kernel sequence over the tile's pixels (NaiveVolPTmk::launchRender / extend,
// RenderKernelLauncher.cu:183-272).  Path state per pixel in `st` (o, d, T as
// three float4) with a live flag; after each bounce the host reads the number
// of live paths and the highest live pixel id (MkCtl), which the reference's
// stable remove_if leaves last in its active list and its count
// end - begin - 1 then drops.
__global__ __launch_bounds__(256) void k_mk_init(MediumParams m, LaunchParams L, uint32_t iteration,
                                                 float4* __restrict__ st, uint32_t* __restrict__ live) {
  const uint32_t img = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (img < L.tile_px) {
    PathState ps;
    const uint32_t r = mk_init(m, L, iteration, img, ps);
    c[STAT_PATHS] = 1;
    c[STAT_SEGMENTS] = 1;
    live[img] = r == MK_ALIVE ? 1u : 0u;
    if (r == MK_MISSED) {  // d_output[img_id] += (1,1,1,1); w = 1 as every contribution here
      splat(L, ps);
      c[STAT_ESCAPED] = 1;
    } else if (r == MK_ALIVE) {
      st[3 * (size_t)img] = make_float4(ps.o.x, ps.o.y, ps.o.z, 0.0f);
      st[3 * (size_t)img + 1] = make_float4(ps.d.x, ps.d.y, ps.d.z, 0.0f);
      st[3 * (size_t)img + 2] = make_float4(ps.T.x, ps.T.y, ps.T.z, 0.0f);
    }
  }
  flush_stats(L, c);
}

__global__ __launch_bounds__(256) void k_mk_extend(MediumParams m, LaunchParams L, uint32_t iteration, uint32_t depth,
                                                   float4* __restrict__ st, uint32_t* __restrict__ live,
                                                   MkCtl* __restrict__ ctl) {
  const uint32_t img = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool alive = false;
  if (img < L.tile_px && live[img]) {
    PathState ps;
    ps.image_id = img;
    const float4 a = st[3 * (size_t)img], b = st[3 * (size_t)img + 1], f = st[3 * (size_t)img + 2];
    ps.o = mk3(a.x, a.y, a.z);
    ps.d = mk3(b.x, b.y, b.z);
    ps.T = mk3(f.x, f.y, f.z);
    c[STAT_SEGMENTS] = 1;
    const uint32_t r =
        mk_extend(m, iteration, depth, ps, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH], c[STAT_ALBEDO]);
    if (r == MK_ESCAPED) {
      splat(L, ps);
      c[STAT_ESCAPED] = 1;
    }
    if (r == MK_ALIVE) {
      st[3 * (size_t)img] = make_float4(ps.o.x, ps.o.y, ps.o.z, 0.0f);
      st[3 * (size_t)img + 1] = make_float4(ps.d.x, ps.d.y, ps.d.z, 0.0f);
      st[3 * (size_t)img + 2] = make_float4(ps.T.x, ps.T.y, ps.T.z, 0.0f);
      alive = true;
    } else {
      live[img] = 0u;
    }
  }
  // wave-aggregated survivors: count and highest pixel id
  const unsigned long long mask = __ballot(alive);
  if (mask) {
    uint32_t mx = alive ? img : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
    if ((threadIdx.x & 63u) == 0u) {
      atomicAdd(&ctl->count, (uint32_t)__popcll(mask));
      atomicMax(&ctl->max_id, mx);
    }
  }
  flush_stats(L, c);
}

// --------------------------------------------------------------- trace ----
template <bool kScatterEps>
__global__ __launch_bounds__(256) void k_trace(MediumParams m, LaunchParams L, PathRecord* rec) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= L.path_count) return;
  if (L.naive_mk & 1u) {
    const MkResult mr = walk_mk(m, L, L.path_first + tid);
    PathRecord r = {};
    r.image_id = (L.path_first + tid) % L.tile_px;
    r.flags = mr.flags;
    r.T[0] = mr.T.x;
    r.T[1] = mr.T.y;
    r.T[2] = mr.T.z;
    r.n_segments = mr.n_segments;
    r.n_steps = mr.n_steps;
    r.n_density = mr.n_density;
    r.n_albedo = mr.n_albedo;
    rec[tid] = r;
    if (mr.n_fetch) atomicAdd(L.stats + STAT_FETCH, (unsigned long long)mr.n_fetch);
    return;
  }
  PathState ps;
  path_begin(L, L.path_first + tid, ps);
  Isect is;
  is.dist = 0.0f;
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  PathRecord r = {};
  r.image_id = ps.image_id;
  uint32_t n_fetch = 0;
  for (;;) {
    if (L.max_segments && r.n_segments >= L.max_segments) {
      r.flags |= 2u;
      break;
    }
    ++r.n_segments;
    if (!aabb_intersect(m, ps.o, ps.d, is)) {
      r.flags |= 1u;
      break;
    }
    float t = 0.0f;
    bool collided = false;
    if (is.inside) {
      int s;
      do {
        s = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, r.n_steps, r.n_density, n_fetch);
      } while (s == 0);
      collided = t < is.dist;
    }
    if (!collided) {
      boundary_event(m, ps, is);
    } else {
      scatter_event<kScatterEps>(m, ps, t);
      ++r.n_albedo;
    }
    if (!roulette(ps)) break;
  }
  r.T[0] = ps.T.x;
  r.T[1] = ps.T.y;
  r.T[2] = ps.T.z;
  rec[tid] = r;
  if (n_fetch) atomicAdd(L.stats + STAT_FETCH, (unsigned long long)n_fetch);
}

// ------------------------------------------- thread-bound regenerationSK ---
// RegenerationVolPTsk_kernel::d_render_single_thread_regeneration
// (RegenerationVolPTsk_kernel.cuh:146-232) with the reference's RNG binding
// (CVR_OPT_RNG_BINDING = 1): persistent thread tid draws every
// path it takes from one stream, Rng(seed + tid); one loop iteration takes a
// path if idle, runs one segment and the roulette, which also runs (one
// draw) after an escape (:220-229); the isect lives across the thread's paths
// (:155).  Idle lanes take consecutive path ids in lane order from one
// wave-aggregated atomic, so a one-wave launch is deterministic (the oracle's
// oracle_render_thread_bound); with more waves the path -> thread assignment
// depends on timing, as in the reference.  Lanes whose queue ran dry stay in
// the loop (idle) until the whole wave is done, so the wave's collectives
// always see lane 0.
template <bool kScatterEps>
__global__ __launch_bounds__(64) void k_regen_thread(MediumParams m, LaunchParams L) {
  const uint32_t lane = threadIdx.x;
  const uint32_t tid = blockIdx.x * 64u + lane;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  PathState ps;
  rng_init(ps.rng, (int32_t)(L.seed_base + tid));  // Rng(seed + tid): int, sign-extended (Q3)
  ps.o = ps.d = ps.T = mk3(0, 0, 0);
  ps.image_id = 0;
  Isect is;
  is.dist = 0.0f;
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  bool active = false, done = false;
  uint32_t nseg = 0;
  for (;;) {
    // ---- regenerate (:160-180)
    const unsigned long long need = __ballot(!active && !done);
    if (need) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(L.queue, (unsigned int)__popcll(need));
      base = __shfl(base, 0);
      if (!active && !done) {
        const uint32_t h =
            base + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        if (h >= L.path_count) {
          done = true;
        } else {
          const uint32_t path_id = L.path_first + h;
          ps.image_id = path_id - fastdiv(path_id, L.div_tile_px) * L.tile_px;
          camera_ray(L, ps);  // from the thread's stream
          nseg = 0;
          active = true;
          ++c[STAT_PATHS];
        }
      }
    }
    if (__ballot(!done) == 0ull) break;
    if (!active) continue;
    if (L.max_segments && nseg >= L.max_segments) {  // safety cap, as the path-bound walk
      ++c[STAT_TRUNCATED];
      active = false;
      continue;
    }
    ++nseg;
    ++c[STAT_SEGMENTS];
    if (!aabb_intersect(m, ps.o, ps.d, is)) {
      splat(L, ps);
      ++c[STAT_ESCAPED];
      active = false;
      (void)roulette(ps);  // the reference's roulette block draws after an escape too
      continue;
    }
    float t = 0.0f;
    bool collided = false;
    if (is.inside) {
      int r;
      do {
        r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
      } while (r == 0);
      collided = t < is.dist;
    }
    if (!collided) {
      boundary_event(m, ps, is);
    } else {
      scatter_event<kScatterEps>(m, ps, t);
      ++c[STAT_ALBEDO];
    }
    if (!roulette(ps)) active = false;
  }
  flush_stats(L, c);
}

// StreamingVolPTsk / SortingVolPTsk (StreamingVolPTsk_kernel.cuh:328-349,
// SortingVolPTsk_kernel.cuh:306-330) with the reference's thread-bound RNG
// (CVR_OPT_RNG_BINDING 1): blocks of 256 threads
// (STREAMING_THREADS_BLOCK, one item per thread), thread tid owning
// Rng(seed + tid) (:341) for whichever path it holds; every iteration the
// block regenerates the threads past n_active, extends every active path
// (streamingSK: one segment, or until the path ends once the head has passed
// n_paths; sortingSK: one segment with the collision's albedo deferred past
// the roulette while paths remain, else until the path ends) and compacts by a
// stable Morton sort of the ray origins (MortonSort.h:28-49): the paths move
// between threads, the RNG streams do not.  The oracle's
// oracle_render_stream_thread_bound restates one block in lockstep:
// regeneration reads the head once and hands out ids in thread order (one
// atomic per block here), so a one-block launch is deterministic; with more
// blocks the assignment depends on timing, as in the reference.
constexpr uint32_t kStreamThreads = 256;
__device__ __forceinline__ uint32_t lane_rank64(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint32_t expand_bits10(uint32_t v) {  // Utilities.h:35-41
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}
__device__ __forceinline__ uint32_t morton3d_ref(float x, float y, float z) {  // Utilities.h:45-55
  x = det_fminf(det_fmaxf(x * 1024.0f, 0.0f), 1023.0f);
  y = det_fminf(det_fmaxf(y * 1024.0f, 0.0f), 1023.0f);
  z = det_fminf(det_fmaxf(z * 1024.0f, 0.0f), 1023.0f);
  return expand_bits10((uint32_t)x) * 4u + expand_bits10((uint32_t)y) * 2u + expand_bits10((uint32_t)z);
}
template <bool kSorting>
__global__ __launch_bounds__(256) void k_stream_thread(MediumParams m, LaunchParams L) {
  __shared__ unsigned long long s_key[kStreamThreads];
  __shared__ float s_f[9][kStreamThreads];  // o, d, T of the threads' paths (the swap)
  __shared__ uint32_t s_u[3][kStreamThreads];  // image_id, nseg, texture_access
  __shared__ uint32_t s_wave[4], s_base, s_head;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  PathState ps;
  rng_init(ps.rng, (int32_t)(L.seed_base + blockIdx.x * kStreamThreads + tid));  // Rng(c_seed + gtid), Q3
  ps.o = ps.d = ps.T = mk3(0, 0, 0);
  ps.image_id = 0;
  uint32_t nseg = 0, n_active = 0;
  const V3 ext = sub3(m.bmax, m.bmin);
  for (;;) {
    // ---- regenerate (StreamingVolPTsk_kernel.cuh:66-105): the head read once for the block
    const bool req = tid >= n_active;
    const unsigned long long rq = __ballot(req);
    if (lane == 0) s_wave[wave] = (uint32_t)__popcll(rq);
    __syncthreads();
    uint32_t before = 0, n_req = 0;
    for (uint32_t w = 0; w < 4u; ++w) {
      before += w < wave ? s_wave[w] : 0u;
      n_req += s_wave[w];
    }
    if (tid == 0) {
      const uint32_t h = __hip_atomic_load(L.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_base = h < L.path_count ? atomicAdd(L.queue, n_req) : 0xFFFFFFFFu;
      s_head = __hip_atomic_load(L.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint32_t base = s_base;
    bool active = true;
    if (req) {
      const uint32_t h = base + before + lane_rank64(rq);
      if (base == 0xFFFFFFFFu || h >= L.path_count) {
        active = false;
      } else {
        const uint32_t path_id = L.path_first + h;
        ps.image_id = path_id - fastdiv(path_id, L.div_tile_px) * L.tile_px;
        camera_ray(L, ps);  // from the thread's stream
        nseg = 0;
        ++c[STAT_PATHS];
      }
    }
    // ---- extend
    const bool should_regenerate = s_head <= L.path_count;  // sortingSK, once per extend (:193)
    bool texacc = false;
    if (active) {
      do {
        if (L.max_segments && nseg >= L.max_segments) {  // safety cap, as the path-bound walk
          ++c[STAT_TRUNCATED];
          active = false;
          break;
        }
        ++nseg;
        ++c[STAT_SEGMENTS];
        Isect is;  // a fresh SimpleIsect per segment
        is.dist = 0.0f;
        is.normal = mk3(0, 0, 0);
        is.inside = false;
        if (!aabb_intersect(m, ps.o, ps.d, is)) {
          splat(L, ps);
          ++c[STAT_ESCAPED];
          active = false;
        } else {
          float t = 0.0f;
          bool collided = false;
          if (is.inside) {
            int r;
            do {
              r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
            } while (r == 0);
            collided = t < is.dist;
          }
          if (!collided) {
            boundary_event(m, ps, is);
          } else {
            ps.o = sub3(add3(ps.o, scl3(ps.d, t)), scl3(ps.d, CVR_EPSILON_F));
            ++c[STAT_ALBEDO];
            if (kSorting && should_regenerate) {
              texacc = true;  // delayed texture access (SortingVolPTsk_kernel.cuh:230-237)
            } else {
              ps.T = mul3(ps.T, albedo_lookup(m, div3(sub3(ps.o, m.bmin), ext)));
            }
            const float e1 = rng_float(ps.rng);
            const float e2 = rng_float(ps.rng);
            ps.d = hg_sample(ps.d, m.g, e1, e2);
          }
        }
        // roulette after every segment, an escape included, T / p either way
        const float p = det_fminf(1.0f, det_fmaxf(det_fmaxf(ps.T.x, ps.T.y), ps.T.z));
        if (rng_float(ps.rng) > p) active = false;
        ps.T = mk3(ps.T.x / p, ps.T.y / p, ps.T.z / p);
      } while ((kSorting ? !should_regenerate
                         : __hip_atomic_load(L.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > L.path_count) &&
               active);
    }
    // ---- compaction: stable Morton sort of the origins (inactive: morton3D(1,1,1) = 2^30 - 1)
    uint32_t code = 0x3FFFFFFFu;
    if (active) {
      const V3 q = div3(sub3(ps.o, m.bmin), ext);  // AABB::transform
      code = morton3d_ref(q.x, q.y, q.z);
    }
    s_key[tid] = ((unsigned long long)code << 10) | tid;
    const unsigned long long am = __ballot(active);
    __syncthreads();
    if (lane == 0) s_wave[wave] = (uint32_t)__popcll(am);
    for (uint32_t k = 2; k <= kStreamThreads; k <<= 1) {  // bitonic sort of 256 unique keys
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        const uint32_t ix = tid ^ j;
        if (ix > tid) {
          const unsigned long long a = s_key[tid], b = s_key[ix];
          if (((tid & k) == 0) == (a > b)) {
            s_key[tid] = b;
            s_key[ix] = a;
          }
        }
        __syncthreads();
      }
    }
    n_active = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    // swap (SortingVolPTsk_kernel.cuh:105-146): the path of thread key[tid] & 1023 moves here
    s_f[0][tid] = ps.o.x;
    s_f[1][tid] = ps.o.y;
    s_f[2][tid] = ps.o.z;
    s_f[3][tid] = ps.d.x;
    s_f[4][tid] = ps.d.y;
    s_f[5][tid] = ps.d.z;
    s_f[6][tid] = ps.T.x;
    s_f[7][tid] = ps.T.y;
    s_f[8][tid] = ps.T.z;
    s_u[0][tid] = ps.image_id;
    s_u[1][tid] = nseg;
    s_u[2][tid] = texacc ? 1u : 0u;
    __syncthreads();
    const uint32_t src = (uint32_t)(s_key[tid] & 1023u);
    ps.o = mk3(s_f[0][src], s_f[1][src], s_f[2][src]);
    ps.d = mk3(s_f[3][src], s_f[4][src], s_f[5][src]);
    ps.T = mk3(s_f[6][src], s_f[7][src], s_f[8][src]);
    ps.image_id = s_u[0][src];
    nseg = s_u[1][src];
    if (kSorting && s_u[2][src]) ps.T = mul3(ps.T, albedo_lookup(m, div3(sub3(ps.o, m.bmin), ext)));
    if (tid == 0) s_head = __hip_atomic_load(L.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (n_active == 0u && s_head >= L.path_count) break;  // block-uniform (:349)
  }
  flush_stats(L, c);
}

// ------------------------------------------- thread-bound streamingMK -----
// StreamingVolPTmk_kernel::d_regenerate / d_extend (StreamingVolPTmk_kernel.cuh
// :26-69, :74-253) with the reference's RNG binding (CVR_OPT_RNG_BINDING
// 1), one kernel each per iteration of the host loop (smk_thread_render,
// RenderKernelLauncher.cu:435-470).  Slot j = thread j (ITEMS_PER_THREAD 1);
// a slot's path lives in SmkSlots (o | image_id, d | nseg, T), its RNG state in
// the thread's `state` entry, which stays with the thread when compaction moves
// the path.  ctl[0] = n_active (d_n_active), ctl[1] = the path head.
// Thread order inside a block (the head and the compaction offset taken once
// per block): the lockstep order of oracle_render_smk_thread_bound.
__device__ __forceinline__ void block_rank256(bool flag, uint32_t* s_wave, uint32_t& before, uint32_t& total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned long long mk = __ballot(flag);
  if (lane == 0) s_wave[wave] = (uint32_t)__popcll(mk);
  __syncthreads();
  before = lane_rank64(mk);
  total = 0;
  for (uint32_t w = 0; w < 4u; ++w) {
    before += w < wave ? s_wave[w] : 0u;
    total += s_wave[w];
  }
}

__global__ __launch_bounds__(256) void k_smk_regen(LaunchParams L, SmkSlots out, uint4* __restrict__ st0,
                                                   uint2* __restrict__ st1, uint32_t* __restrict__ ctl) {
  __shared__ uint32_t s_wave[4], s_base;
  const uint32_t tid = threadIdx.x, j = blockIdx.x * kStreamThreads + tid;
  const uint32_t n_active = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool req = j >= n_active;
  uint32_t before, n_req;
  block_rank256(req, s_wave, before, n_req);
  if (tid == 0) {
    const uint32_t h = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_base = h < L.path_count ? atomicAdd(ctl + 1, n_req) : 0xFFFFFFFFu;
  }
  __syncthreads();
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (req) {  // no early return: flush_stats reduces over the whole wave
    const uint32_t base = s_base, h = base + before;
    if (base == 0xFFFFFFFFu || h >= L.path_count) {
      out.act[j] = 0;
    } else {
      PathState ps;
      path_begin(L, L.path_first + h, ps);  // Rng(c_seed + path_id) and the camera ray (:55-59)
      out.a[j] = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.image_id));
      out.b[j] = make_float4(ps.d.x, ps.d.y, ps.d.z, __uint_as_float(0u));
      out.t[j] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
      out.act[j] = 1;
      st0[j] = make_uint4(ps.rng.v0, ps.rng.v1, ps.rng.v2, ps.rng.v3);  // states[tid] = rng.getState() (:66)
      st1[j] = make_uint2(ps.rng.v4, ps.rng.d);
      c[STAT_PATHS] = 1;
    }
  }
  flush_stats(L, c);
}

__global__ __launch_bounds__(256) void k_smk_extend(MediumParams m, LaunchParams L, SmkSlots in, SmkSlots out,
                                                    uint4* __restrict__ st0, uint2* __restrict__ st1,
                                                    uint32_t* __restrict__ ctl) {
  __shared__ uint32_t s_wave[4], s_start;
  const uint32_t tid = threadIdx.x, j = blockIdx.x * kStreamThreads + tid;
  const uint32_t head = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint4 r0 = st0[j];
  const uint2 r1 = st1[j];
  PathState ps;
  ps.rng = Rng{r0.x, r0.y, r0.z, r0.w, r1.x, r1.y};  // the thread's state, whatever path slot j holds
  bool active = in.act[j] != 0;
  uint32_t nseg = 0;
  ps.o = ps.d = ps.T = mk3(0, 0, 0);
  ps.image_id = 0;
  if (active) {
    const float4 a = in.a[j], b = in.b[j], t = in.t[j];
    ps.o = mk3(a.x, a.y, a.z);
    ps.image_id = __float_as_uint(a.w);
    ps.d = mk3(b.x, b.y, b.z);
    nseg = __float_as_uint(b.w);
    ps.T = mk3(t.x, t.y, t.z);
  }
  const V3 ext = sub3(m.bmax, m.bmin);
  if (active) {
    do {
      if (L.max_segments && nseg >= L.max_segments) {  // safety cap, as the path-bound walk
        ++c[STAT_TRUNCATED];
        active = false;
        break;
      }
      ++nseg;
      ++c[STAT_SEGMENTS];
      Isect is;  // a fresh isect per segment (:163)
      is.dist = 0.0f;
      is.normal = mk3(0, 0, 0);
      is.inside = false;
      if (!aabb_intersect(m, ps.o, ps.d, is)) {
        splat(L, ps);
        ++c[STAT_ESCAPED];
        active = false;
      } else {
        float t = 0.0f;
        bool collided = false;
        if (is.inside) {
          int r;
          do {
            r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
          } while (r == 0);
          collided = t < is.dist;
        }
        if (!collided) {
          boundary_event(m, ps, is);
        } else {
          ps.o = sub3(add3(ps.o, scl3(ps.d, t)), scl3(ps.d, CVR_EPSILON_F));  // - d eps (:194)
          ++c[STAT_ALBEDO];
          ps.T = mul3(ps.T, albedo_lookup(m, div3(sub3(ps.o, m.bmin), ext)));
          const float e1 = rng_float(ps.rng);
          const float e2 = rng_float(ps.rng);
          ps.d = hg_sample(ps.d, m.g, e1, e2);
        }
      }
      // roulette after every segment, an escape included, T / p either way (:203-210)
      const float p = det_fminf(1.0f, det_fmaxf(det_fmaxf(ps.T.x, ps.T.y), ps.T.z));
      if (rng_float(ps.rng) > p) active = false;
      ps.T = mk3(ps.T.x / p, ps.T.y / p, ps.T.z / p);
    } while (head >= L.path_count && active);  // :212-214
  }
  // compaction (:218-252): the block's active paths in thread order at an offset taken once
  uint32_t before, total;
  block_rank256(active, s_wave, before, total);
  if (tid == 0) s_start = atomicAdd(ctl, total);
  __syncthreads();
  st0[j] = make_uint4(ps.rng.v0, ps.rng.v1, ps.rng.v2, ps.rng.v3);  // the state stays with the thread (:241)
  st1[j] = make_uint2(ps.rng.v4, ps.rng.d);
  if (active) {
    const uint32_t k = s_start + before;
    out.a[k] = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.image_id));
    out.b[k] = make_float4(ps.d.x, ps.d.y, ps.d.z, __uint_as_float(nseg));
    out.t[k] = make_float4(ps.T.x, ps.T.y, ps.T.z, 0.0f);
    out.act[k] = 1;
  }
  flush_stats(L, c);
}

// ----------------------------------------------------- image transfer -----
// Intended semantics of HostImageBufferTansferDelegate::transfer
// (ImageBufferTransfer.cu:61-78, fixed per SURVEY Q10): image[off + p] =
// tile[p] / scale, with UtilityFunctors::Scale (Utilities.h:6-15) = x/scale.
__global__ __launch_bounds__(256) void k_tile_to_image(const float4* __restrict__ tile, uint32_t tw, uint32_t th,
                                                       float4* __restrict__ image, uint32_t iw, uint32_t ox,
                                                       uint32_t oy, float scale) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tw * th) return;
  const uint32_t x = i % tw, y = i / tw;
  const float4 v = tile[i];
  image[(size_t)(y + oy) * iw + (x + ox)] = make_float4(v.x / scale, v.y / scale, v.z / scale, v.w / scale);
}

// Normalise + store into pinned host memory in one kernel (the transfer
// delegate's Scale functor and its D->H copy, ImageBufferTransfer.cu:61-78,
// UtilityFunctors::Scale x/scale, Utilities.h:6-15): the GPU writes the host
// buffer directly, so the copy is an ordinary kernel in stream order (no copy
// engine, which here blocked the host on cross-stream dependencies).
__global__ __launch_bounds__(256) void k_image_to_host(const float4* __restrict__ src, float4* __restrict__ dst,
                                                       size_t n4, float scale) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = src[i];
    __builtin_nontemporal_store(v.x / scale, &dst[i].x);
    __builtin_nontemporal_store(v.y / scale, &dst[i].y);
    __builtin_nontemporal_store(v.z / scale, &dst[i].z);
    __builtin_nontemporal_store(v.w / scale, &dst[i].w);
  }
}
// unaligned buffers and the ragged tail, one float per work-item
__global__ __launch_bounds__(256) void k_image_to_host_scalar(const float* __restrict__ src, float* __restrict__ dst,
                                                             size_t first, size_t n, float scale) {
  for (size_t i = first + (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = src[i] / scale;
}

hipError_t launch_image_to_host(const float* src, float* dst, size_t n, float scale, hipStream_t s) {
  const bool aligned = (((uintptr_t)src | (uintptr_t)dst) & 15u) == 0;
  const size_t n4 = aligned ? n / 4 : 0;
  if (n4) {
    const size_t blocks = std::min<size_t>((n4 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_image_to_host, dim3((uint32_t)blocks), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                       reinterpret_cast<float4*>(dst), n4, scale);
  }
  if (n4 * 4 < n) {
    const size_t blocks = std::min<size_t>((n - n4 * 4 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_image_to_host_scalar, dim3((uint32_t)blocks), dim3(256), 0, s, src, dst, n4 * 4, n, scale);
  }
  return hipGetLastError();
}

// The pixels of one block shard (cvr_set_block_shard(rank, world): 8x8 blocks
// rank, rank + world, ..., row-major) normalised into the host image, at their
// places in the full image: a multi-GPU render's whole output step, since the
// ranks' block shards are pixel-disjoint (no reduction).  Four blocks per
// workgroup, one pixel per work-item; eight work-items store one 128-byte row.
__global__ __launch_bounds__(256) void k_blocks_to_host(const float4* __restrict__ src, float4* __restrict__ dst,
                                                        uint32_t w, uint32_t blocks_x, uint32_t n_mine, uint32_t rank,
                                                        uint32_t world, float scale) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6); k < n_mine; k += gridDim.x * 4u) {
    const uint32_t b = rank + k * world;
    const uint32_t by = b / blocks_x, bx = b - by * blocks_x;
    const size_t i = (size_t)(by * 8u + (lane >> 3)) * w + bx * 8u + (lane & 7u);
    const float4 v = src[i];
    __builtin_nontemporal_store(v.x / scale, &dst[i].x);
    __builtin_nontemporal_store(v.y / scale, &dst[i].y);
    __builtin_nontemporal_store(v.z / scale, &dst[i].z);
    __builtin_nontemporal_store(v.w / scale, &dst[i].w);
  }
}

hipError_t launch_blocks_to_host(const float* src, float* dst, uint32_t w, uint32_t h, uint32_t rank, uint32_t world,
                                 float scale, hipStream_t s) {
  const uint32_t blocks_x = w / 8u, n_blocks = blocks_x * (h / 8u);
  const uint32_t n_mine = n_blocks > rank ? (n_blocks - rank + world - 1u) / world : 0u;
  if (n_mine == 0u) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>((n_mine + 3u) / 4u, 1024u);
  hipLaunchKernelGGL(k_blocks_to_host, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                     reinterpret_cast<float4*>(dst), w, blocks_x, n_mine, rank, world, scale);
  return hipGetLastError();
}

// ----------------------------------------------------------- cell table ---
// Corner-replicated density cells (see MediumParams::cells).
__global__ __launch_bounds__(256) void k_build_cells(const float* __restrict__ D, uint32_t rx, uint32_t ry,
                                                     uint32_t rz, float4* __restrict__ cells) {
  const size_t n = (size_t)rx * ry * rz;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint32_t x = (uint32_t)(i % rx), y = (uint32_t)((i / rx) % ry), z = (uint32_t)(i / ((size_t)rx * ry));
    const uint32_t xb = min(x + 1, rx - 1), yb = min(y + 1, ry - 1), zb = min(z + 1, rz - 1);
    auto at = [&](uint32_t a, uint32_t b, uint32_t c) { return D[((size_t)c * ry + b) * rx + a]; };
    // trilerp_cell layout: (d000, d100, d001, d101), (d010, d110, d011, d111), d{z}{y}{x}
    cells[2 * i] = make_float4(at(x, y, z), at(x, y, zb), at(xb, y, z), at(xb, y, zb));
    cells[2 * i + 1] = make_float4(at(x, yb, z), at(x, yb, zb), at(xb, yb, z), at(xb, yb, zb));
  }
}

// --------------------------------------------------------- brick bounds ---
// MediumParams::bounds.  One work-item per brick: the max over the voxels
// its cells interpolate (cells [b*B, b*B+B-1] use voxels up to b*B+B, clamped
// as texel() clamps), quantised upwards to q/254 of max_density.
// Brick-bound code (MediumParams::bounds, bound_value) of a brick whose
// largest density is mx: the smallest c with bound_value(c) >= (mx /
// max_density) (1 + 2^-16).  The test value fl(fl(scale rho) inv_sigma) of a
// point whose 8 corners are <= mx is <= mx / max_density (1 + 14 u), u = 2^-24
// (three fma lerps of values <= mx, then two rounded products), so the code
// bounds every test value of the brick.  255 (no bound): NaN / inf densities,
// or mx above the majorant (Q15: XML densities may exceed it).
__device__ uint32_t bound_code(float mx, float max_density, bool nan) {
  const double r = (double)mx / (double)max_density;
  if (nan || !(r <= 1.0)) return 255u;
  const double target = r * (1.0 + 1.0 / 65536.0);
  uint32_t c = 0;
  while (c < 255u && (double)bound_value(c) < target) ++c;
  return c;
}

__global__ __launch_bounds__(256) void k_build_bounds(const float* __restrict__ D, uint32_t rx, uint32_t ry,
                                                      uint32_t rz, uint32_t bshift, uint32_t bnx, uint32_t bny,
                                                      uint32_t bnz, float max_density, uint8_t* __restrict__ q) {
  const size_t nb = (size_t)bnx * bny * bnz;
  const uint32_t B = 1u << bshift;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (size_t)gridDim.x * 256) {
    const uint32_t bx = (uint32_t)(i % bnx), by = (uint32_t)((i / bnx) % bny), bz = (uint32_t)(i / ((size_t)bnx * bny));
    const uint32_t x0 = bx * B, y0 = by * B, z0 = bz * B;
    const uint32_t x1 = min(x0 + B, rx - 1), y1 = min(y0 + B, ry - 1), z1 = min(z0 + B, rz - 1);
    float mx = 0.0f;
    bool nan = false;
    for (uint32_t z = z0; z <= z1; ++z)
      for (uint32_t y = y0; y <= y1; ++y)
        for (uint32_t x = x0; x <= x1; ++x) {
          const float v = D[((size_t)z * ry + y) * rx + x];
          nan |= !(v == v) || v == __builtin_inff();
          mx = fmaxf(mx, v);
        }
    q[i] = (uint8_t)bound_code(mx, max_density, nan);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) q[nb] = 255u;  // MediumParams::bsentinel: no bound
}

// ------------------------------------------------------ sparse medium -----
// Cell-leaf pool (MediumParams::cells for a sparse medium): slot s holds the
// corner-replicated cells of leaf coords[s] (x, y, z leaf coordinates; slot 0
// is the all-zero leaf).  Cells past the grid edge are never fetched (the
// Woodcock range test) and are written as zeros.
__global__ __launch_bounds__(256) void k_build_sparse_cells(MediumParams m, const uint32_t* __restrict__ coords,
                                                            size_t n_cells, float4* __restrict__ cells) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n_cells; i += (size_t)gridDim.x * 256) {
    const size_t slot = i >> 9;
    const uint32_t local = (uint32_t)(i & 511u);
    const uint32_t x = coords[3 * slot] * 8u + (local & 7u), y = coords[3 * slot + 1] * 8u + ((local >> 3) & 7u),
                   z = coords[3 * slot + 2] * 8u + (local >> 6);
    if (slot == 0 || x >= m.rx || y >= m.ry || z >= m.rz) {
      cells[2 * i] = make_float4(0.f, 0.f, 0.f, 0.f);
      cells[2 * i + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    const uint32_t xb = min(x + 1, m.rx - 1), yb = min(y + 1, m.ry - 1), zb = min(z + 1, m.rz - 1);
    cells[2 * i] = make_float4(texel_density(m, x, y, z), texel_density(m, x, y, zb), texel_density(m, xb, y, z),
                               texel_density(m, xb, y, zb));
    cells[2 * i + 1] = make_float4(texel_density(m, x, yb, z), texel_density(m, x, yb, zb),
                                   texel_density(m, xb, yb, z), texel_density(m, xb, yb, zb));
  }
}

// Sparse brick words: q << 24 | cell-leaf slot of the brick's leaf (bricks of
// 2^bshift <= 8 cells never straddle leaves).  q as k_build_bounds; 0 for a
// brick whose leaf has no cell slot (all its corners are 0), 255 everywhere
// when `unbounded` (bounds off or no finite majorant: every point fetches).
__global__ __launch_bounds__(256) void k_build_sparse_bounds(MediumParams m, const uint32_t* __restrict__ cell_slot,
                                                             uint32_t bnz, float max_density, int unbounded,
                                                             uint32_t* __restrict__ sb) {
  const size_t nb = (size_t)m.bnx * m.bny * bnz;
  const uint32_t B = 1u << m.bshift, up = 3u - m.bshift;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (size_t)gridDim.x * 256) {
    const uint32_t bx = (uint32_t)(i % m.bnx), by = (uint32_t)((i / m.bnx) % m.bny),
                   bz = (uint32_t)(i / ((size_t)m.bnx * m.bny));
    const uint32_t slot = cell_slot[((size_t)(bz >> up) * m.lny + (by >> up)) * m.lnx + (bx >> up)];
    uint32_t v = 0u;
    if (unbounded) {
      v = 255u;
    } else if (slot != 0u) {
      const uint32_t x0 = bx * B, y0 = by * B, z0 = bz * B;
      const uint32_t x1 = min(x0 + B, m.rx - 1), y1 = min(y0 + B, m.ry - 1), z1 = min(z0 + B, m.rz - 1);
      float mx = 0.0f;
      bool nan = false;
      for (uint32_t z = z0; z <= z1; ++z)
        for (uint32_t y = y0; y <= y1; ++y)
          for (uint32_t x = x0; x <= x1; ++x) {
            const float d = texel_density(m, x, y, z);
            nan |= !(d == d) || d == __builtin_inff();
            mx = fmaxf(mx, d);
          }
      v = bound_code(mx, max_density, nan);
    }
    sb[i] = (v << 24) | slot;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) sb[nb] = 255u << 24;  // MediumParams::bsentinel: no bound, slot 0
}

// ---------------------------------------------------------- launchers -----
hipError_t launch_naive(const MediumParams& m, const LaunchParams& L, bool scatter_eps, hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  const uint32_t grid = (L.path_count + 255u) / 256u;
  if (scatter_eps)
    hipLaunchKernelGGL(k_naive<true>, dim3(grid), dim3(256), 0, s, m, L);
  else
    hipLaunchKernelGGL(k_naive<false>, dim3(grid), dim3(256), 0, s, m, L);
  return hipGetLastError();
}

hipError_t launch_naive_mk(const MediumParams& m, const LaunchParams& L, hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_naive_mk, dim3((L.path_count + 255u) / 256u), dim3(256), 0, s, m, L);
  return hipGetLastError();
}

hipError_t launch_mk_init(const MediumParams& m, const LaunchParams& L, uint32_t iteration, float4* st,
                          uint32_t* live, hipStream_t s) {
  hipLaunchKernelGGL(k_mk_init, dim3((L.tile_px + 255u) / 256u), dim3(256), 0, s, m, L, iteration, st, live);
  return hipGetLastError();
}

hipError_t launch_mk_extend(const MediumParams& m, const LaunchParams& L, uint32_t iteration, uint32_t depth,
                            float4* st, uint32_t* live, MkCtl* ctl, hipStream_t s) {
  hipLaunchKernelGGL(k_mk_extend, dim3((L.tile_px + 255u) / 256u), dim3(256), 0, s, m, L, iteration, depth, st, live,
                     ctl);
  return hipGetLastError();
}

hipError_t launch_trace(const MediumParams& m, const LaunchParams& L, bool scatter_eps, PathRecord* rec,
                        hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  const uint32_t grid = (L.path_count + 255u) / 256u;
  if (scatter_eps)
    hipLaunchKernelGGL(k_trace<true>, dim3(grid), dim3(256), 0, s, m, L, rec);
  else
    hipLaunchKernelGGL(k_trace<false>, dim3(grid), dim3(256), 0, s, m, L, rec);
  return hipGetLastError();
}

hipError_t launch_stream_thread(const MediumParams& m, const LaunchParams& L, bool sorting, uint32_t grid,
                                hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  if (sorting)
    hipLaunchKernelGGL(k_stream_thread<true>, dim3(grid), dim3(kStreamThreads), 0, s, m, L);
  else
    hipLaunchKernelGGL(k_stream_thread<false>, dim3(grid), dim3(kStreamThreads), 0, s, m, L);
  return hipGetLastError();
}

hipError_t launch_smk_regen(const LaunchParams& L, const SmkSlots& out, uint4* st0, uint2* st1, uint32_t* ctl,
                            uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(k_smk_regen, dim3(grid), dim3(kStreamThreads), 0, s, L, out, st0, st1, ctl);
  return hipGetLastError();
}

hipError_t launch_smk_extend(const MediumParams& m, const LaunchParams& L, const SmkSlots& in, const SmkSlots& out,
                             uint4* st0, uint2* st1, uint32_t* ctl, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(k_smk_extend, dim3(grid), dim3(kStreamThreads), 0, s, m, L, in, out, st0, st1, ctl);
  return hipGetLastError();
}

hipError_t launch_regen_thread(const MediumParams& m, const LaunchParams& L, bool scatter_eps, uint32_t grid,
                               hipStream_t s) {
  if (L.path_count == 0 || grid == 0) return hipSuccess;
  if (scatter_eps)
    hipLaunchKernelGGL(k_regen_thread<true>, dim3(grid), dim3(64), 0, s, m, L);
  else
    hipLaunchKernelGGL(k_regen_thread<false>, dim3(grid), dim3(64), 0, s, m, L);
  return hipGetLastError();
}

hipError_t launch_tile_to_image(const float4* tile, uint32_t tw, uint32_t th, float4* image, uint32_t iw,
                                uint32_t ox, uint32_t oy, float scale, hipStream_t s) {
  const uint32_t n = tw * th;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tile_to_image, dim3((n + 255u) / 256u), dim3(256), 0, s, tile, tw, th, image, iw, ox, oy,
                     scale);
  return hipGetLastError();
}

hipError_t launch_build_bounds(const float* density, uint32_t rx, uint32_t ry, uint32_t rz, uint32_t bshift,
                               float max_density, uint8_t* bounds, hipStream_t s) {
  const uint32_t B = 1u << bshift;
  const uint32_t bnx = (rx + B - 1) / B, bny = (ry + B - 1) / B, bnz = (rz + B - 1) / B;
  hipLaunchKernelGGL(k_build_bounds, dim3(1024), dim3(256), 0, s, density, rx, ry, rz, bshift, bnx, bny, bnz,
                     max_density, bounds);
  return hipGetLastError();
}

hipError_t launch_build_cells(const float* density, uint32_t rx, uint32_t ry, uint32_t rz, float4* cells,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_build_cells, dim3(4096), dim3(256), 0, s, density, rx, ry, rz, cells);
  return hipGetLastError();
}

hipError_t launch_build_sparse(const MediumParams& m, const uint32_t* coords, size_t n_cell_leaves,
                               const uint32_t* cell_slot, uint32_t bnz, float max_density, int unbounded,
                               float4* cells, uint32_t* sbounds, hipStream_t s) {
  hipLaunchKernelGGL(k_build_sparse_cells, dim3(8192), dim3(256), 0, s, m, coords, n_cell_leaves * 512, cells);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_build_sparse_bounds, dim3(4096), dim3(256), 0, s, m, cell_slot, bnz, max_density, unbounded,
                     sbounds);
  return hipGetLastError();
}

}  // namespace cvr
