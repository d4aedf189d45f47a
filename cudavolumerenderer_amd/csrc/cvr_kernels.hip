// cvr_kernels.hip - gfx950 schedulers for the volumetric random walk.
//
//   k_naive        NaiveVolPTsk_kernel::d_render (NaiveVolPTsk_kernel.cuh:17-87):
//                  one work-item per path, the whole walk in one loop.
//   k_persistent   RegenerationVolPTsk_kernel::d_render_single_thread_regeneration
//                  (RegenerationVolPTsk_kernel.cuh:146-232) re-designed for
//                  wave64: persistent waves; the unit of scheduling is ONE
//                  Woodcock step, not one path segment.  Lanes whose path needs
//                  an event (new path, AABB test, GGX boundary, scatter,
//                  roulette) wait masked until EV_THRESH lanes of the wave
//                  need one, then the wave runs the event code once for all
//                  of them.  New paths come from a wave-aggregated work queue
//                  (one atomic per CHUNK paths, ballot + mbcnt to hand ids to
//                  idle lanes).  The RNG is bound to path_id, so the result is
//                  independent of scheduling.
//   k_trace        debug: one work-item per path, writes a per-path record
//                  instead of splatting (bit-exact parity vs the oracle).
#include <hip/hip_runtime.h>

#include "cvr_kernels.h"
#include "cvr_walk.h"

#ifndef CVR_STAMPS
#define CVR_STAMPS 0
#endif

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
          r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY]);
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

// --------------------------------------------------------- persistent -----
enum : uint32_t { S_IDLE = 0, S_ISECT = 1, S_TRACK = 2, S_BOUNDARY = 3, S_COLLIDE = 4, S_DONE = 5 };

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <bool kScatterEps, int kWaves>
__global__ __launch_bounds__(256, kWaves) void k_persistent(MediumParams m, LaunchParams L) {
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0};
  PathState ps;
  Isect is;
  is.dist = 0.0f;
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  ps.image_id = 0;
  ps.o = ps.d = ps.T = mk3(0, 0, 0);
  uint32_t state = S_IDLE;
  float t = 0.0f;
  uint32_t nseg = 0;

  // wave-uniform work cursor [q_next, q_end) into queue q_cur's units; the
  // home queue is this XCD's band (HW_REG_XCC_ID, speed only: any wave may
  // take any unit, every unit is taken exactly once).
  uint32_t q_next = 0, q_end = 0, q_cur = 0;
  uint32_t q_home = (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u) % L.n_queues;
  bool exhausted = false;
  const uint32_t ev_thresh = L.ev_thresh;
#if CVR_STAMPS
  // diagnostic build only: cycles per phase (s_memtime), DESIGN.md §Profiling
  unsigned long long st_ev = 0, st_tr = 0, n_ev = 0, n_tr = 0, t_mark = __builtin_amdgcn_s_memtime();
#endif

  for (;;) {
    // ------------------------------------------------ event phase --------
#if CVR_STAMPS
    ++n_ev;
#endif
    for (;;) {
      // regenerate idle lanes from the wave's chunk of the queue
      unsigned long long idle = __ballot(state == S_IDLE);
      while (idle != 0ull && !exhausted) {
        if (q_next == q_end) {
          // dequeue a chunk: home band first (this XCD's), then steal
          uint32_t base = 0xFFFFFFFFu, qsel = 0;
          if ((threadIdx.x & 63) == 0) {
            for (uint32_t k = 0; k < L.n_queues; ++k) {
              const uint32_t q = (q_home + k) % L.n_queues;
              const uint32_t units = queue_units(L, q);
              const uint32_t b = atomicAdd(L.queue + 16 * q, L.chunk);
              if (b < units) {
                base = b;
                qsel = q;
                break;
              }
            }
          }
          base = __shfl(base, 0);
          qsel = __shfl(qsel, 0);
          if (base == 0xFFFFFFFFu) {
            exhausted = true;
            break;
          }
          q_cur = qsel;
          q_home = qsel;
          q_next = base;
          q_end = min(base + L.chunk, queue_units(L, qsel));
        }
        const uint32_t take = min((uint32_t)__popcll(idle), q_end - q_next);
        const uint32_t rank = lane_rank(idle);
        if (state == S_IDLE && rank < take) {
          path_begin(L, unit_to_path(L, q_cur, q_next + rank), ps);
          is.normal = mk3(0, 0, 0);
          nseg = 0;
          c[STAT_PATHS]++;
          state = S_ISECT;
        }
        q_next += take;
        idle = __ballot(state == S_IDLE);
      }
      if (exhausted && state == S_IDLE) state = S_DONE;

      if (state == S_ISECT) {
        if (L.max_segments && nseg >= L.max_segments) {
          c[STAT_TRUNCATED]++;
          c[STAT_SEGMENTS] += nseg;
          state = S_IDLE;
        } else {
          ++nseg;
          if (!aabb_intersect(m, ps.o, ps.d, is)) {
            splat(L, ps);
            c[STAT_ESCAPED]++;
            c[STAT_SEGMENTS] += nseg;
            state = S_IDLE;
          } else if (is.inside) {
            t = 0.0f;
            state = S_TRACK;
          } else {
            state = S_BOUNDARY;
          }
        }
      }
      if (state == S_BOUNDARY || state == S_COLLIDE) {
        if (state == S_BOUNDARY) {
          boundary_event(m, ps, is);
        } else {
          scatter_event<kScatterEps>(m, ps, t);
          c[STAT_ALBEDO]++;
        }
        if (roulette(ps)) {
          state = S_ISECT;
        } else {
          c[STAT_SEGMENTS] += nseg;
          state = S_IDLE;
        }
      }
      const bool pending = (state == S_ISECT) || (state == S_IDLE && !exhausted);
      if (!__any(pending)) break;
    }

    // ------------------------------------------------ track phase --------
#if CVR_STAMPS
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_ev += now - t_mark;
      t_mark = now;
    }
#endif
    if (!__any(state == S_TRACK)) {
      if (__all(state == S_DONE)) break;
      continue;
    }
    for (;;) {
#if CVR_STAMPS
      ++n_tr;
#endif
      if (state == S_TRACK) {
        const int r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY]);
        if (r == 1) state = S_BOUNDARY;
        else if (r == 2) state = (t < is.dist) ? S_COLLIDE : S_BOUNDARY;
      }
      const unsigned long long tracking = __ballot(state == S_TRACK);
      if (tracking == 0ull) break;
      const uint32_t waiting =
          (uint32_t)__popcll(__ballot(state == S_BOUNDARY || state == S_COLLIDE || (state == S_IDLE && !exhausted)));
      if (waiting >= ev_thresh) break;
    }
#if CVR_STAMPS
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      st_tr += now - t_mark;
      t_mark = now;
    }
#endif
  }
#if CVR_STAMPS
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(L.stats + 16, st_ev);
    atomicAdd(L.stats + 17, st_tr);
    atomicAdd(L.stats + 18, n_ev);
    atomicAdd(L.stats + 19, n_tr);
  }
#endif
  flush_stats(L, c);
}

// --------------------------------------------------------------- trace ----
template <bool kScatterEps>
__global__ __launch_bounds__(256) void k_trace(MediumParams m, LaunchParams L, PathRecord* rec) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= L.path_count) return;
  PathState ps;
  path_begin(L, L.path_first + tid, ps);
  Isect is;
  is.dist = 0.0f;
  is.normal = mk3(0, 0, 0);
  is.inside = false;
  PathRecord r = {};
  r.image_id = ps.image_id;
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
        s = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, r.n_steps, r.n_density);
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

// Persistent-kernel instantiations: scatter -eps on/off x register budget
// (launch-bounds waves per SIMD; 4 = no cap: ~125 VGPRs, no spills).
template <bool E>
static const void* persistent_fn(int waves) {
  switch (waves) {
    case 5: return reinterpret_cast<const void*>(&k_persistent<E, 5>);
    case 6: return reinterpret_cast<const void*>(&k_persistent<E, 6>);
    case 8: return reinterpret_cast<const void*>(&k_persistent<E, 8>);
    default: return reinterpret_cast<const void*>(&k_persistent<E, 4>);
  }
}

hipError_t launch_persistent(const MediumParams& m, const LaunchParams& L, bool scatter_eps, int waves,
                             uint32_t grid, hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  const void* fn = scatter_eps ? persistent_fn<true>(waves) : persistent_fn<false>(waves);
  MediumParams mm = m;
  LaunchParams ll = L;
  void* args[] = {&mm, &ll};
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s);
}

hipError_t persistent_occupancy(bool scatter_eps, int waves, int* blocks_per_cu) {
  const void* fn = scatter_eps ? persistent_fn<true>(waves) : persistent_fn<false>(waves);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 256, 0);
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

hipError_t launch_tile_to_image(const float4* tile, uint32_t tw, uint32_t th, float4* image, uint32_t iw,
                                uint32_t ox, uint32_t oy, float scale, hipStream_t s) {
  const uint32_t n = tw * th;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tile_to_image, dim3((n + 255u) / 256u), dim3(256), 0, s, tile, tw, th, image, iw, ox, oy,
                     scale);
  return hipGetLastError();
}

}  // namespace cvr

namespace cvr {
// ----------------------------------------------------------- cell table ---
// Corner-replicated density cells (see MediumParams::cells).
__global__ __launch_bounds__(256) void k_build_cells(const float* __restrict__ D, uint32_t rx, uint32_t ry,
                                                     uint32_t rz, float4* __restrict__ cells) {
  const size_t n = (size_t)rx * ry * rz;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint32_t x = (uint32_t)(i % rx), y = (uint32_t)((i / rx) % ry), z = (uint32_t)(i / ((size_t)rx * ry));
    const uint32_t xb = min(x + 1, rx - 1), yb = min(y + 1, ry - 1), zb = min(z + 1, rz - 1);
    auto at = [&](uint32_t a, uint32_t b, uint32_t c) { return D[((size_t)c * ry + b) * rx + a]; };
    cells[2 * i] = make_float4(at(x, y, z), at(xb, y, z), at(x, yb, z), at(xb, yb, z));
    cells[2 * i + 1] = make_float4(at(x, y, zb), at(xb, y, zb), at(x, yb, zb), at(xb, yb, zb));
  }
}

hipError_t launch_build_cells(const float* density, uint32_t rx, uint32_t ry, uint32_t rz, float4* cells,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_build_cells, dim3(4096), dim3(256), 0, s, density, rx, ry, rz, cells);
  return hipGetLastError();
}
}  // namespace cvr
