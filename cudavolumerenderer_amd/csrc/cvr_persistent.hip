// cvr_persistent.hip - the regenerationSK scheduler for gfx950.
//
// Semantics: RegenerationVolPTsk_kernel::d_render_single_thread_regeneration
// (RegenerationVolPTsk_kernel.cuh:146-232): persistent work-items, each takes
// a new path from a global counter when its path ends; the scatter point has
// no -eps (:212).  The RNG is bound to the path id, so the image
// does not depend on how paths are scheduled.
//
// Design (wave64):
//  * The unit of scheduling is one Woodcock step.  A lane whose path needs an
//    event (new path, AABB test, GGX boundary, scatter, roulette) waits masked
//    until `ev_thresh` lanes of the wave wait, then the wave runs the event
//    code once for all of them (the event code is ~10x the step code).
//  * New paths come in chunks of `chunk` work units per wave (one atomic per
//    chunk, ballot + mbcnt hand-out).  Work units are ordered pixel-major
//    (8x8-pixel blocks, samples innermost) and the block range is split into
//    one band per XCD, so a wave's lanes trace neighbouring rays and an XCD's
//    in-flight rays stay in one band of the volume (L2 locality).
//  * Density comes from the corner-replicated cell table (one 32-byte cell
//    fetch per Woodcock step, MediumParams::cells).
// Tried and measured slower on C2 (DESIGN.md §Performance log): a
// software-pipelined Woodcock loop with two cell fetches in flight per lane
// (spills at 4 waves/SIMD), wave-uniform ballot counters (more VGPRs), and
// 5/6/8 waves per SIMD (spills).
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
        const int r = woodcock_step(m, ps.o, ps.d, is.dist, t, ps.rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
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

// Instantiations: scatter -eps on/off x register budget (launch-bounds waves
// per SIMD; 4 = no cap, no spills).
template <bool E>
static const void* persistent_fn(int waves) {
  switch (waves) {
    case 3: return reinterpret_cast<const void*>(&k_persistent<E, 3>);
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

}  // namespace cvr
