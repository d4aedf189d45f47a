// cvr_wavefront.hip - the wavefront scheduler behind regenerationSK (and the
// other persistent/streaming kernel ids).
//
// Why: in the reference's single-kernel schedulers
// (RegenerationVolPTsk_kernel.cuh:146-232, StreamingVolPTsk_kernel.cuh:27-360)
// each thread runs both the Woodcock loop and the rare but long event code
// (GGX boundary ~400 VALU ops, scatter, roulette, camera rays).  On 64-wide
// waves that event code runs for a handful of lanes at a time, and the
// measured persistent single-kernel version executed ~10x the VALU
// instructions the walk needs (profiles/ROUND1_NOTES.md).  Here the walk is
// split at segment boundaries into two kernels over a pool of ray slots in
// HBM (SoA, coalesced):
//
//   k_wf_events  one lane per slot: finishes the segment the tracker ended
//                (scatter or GGX boundary), Russian roulette, AABB test, and
//                regenerates dead slots with new path ids (wave-aggregated
//                chunks of path ids; the RNG is re-seeded from the path id so
//                results do not depend on which slot/lane runs a path).  Stops
//                when the slot needs Woodcock tracking.
//   k_wf_track   persistent: each wave owns a contiguous range of slots and
//                keeps all 64 lanes stepping Woodcock; a lane whose segment
//                ends writes t + RNG back and is refilled from the next
//                TRACK slots of its range (ballot + mbcnt compaction through
//                a 256-byte LDS window) - no atomics, no events inline.
//
// The host alternates the two kernels until no slot is alive.
#include <hip/hip_runtime.h>

#include "cvr_kernels.h"
#include "cvr_walk.h"

namespace cvr {

enum : uint32_t { WF_FREE = 0, WF_TRACK = 1, WF_DONE = 2, WF_EXHAUSTED = 3 };
// meta word: bits 0-1 state, bits 2-4 normal code (0..5 axis, 6 = zero),
// bits 8-31 segments so far (saturating at 2^24-1).
__device__ __forceinline__ uint32_t normal_code(V3 n) {
  if (n.x == 1.0f) return 0;
  if (n.y == 1.0f) return 1;
  if (n.z == 1.0f) return 2;
  if (n.x == -1.0f) return 3;
  if (n.y == -1.0f) return 4;
  if (n.z == -1.0f) return 5;
  return 6;
}
__device__ __forceinline__ V3 normal_from_code(uint32_t c) {
  switch (c) {
    case 0: return mk3(1, 0, 0);
    case 1: return mk3(0, 1, 0);
    case 2: return mk3(0, 0, 1);
    case 3: return mk3(-1, 0, 0);
    case 4: return mk3(0, -1, 0);
    case 5: return mk3(0, 0, -1);
    default: return mk3(0, 0, 0);
  }
}

__device__ __forceinline__ uint32_t wf_lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Per-wave stats row: plain read-modify-write by lane 0 (each wave row is
// owned by exactly one wave of one launch at a time; launches are ordered).
__device__ __forceinline__ void wf_flush_stats(unsigned long long* row, const uint32_t (&c)[STAT_COUNT]) {
#pragma unroll
  for (int k = 0; k < STAT_COUNT; ++k) {
    unsigned long long v = c[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) row[k] += v;
  }
}

// ------------------------------------------------------------- events -----
template <bool kScatterEps>
__global__ __launch_bounds__(256) void k_wf_events(MediumParams m, LaunchParams L, WfPool P) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t wave = s >> 6;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0};
  enum : uint32_t { PH_EVENT = 0, PH_NEW = 1, PH_ISECT = 2, PH_SETTLED = 3 };
  uint32_t phase = PH_SETTLED;
  uint32_t meta = WF_EXHAUSTED;
  if (s < P.n) meta = P.meta[s];
  const uint32_t st0 = meta & 3u;
  PathState ps;
  Isect is;
  float t = 0.0f;
  uint32_t nseg = meta >> 8;
  ps.image_id = 0;
  ps.o = ps.d = ps.T = mk3(0, 0, 0);
  ps.rng = Rng{0, 0, 0, 0, 0, 0};
  is.dist = 0.0f;
  is.inside = true;
  is.normal = normal_from_code((meta >> 2) & 7u);
  if (st0 == WF_DONE) {
    ps.o = mk3(P.ox[s], P.oy[s], P.oz[s]);
    ps.d = mk3(P.dx[s], P.dy[s], P.dz[s]);
    ps.T = mk3(P.tx[s], P.ty[s], P.tz[s]);
    ps.rng = Rng{P.r0[s], P.r1[s], P.r2[s], P.r3[s], P.r4[s], P.rd[s]};
    ps.image_id = P.img[s];
    is.dist = P.dist[s];
    t = P.t[s];
    phase = PH_EVENT;
  } else if (st0 == WF_FREE) {
    phase = PH_NEW;
  }
  // this wave's cursor into the path-id space, persisted across launches
  uint32_t q_next = P.cursor[2 * wave], q_end = P.cursor[2 * wave + 1];
  bool exhausted = false;
  bool dirty = false;  // slot state must be written back

  while (__any(phase != PH_SETTLED)) {
    // ---- regeneration: hand fresh path ids to slots that need one ---------
    unsigned long long need = __ballot(phase == PH_NEW);
    while (need != 0ull && !exhausted) {
      if (q_next == q_end) {
        uint32_t base = 0;
        const uint32_t leader = (uint32_t)__builtin_ctzll(need);
        if ((threadIdx.x & 63) == leader) base = atomicAdd(P.head, L.chunk);
        base = __builtin_amdgcn_readlane(base, leader);
        if (base >= L.path_count) {
          exhausted = true;
          q_next = q_end = 0;
          break;
        }
        q_next = base;
        q_end = min(base + L.chunk, L.path_count);
      }
      const uint32_t take = min((uint32_t)__popcll(need), q_end - q_next);
      const uint32_t rank = wf_lane_rank(need);
      if (phase == PH_NEW && rank < take) {
        path_begin(L, L.path_first + q_next + rank, ps);
        is.normal = mk3(0, 0, 0);
        nseg = 0;
        c[STAT_PATHS]++;
        phase = PH_ISECT;
      }
      q_next += take;
      need = __ballot(phase == PH_NEW);
    }
    if (phase == PH_NEW && exhausted) {
      phase = PH_SETTLED;
      meta = WF_EXHAUSTED;
      dirty = true;
    }
    // ---- finish the tracked segment: scatter or GGX boundary, roulette -----
    if (phase == PH_EVENT) {
      if (t < is.dist) {  // sampleDistance: sampled_distance < dist
        scatter_event<kScatterEps>(m, ps, t);
        c[STAT_ALBEDO]++;
      } else {
        boundary_event(m, ps, is);
      }
      if (roulette(ps)) {
        phase = PH_ISECT;
      } else {
        c[STAT_SEGMENTS] += nseg;
        phase = PH_NEW;
      }
    }
    // ---- next segment: AABB test ------------------------------------------
    if (phase == PH_ISECT) {
      if (L.max_segments && nseg >= L.max_segments) {
        c[STAT_TRUNCATED]++;
        c[STAT_SEGMENTS] += nseg;
        phase = PH_NEW;
      } else {
        ++nseg;
        if (!aabb_intersect(m, ps.o, ps.d, is)) {
          splat(L, ps);
          c[STAT_ESCAPED]++;
          c[STAT_SEGMENTS] += nseg;
          phase = PH_NEW;
        } else if (is.inside) {
          t = 0.0f;
          meta = WF_TRACK;
          phase = PH_SETTLED;
          dirty = true;
        } else {
          t = __builtin_inff();  // no medium: boundary event at is.dist
          phase = PH_EVENT;
        }
      }
    }
  }
  if (s < P.n && dirty) {
    if (meta == WF_TRACK) {
      P.ox[s] = ps.o.x;
      P.oy[s] = ps.o.y;
      P.oz[s] = ps.o.z;
      P.dx[s] = ps.d.x;
      P.dy[s] = ps.d.y;
      P.dz[s] = ps.d.z;
      P.tx[s] = ps.T.x;
      P.ty[s] = ps.T.y;
      P.tz[s] = ps.T.z;
      P.r0[s] = ps.rng.v0;
      P.r1[s] = ps.rng.v1;
      P.r2[s] = ps.rng.v2;
      P.r3[s] = ps.rng.v3;
      P.r4[s] = ps.rng.v4;
      P.rd[s] = ps.rng.d;
      P.img[s] = ps.image_id;
      P.dist[s] = is.dist;
      P.meta[s] = WF_TRACK | (normal_code(is.normal) << 2) | (min(nseg, 0xFFFFFFu) << 8);
      P.alive[0] = 1u;
    } else {
      P.meta[s] = WF_EXHAUSTED;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    P.cursor[2 * wave] = q_next;
    P.cursor[2 * wave + 1] = q_end;
  }
  wf_flush_stats(P.stats_events + (size_t)wave * 8, c);
}

// -------------------------------------------------------------- track -----
__global__ __launch_bounds__(256) void k_wf_track(MediumParams m, LaunchParams L, WfPool P) {
  __shared__ uint32_t window[4][64];
  const uint32_t lane = threadIdx.x & 63, wslot = threadIdx.x >> 6;
  const uint32_t wave = blockIdx.x * 4 + wslot;
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t per = (P.n + nwaves - 1) / nwaves;
  const uint32_t r_begin = min(wave * per, P.n), r_end = min(r_begin + per, P.n);
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0};

  uint32_t win = r_begin;  // current 64-slot window
  uint32_t win_used = 0;   // TRACK slots of the window already handed out
  unsigned long long win_mask = 0ull;
  bool win_loaded = false;

  bool active = false;
  uint32_t slot = 0;
  V3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
  float max_t = 0.0f, t = 0.0f;
  Rng rng{0, 0, 0, 0, 0, 0};
  const uint32_t thresh = L.ev_thresh;

  for (;;) {
    // ---- refill idle lanes from this wave's slot range --------------------
    unsigned long long idle = __ballot(!active);
    const uint32_t n_idle = (uint32_t)__popcll(idle);
    if (n_idle >= thresh || n_idle == 64u) {
      while (idle != 0ull && win < r_end) {
        if (!win_loaded) {
          const uint32_t sl = win + lane;
          const bool tr = sl < r_end && (P.meta[sl] & 3u) == WF_TRACK;
          win_mask = __ballot(tr);
          if (tr) window[wslot][wf_lane_rank(win_mask)] = sl;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          win_used = 0;
          win_loaded = true;
        }
        const uint32_t avail = (uint32_t)__popcll(win_mask) - win_used;
        const uint32_t take = min(avail, (uint32_t)__popcll(idle));
        const uint32_t rank = wf_lane_rank(idle);
        if (!active && rank < take) {
          slot = window[wslot][win_used + rank];
          active = true;
          o = mk3(P.ox[slot], P.oy[slot], P.oz[slot]);
          d = mk3(P.dx[slot], P.dy[slot], P.dz[slot]);
          max_t = P.dist[slot];
          rng = Rng{P.r0[slot], P.r1[slot], P.r2[slot], P.r3[slot], P.r4[slot], P.rd[slot]};
          t = 0.0f;
        }
        win_used += take;
        if (win_used == (uint32_t)__popcll(win_mask)) {
          win += 64;
          win_loaded = false;
        }
        idle = __ballot(!active);
      }
    }
    if (!__any(active)) break;
    // ---- one Woodcock step per active lane ---------------------------------
    if (active) {
      const int r = woodcock_step(m, o, d, max_t, t, rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
      if (r != 0) {
        P.t[slot] = t;
        P.r0[slot] = rng.v0;
        P.r1[slot] = rng.v1;
        P.r2[slot] = rng.v2;
        P.r3[slot] = rng.v3;
        P.r4[slot] = rng.v4;
        P.rd[slot] = rng.d;
        P.meta[slot] = (P.meta[slot] & ~3u) | WF_DONE;
        active = false;
      }
    }
  }
  wf_flush_stats(P.stats_track + (size_t)wave * 8, c);
}

// --------------------------------------------------------- stats reduce ---
__global__ __launch_bounds__(256) void k_wf_reduce(const unsigned long long* rows, uint32_t nrows,
                                                   unsigned long long* out) {
  __shared__ unsigned long long part[256][STAT_COUNT];
  unsigned long long acc[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0};
  for (uint32_t r = threadIdx.x; r < nrows; r += 256)
#pragma unroll
    for (int k = 0; k < STAT_COUNT; ++k) acc[k] += rows[(size_t)r * 8 + k];
#pragma unroll
  for (int k = 0; k < STAT_COUNT; ++k) part[threadIdx.x][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < STAT_COUNT) {
    unsigned long long v = 0;
    for (int i = 0; i < 256; ++i) v += part[i][threadIdx.x];
    out[threadIdx.x] = v;
  }
}

// ----------------------------------------------------------- launchers ----
hipError_t wf_launch_events(const MediumParams& m, const LaunchParams& L, const WfPool& P, bool scatter_eps,
                            hipStream_t s) {
  const uint32_t grid = (P.n + 255u) / 256u;
  if (scatter_eps)
    hipLaunchKernelGGL(k_wf_events<true>, dim3(grid), dim3(256), 0, s, m, L, P);
  else
    hipLaunchKernelGGL(k_wf_events<false>, dim3(grid), dim3(256), 0, s, m, L, P);
  return hipGetLastError();
}

hipError_t wf_launch_track(const MediumParams& m, const LaunchParams& L, const WfPool& P, uint32_t grid,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_wf_track, dim3(grid), dim3(256), 0, s, m, L, P);
  return hipGetLastError();
}

hipError_t wf_track_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_wf_track, 256, 0);
}

hipError_t wf_launch_reduce(const unsigned long long* rows, uint32_t nrows, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_wf_reduce, dim3(1), dim3(256), 0, s, rows, nrows, out);
  return hipGetLastError();
}

}  // namespace cvr
