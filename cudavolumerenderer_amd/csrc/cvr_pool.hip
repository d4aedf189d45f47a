// cvr_pool.hip - regenerationSK with a per-workgroup path pool in LDS (gfx950).
//
// Semantics: RegenerationVolPTsk_kernel::d_render_single_thread_regeneration
// (RegenerationVolPTsk_kernel.cuh:146-232): persistent work-items take new
// paths from a global counter as paths end; no -eps at the scatter point
// (:212).  The RNG is bound to the path id, so the image is
// independent of the scheduling below.
//
// Why a pool: the walk is VALU-bound once the brick
// bounds remove most density fetches, and a wave that owns its 64 paths runs
// its Woodcock loop with about half the lanes idle (paths wait for the rest
// of the wave before their event code runs) and runs the event code for a mix
// of event kinds.  Here a workgroup keeps kSlots paths in LDS and alternates
// two bulk-synchronous phases:
//   EVENT  every path whose segment ended is handled by one lane, the items
//          ordered [boundary | collision | new], so a wave runs one kind of
//          event code; the lane then runs roulette, regeneration and the AABB
//          test, and files the path as track-ready or as a deferred boundary.
//   TRACK  lanes pull track-ready paths from the pool and run Woodcock steps;
//          a lane whose segment ends files it as an event and pulls the next
//          path, so lanes stay busy while the pool has work.  When the pool
//          is empty and fewer than `tail` lanes of a wave still track, they
//          park their (t, rng) back in the pool and the wave stops.
// Pool slots are SoA in LDS; the lists are u16 slot indices.  Every list is
// either read or appended to within a phase, never both, so the only
// synchronisation is one barrier between phases and wave-aggregated LDS
// atomics for appends.
#include <hip/hip_runtime.h>

#include "cvr_kernels.h"
#include "cvr_walk.h"

#ifndef CVR_STAMPS
#define CVR_STAMPS 0
#endif
#ifndef CVR_POOL_WATCHDOG
#define CVR_POOL_WATCHDOG 1
#endif

namespace cvr {

namespace {

constexpr int kThreads = 256;
constexpr int kSlots = 448;

struct PoolLds {
  float ox[kSlots], oy[kSlots], oz[kSlots], dx[kSlots], dy[kSlots], dz[kSlots];
  float tx[kSlots], ty[kSlots], tz[kSlots], dist[kSlots], t[kSlots];
  uint32_t r0[kSlots], r1[kSlots], r2[kSlots], r3[kSlots], r4[kSlots], rd[kSlots];
  uint32_t img[kSlots];
  uint32_t meta[kSlots];  // bits 0-2 normal code, bit 3 inside, bits 4.. segments so far
  uint16_t ready[2][kSlots];  // track-ready slots (read by TRACK / appended by EVENT and TRACK)
  uint16_t lb[2][kSlots];     // boundary events (read by EVENT / appended by TRACK and EVENT)
  uint16_t lc[kSlots];        // real collisions (appended by TRACK, read by EVENT)
  uint32_t n_ready[2], n_lb[2], n_lc, n_new, ready_head;
  uint32_t cur_next, cur_end, cur_q, exhausted;  // workgroup path cursor into the global queues
  uint32_t skey[512];  // Morton sort of a track phase's ready list (streamingSK): code << 9 | slot
};
static_assert(kSlots <= 512, "Morton sort keys hold 9-bit slot indices");

// Utilities.h:35-55: 30-bit Morton code of a point in the unit cube.
__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}
__device__ __forceinline__ uint32_t morton3d(float x, float y, float z) {
  x = fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f);
  y = fminf(fmaxf(y * 1024.0f, 0.0f), 1023.0f);
  z = fminf(fmaxf(z * 1024.0f, 0.0f), 1023.0f);
  return expand_bits((uint32_t)x) * 4u + expand_bits((uint32_t)y) * 2u + expand_bits((uint32_t)z);
}

// streamingSK's ray order (StreamingVolPTsk_kernel.cuh:188-216,
// MortonSort.h:28-49): the track phase's ready paths sorted by the Morton code
// of their origin in the box (AABB::transform), so the lanes of a wave, which
// take consecutive ready entries, trace nearby rays.  Bitonic sort of up to
// 512 keys (the code's top 23 bits above the 9-bit slot) by the workgroup.
// Scheduling only: every path still runs its own RNG stream.
__device__ void morton_sort_ready(PoolLds& S, const MediumParams& m, uint16_t* ready, uint32_t n) {
  const uint32_t tid = threadIdx.x;
  uint32_t P = 64u;
  while (P < n) P <<= 1;
  const V3 ext = sub3(m.bmax, m.bmin);
  for (uint32_t i = tid; i < P; i += kThreads) {
    uint32_t key = 0xFFFFFFFFu;
    if (i < n) {
      const uint32_t sl = ready[i];
      const V3 p = div3(sub3(mk3(S.ox[sl], S.oy[sl], S.oz[sl]), m.bmin), ext);
      key = ((morton3d(p.x, p.y, p.z) >> 7) << 9) | sl;
    }
    S.skey[i] = key;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = tid; t < P / 2; t += kThreads) {
        const uint32_t lo = ((t & ~(j - 1u)) << 1) | (t & (j - 1u)), hi = lo + j;
        const uint32_t a = S.skey[lo], b = S.skey[hi];
        if ((a > b) == ((lo & k) == 0u)) {
          S.skey[lo] = b;
          S.skey[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = tid; i < n; i += kThreads) ready[i] = (uint16_t)(S.skey[i] & 511u);
  __syncthreads();
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Append the calling lanes (pred) to an LDS list: one atomic per wave.
__device__ __forceinline__ void list_append(bool pred, uint32_t* count, uint16_t* list, uint32_t slot) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0ull) return;
  uint32_t base = 0;
  if ((threadIdx.x & 63) == (uint32_t)(__ffsll((long long)mask) - 1)) base = atomicAdd(count, (uint32_t)__popcll(mask));
  base = __shfl(base, __ffsll((long long)mask) - 1);
  if (pred) list[base + lane_rank(mask)] = (uint16_t)slot;
}

__device__ __forceinline__ uint32_t normal_code(V3 n) {
  return n.x > 0.f ? 1u : n.x < 0.f ? 2u : n.y > 0.f ? 3u : n.y < 0.f ? 4u : n.z > 0.f ? 5u : n.z < 0.f ? 6u : 0u;
}
__device__ __forceinline__ V3 normal_of(uint32_t c) {
  const float s = (c & 1u) ? 1.0f : -1.0f;
  return c == 0u ? mk3(0, 0, 0) : c <= 2u ? mk3(s, 0, 0) : c <= 4u ? mk3(0, s, 0) : mk3(0, 0, s);
}

__device__ __forceinline__ void store_full(PoolLds& S, uint32_t s, const PathState& ps, const Isect& is, uint32_t nseg,
                                           float t) {
  S.ox[s] = ps.o.x;
  S.oy[s] = ps.o.y;
  S.oz[s] = ps.o.z;
  S.dx[s] = ps.d.x;
  S.dy[s] = ps.d.y;
  S.dz[s] = ps.d.z;
  S.tx[s] = ps.T.x;
  S.ty[s] = ps.T.y;
  S.tz[s] = ps.T.z;
  S.dist[s] = is.dist;
  S.t[s] = t;
  S.r0[s] = ps.rng.v0;
  S.r1[s] = ps.rng.v1;
  S.r2[s] = ps.rng.v2;
  S.r3[s] = ps.rng.v3;
  S.r4[s] = ps.rng.v4;
  S.rd[s] = ps.rng.d;
  S.img[s] = ps.image_id;
  S.meta[s] = normal_code(is.normal) | (is.inside ? 8u : 0u) | (nseg << 4);
}
__device__ __forceinline__ void load_full(const PoolLds& S, uint32_t s, PathState& ps, Isect& is, uint32_t& nseg,
                                          float& t) {
  ps.o = mk3(S.ox[s], S.oy[s], S.oz[s]);
  ps.d = mk3(S.dx[s], S.dy[s], S.dz[s]);
  ps.T = mk3(S.tx[s], S.ty[s], S.tz[s]);
  is.dist = S.dist[s];
  t = S.t[s];
  ps.rng = Rng{S.r0[s], S.r1[s], S.r2[s], S.r3[s], S.r4[s], S.rd[s]};
  ps.image_id = S.img[s];
  const uint32_t meta = S.meta[s];
  is.normal = normal_of(meta & 7u);
  is.inside = (meta & 8u) != 0u;
  nseg = meta >> 4;
}

enum : uint32_t { K_BOUNDARY = 0, K_COLLIDE = 1, K_NEW = 2, K_NONE = 3 };

}  // namespace

// Global work queues (LaunchParams::queue, 8 bands): take up to `want` units,
// home band first, then the others.  One lane calls; returns the count.
__device__ __forceinline__ uint32_t queue_take(const LaunchParams& L, uint32_t& q_home, uint32_t want,
                                               uint32_t& base, uint32_t& q) {
  for (uint32_t k = 0; k < L.n_queues; ++k) {
    const uint32_t qq = (q_home + k) % L.n_queues;
    const uint32_t units = queue_units(L, qq);
    const uint32_t b = atomicAdd(L.queue + 16 * qq, want);
    if (b < units) {
      q_home = qq;
      base = b;
      q = qq;
      return min(want, units - b);
    }
  }
  return 0;
}

template <bool kScatterEps>
__global__ __launch_bounds__(kThreads, 4) void k_pool(MediumParams m, LaunchParams L) {
  __shared__ PoolLds S;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  uint32_t c[STAT_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t seg_sum = 0;
  // home band of this XCD (HW_REG_XCC_ID; speed only)
  uint32_t q_home = (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u) % L.n_queues;
  const uint32_t tail = L.tail;                // TRACK: park when the pool is dry and fewer lanes track
  const uint32_t batch = L.ev_thresh;          // TRACK: swap finished segments in batches of this many lanes
  const uint32_t wg_chunk = max(L.chunk, 64u);  // units the workgroup cursor takes from a global queue

  if (tid == 0) {
    S.n_ready[0] = S.n_ready[1] = 0;
    S.n_lb[0] = S.n_lb[1] = 0;
    S.n_lc = 0;
    S.n_new = kSlots;  // the first EVENT phase fills every slot with a new path
    S.ready_head = 0;
    S.cur_next = S.cur_end = 0;
    S.cur_q = 0;
    S.exhausted = 0;
  }
  __syncthreads();
  uint32_t rp = 0;  // ready[rp] is read by TRACK, ready[rp^1] appended
  uint32_t bp = 0;  // lb[bp] is read by EVENT, lb[bp^1] appended
#if CVR_POOL_WATCHDOG
  uint32_t rounds = 0;
#endif
#if CVR_STAMPS
  unsigned long long st[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t_mark = __builtin_amdgcn_s_memtime();
#define CVR_STAMP(k)                                              \
  {                                                               \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    st[k] += now_ - t_mark;                                       \
    t_mark = now_;                                                \
  }
#else
#define CVR_STAMP(k)
#endif

  for (;;) {
#if CVR_POOL_WATCHDOG
    if (++rounds > (1u << 22)) {
      if (tid == 0) atomicAdd(L.stats + 16, 1ull);
      break;
    }
#endif
    // ========================================================== EVENT ======
    // refill the workgroup's path cursor (one lane, before anyone reads it)
    if (tid == 0 && S.cur_next >= S.cur_end && !S.exhausted) {
      uint32_t b = 0, q = 0;
      const uint32_t got = queue_take(L, q_home, wg_chunk, b, q);
      if (got) {
        S.cur_next = b;
        S.cur_end = b + got;
        S.cur_q = q;
      } else {
        S.exhausted = 1;
      }
    }
    __syncthreads();
    const uint32_t nb = S.n_lb[bp], nc = S.n_lc, nn = S.n_new;
    const uint32_t total = nb + nc + nn;
    for (uint32_t base = 0; base < total; base += kThreads) {
      const uint32_t v = base + tid;
      uint32_t kind = K_NONE, slot = 0;
      if (v < nb) {
        kind = K_BOUNDARY;
        slot = S.lb[bp][v];
      } else if (v < nb + nc) {
        kind = K_COLLIDE;
        slot = S.lc[v - nb];
      } else if (v < total) {
        kind = K_NEW;
        slot = v - nb - nc;
      }
      PathState ps;
      Isect is;
      uint32_t nseg = 0;
      float t_hit = 0.0f;
      bool alive = false;
      if (kind <= K_COLLIDE) load_full(S, slot, ps, is, nseg, t_hit);
      if (kind == K_BOUNDARY) {
        boundary_event(m, ps, is);
        alive = true;
      } else if (kind == K_COLLIDE) {
        scatter_event<kScatterEps>(m, ps, t_hit);
        ++c[STAT_ALBEDO];
        alive = true;
      }
      if (alive) {
        alive = roulette(ps);
        if (!alive) seg_sum += nseg;
      }
      bool need = kind != K_NONE;  // the slot must be resolved in this round
      bool to_ready = false, to_lb = false;
#if CVR_POOL_WATCHDOG
      uint32_t guard = 0;
#endif
      for (;;) {
#if CVR_POOL_WATCHDOG
        if (++guard > (1u << 20)) {
          if (lane == 0) atomicAdd(L.stats + 17, 1ull);
          break;
        }
#endif
        // ---- regeneration: lanes whose slot has no live path take a new one:
        // from the workgroup cursor, then straight from the global queues.
        const unsigned long long idle = __ballot(need && !alive);
        if (idle != 0ull) {
          const uint32_t want = (uint32_t)__popcll(idle), rank = lane_rank(idle);
          uint32_t b0 = 0, g0 = 0, q0 = 0, b1 = 0, g1 = 0, q1 = 0;
          if (lane == 0) {
            const uint32_t b = atomicAdd(&S.cur_next, want);
            const uint32_t end = S.cur_end;
            q0 = S.cur_q;
            if (b < end) {
              b0 = b;
              g0 = min(want, end - b);
            }
            if (g0 < want && !*(volatile uint32_t*)&S.exhausted) {
              g1 = queue_take(L, q_home, want - g0, b1, q1);
              if (g1 == 0) atomicOr(&S.exhausted, 1u);
            }
          }
          b0 = __shfl(b0, 0);
          g0 = __shfl(g0, 0);
          q0 = __shfl(q0, 0);
          b1 = __shfl(b1, 0);
          g1 = __shfl(g1, 0);
          q1 = __shfl(q1, 0);
          if (need && !alive) {
            if (rank < g0 + g1) {
              const uint32_t unit = rank < g0 ? unit_to_path(L, q0, b0 + rank) : unit_to_path(L, q1, b1 + rank - g0);
              path_begin(L, unit, ps);
              is.normal = mk3(0, 0, 0);
              nseg = 0;
              alive = true;
              ++c[STAT_PATHS];
            } else {
              need = false;  // no paths left anywhere: the slot stays empty
            }
          }
        }
        // ---- next segment: AABB test (NaiveVolPTsk_kernel.cuh:33-47) -----
        if (need && alive) {
          if (L.max_segments && nseg >= L.max_segments) {
            ++c[STAT_TRUNCATED];
            seg_sum += nseg;
            alive = false;
          } else {
            ++nseg;
            if (!aabb_intersect(m, ps.o, ps.d, is)) {
              splat(L, ps);
              ++c[STAT_ESCAPED];
              seg_sum += nseg;
              alive = false;
            } else {
              store_full(S, slot, ps, is, nseg, 0.0f);
              to_ready = is.inside;  // medium: Woodcock from t = 0
              to_lb = !is.inside;    // no medium: boundary at isect.dist
              need = false;
            }
          }
        }
        if (!__any(need)) break;
      }
      list_append(to_ready, &S.n_ready[rp ^ 1], S.ready[rp ^ 1], slot);
      list_append(to_lb, &S.n_lb[bp ^ 1], S.lb[bp ^ 1], slot);
#if CVR_STAMPS
      ++st[5];
#endif
    }
    CVR_STAMP(0)
    __syncthreads();
    // No live path in this workgroup (nothing to track, no deferred boundary;
    // the cursor is drained because every dead path tried to regenerate).
    // Read before the next barrier: TRACK appends to lb[bp^1].
    const bool done = S.n_ready[rp ^ 1] == 0 && S.n_lb[bp ^ 1] == 0;
    __syncthreads();
    if (tid == 0) {
      S.n_ready[rp] = 0;
      S.n_lb[bp] = 0;
      S.n_lc = 0;
      S.n_new = 0;
      S.ready_head = 0;
    }
    rp ^= 1;
    __syncthreads();
    CVR_STAMP(1)
    if (done) break;
    if ((L.naive_mk & 2u) && S.n_ready[rp] > 64u) morton_sort_ready(S, m, S.ready[rp], S.n_ready[rp]);

    // ========================================================== TRACK ======
    {
      const uint32_t n_ready = S.n_ready[rp];
      int slot = -1;      // pool slot of the lane's path, -1 = none
      bool fin = false;   // the lane's segment ended; filed at the next swap
      bool coll = false;  // ... as a real collision (else a boundary)
      V3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
      Rng rng{0, 0, 0, 0, 0, 0};
      float t = 0.0f, max_t = 0.0f;
      bool dry = false;  // wave-uniform: the ready list is used up
#if CVR_POOL_WATCHDOG
      uint32_t guard = 0;
#endif
      for (;;) {
#if CVR_POOL_WATCHDOG
        if (++guard > (1u << 24)) {
          if (lane == 0) atomicAdd(L.stats + 18, 1ull);
          break;
        }
#endif
        const unsigned long long trk = __ballot(slot >= 0 && !fin);
        const unsigned long long idle = ~trk;  // finished or empty lanes
        const uint32_t n_idle = 64u - (uint32_t)__popcll(trk);
        // ---- swap: file finished segments, pull track-ready paths --------
        if (n_idle != 0u && (n_idle >= batch || trk == 0ull || (dry && n_idle > 0u))) {
          if (fin) {
            S.t[slot] = t;
            S.r0[slot] = rng.v0;
            S.r1[slot] = rng.v1;
            S.r2[slot] = rng.v2;
            S.r3[slot] = rng.v3;
            S.r4[slot] = rng.v4;
            S.rd[slot] = rng.d;
          }
          list_append(fin && coll, &S.n_lc, S.lc, (uint32_t)slot);
          list_append(fin && !coll, &S.n_lb[bp ^ 1], S.lb[bp ^ 1], (uint32_t)slot);
          if (fin) {
            slot = -1;
            fin = false;
          }
          if (!dry) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&S.ready_head, n_idle);
            b = __shfl(b, 0);
            const uint32_t avail = b < n_ready ? min(n_ready - b, n_idle) : 0u;
            if (avail < n_idle) dry = true;
            const uint32_t rank = lane_rank(idle);
            if (slot < 0 && rank < avail) {
              const uint32_t s = S.ready[rp][b + rank];
              slot = (int)s;
              o = mk3(S.ox[s], S.oy[s], S.oz[s]);
              d = mk3(S.dx[s], S.dy[s], S.dz[s]);
              rng = Rng{S.r0[s], S.r1[s], S.r2[s], S.r3[s], S.r4[s], S.rd[s]};
              t = S.t[s];
              max_t = S.dist[s];
            }
          }
        }
        const unsigned long long act = __ballot(slot >= 0 && !fin);
        if (act == 0ull) {
          if (dry) break;
          continue;
        }
        // Park the remaining segments ((t, rng) back to the pool) when the
        // pool is dry, few lanes still track and the workgroup has at least
        // a wave's worth of events waiting; otherwise keep stepping, so every
        // round makes progress.  (Finished lanes were filed by the swap.)
        if (dry && (uint32_t)__popcll(act) < tail &&
            *(volatile uint32_t*)&S.n_lc + *(volatile uint32_t*)&S.n_lb[bp ^ 1] >= 64u) {
          if (slot >= 0) {
            S.t[slot] = t;
            S.r0[slot] = rng.v0;
            S.r1[slot] = rng.v1;
            S.r2[slot] = rng.v2;
            S.r3[slot] = rng.v3;
            S.r4[slot] = rng.v4;
            S.rd[slot] = rng.d;
          }
          list_append(slot >= 0, &S.n_ready[rp ^ 1], S.ready[rp ^ 1], (uint32_t)slot);
          break;
        }
#if CVR_STAMPS
        ++st[4];
#endif
        if (slot >= 0 && !fin) {
          const int r = woodcock_step(m, o, d, max_t, t, rng, c[STAT_STEPS], c[STAT_DENSITY], c[STAT_FETCH]);
          if (r != 0) {
            fin = true;
            coll = (r == 2) && (t < max_t);
          }
        }
      }
    }
    CVR_STAMP(2)
    __syncthreads();
    CVR_STAMP(3)
    bp ^= 1;
  }
#if CVR_STAMPS
  if (lane == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(L.stats + 16 + k, st[k]);
#endif

  // ---- counters ------------------------------------------------------------
  c[STAT_SEGMENTS] = seg_sum;
#pragma unroll
  for (int k = 0; k < STAT_COUNT; ++k) {
    unsigned long long v = c[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(L.stats + k, v);
  }
}

hipError_t launch_pool(const MediumParams& m, const LaunchParams& L, bool scatter_eps, uint32_t grid,
                       hipStream_t s) {
  if (L.path_count == 0) return hipSuccess;
  if (scatter_eps)
    hipLaunchKernelGGL(k_pool<true>, dim3(grid), dim3(kThreads), 0, s, m, L);
  else
    hipLaunchKernelGGL(k_pool<false>, dim3(grid), dim3(kThreads), 0, s, m, L);
  return hipGetLastError();
}

hipError_t pool_occupancy(bool scatter_eps, int* blocks_per_cu) {
  const void* fn = scatter_eps ? reinterpret_cast<const void*>(&k_pool<true>)
                               : reinterpret_cast<const void*>(&k_pool<false>);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, kThreads, 0);
}

}  // namespace cvr
