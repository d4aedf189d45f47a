// cvr_wpool.hip - regenerationSK with a wave-private path pool in LDS (gfx950).
//
// Semantics: RegenerationVolPTsk_kernel::d_render_single_thread_regeneration
// (RegenerationVolPTsk_kernel.cuh:146-232): persistent work-items take new
// paths from a global counter as paths end; no -eps at the scatter point
// (:212).  The RNG is bound to the path id, so the image is
// independent of the scheduling below.
//
// Why: with brick bounds the walk is VALU-bound, and a
// wave whose 64 lanes each own one path keeps about half of its lanes idle in
// the Woodcock loop (a finished segment waits until enough of the wave is
// done before the event code runs, and that code then runs once per event
// kind present).  Here each wave (one workgroup = one wave) owns kSlots > 64
// paths kept in LDS:
//   * TRACK: lanes run Woodcock steps on track-ready paths; a lane whose
//     segment ends files it in the boundary or collision list and takes the
//     next track-ready path, so all 64 lanes keep stepping while the wave has
//     more paths than lanes.
//   * EVENT: once 64 events are waiting, the tracking lanes park (t, rng) in
//     their slots and the wave handles 64 events at once, boundary events
//     first, then collisions, so each part runs one kind of event code on a
//     full wave; roulette, regeneration and the AABB test follow, and each
//     path goes back to the track-ready ring or the boundary list.
// The pool is private to the wave and the wave runs in lockstep, so the lists
// need no atomics and no barriers: their counters are wave-uniform scalars.
#include <hip/hip_runtime.h>

#include "cvr_kernels.h"
#include "cvr_walk.h"

// Woodcock steps per track iteration between swap/event checks.
#ifndef CVR_WPOOL_UNROLL
#define CVR_WPOOL_UNROLL 4
#endif
// Sparse media: stage the empty-region mask in LDS and skip the brick-word
// loads of points in clear super-bricks (woodcock_point_em).
#ifndef CVR_WPOOL_EMASK
#define CVR_WPOOL_EMASK 1
#endif
// Waves per workgroup of the sparse instances (round 6): each wave keeps its own
// pool, and the workgroup stages the launch parameters and the empty-region mask
// (kEmaskWords words) once for all of them, so a finer mask costs each wave
// 1/kWpg of its LDS.  1: one wave per workgroup (every dense instance).
#ifndef CVR_WPOOL_SPARSE_WPG
#define CVR_WPOOL_SPARSE_WPG 4
#endif
// The same for the dense instances (experiment: 1 is one wave per workgroup).
#ifndef CVR_WPOOL_DENSE_WPG
#define CVR_WPOOL_DENSE_WPG 1
#endif
// Tentative points per lane per Woodcock group (the lookahead below).  The
// track loop runs CVR_WPOOL_UNROLL / kLook groups between swap checks.
// Sparse instances: a point that needs its cell parks until the end of the track
// iteration (kLookDefer below).
#ifndef CVR_WPOOL_SPARSE_DEFER
#define CVR_WPOOL_SPARSE_DEFER 1
#endif
// The workgroup-shared event lists (k_wpair, CVR_OPT_WAVE_PAIR): an experiment
// that lost 4.1x, built only into `make variant-pair`.
#ifndef CVR_WPOOL_PAIR
#define CVR_WPOOL_PAIR 0
#endif
// Diagnostic build (make variant NAME=tail DEFS=-DCVR_WPOOL_TAILSTAMP=1, tools/tail_wpool.py):
// per wave, s_memrealtime at its start, when it first finds every queue exhausted and at its
// end, with its live paths and event batches after that point.
#ifndef CVR_WPOOL_TAILSTAMP
#define CVR_WPOOL_TAILSTAMP 0
#endif
// The drain's wide track (round 6, wide_track): once every queue is exhausted and
// at most 64 / CVR_WPOOL_WIDE paths are ready, each gets CVR_WPOOL_WIDE lanes that
// evaluate its next CVR_WPOOL_WIDE tentative points at once.  0: off, the default:
// bit-exact but no faster (K 16 / 8 / 4: one render at a time +0.1-0.3%, the 1/8
// block shard +1%, renders in flight -0.5-1%; profiles/round6/ab/wide_drain_ab.log),
// since half of a draining wave's time is its event batches, which stay one lane
// per path (profiles/round6/tail_c2_stamps.log).
#ifndef CVR_WPOOL_WIDE
#define CVR_WPOOL_WIDE 0
#endif
#ifndef CVR_WPOOL_LOOK
#define CVR_WPOOL_LOOK 2
#endif
// Cell fetches as track-ready work (round-6 experiment, dense instances with cells and
// bounds; 0: off, the default and the only form in libcvr.so).  A point the brick bound
// does not settle ends the lane's turn: the path's (t, rng) go back to the pool and its slot
// joins the track-ready ring marked "fetch pending" (bit 7 of the ring entry); the lanes
// that pull marked entries at a swap fetch their cells together and either file a
// collision or track on, so no lane idles for another lane's cell and the two per-group
// fetch blocks of the track loop (~5% lane fill) go away.  The same points and draws: the
// test value is the path's last draw, re-derived from the stored XORWOW state.
#ifndef CVR_WPOOL_FETCH_LIST
#define CVR_WPOOL_FETCH_LIST 0
#endif
constexpr int kLook = CVR_WPOOL_LOOK;
// The track loop runs CVR_WPOOL_UNROLL / kLook groups: a variant build with
// UNROLL < kLook would run none (tracking lanes never step: the launch never
// ends), one with a remainder would silently drop the remainder's steps.
static_assert(CVR_WPOOL_UNROLL >= kLook && CVR_WPOOL_UNROLL % kLook == 0,
              "CVR_WPOOL_UNROLL must be a positive multiple of kLook");
// Wave priorities (s_setprio): the track loop above the event code, so a
// stepping wave issues its brick-bound and cell loads ahead of the
// VALU-dense event batches of the other waves on its SIMD (C2: -0.7%).
constexpr int kPrioTrack = 1, kPrioEvent = 0;

namespace cvr {

namespace {

// An SGPR value the compiler may not look through: computations that depend on
// it stay where they are written (inside the event batch) instead of being
// hoisted to the kernel prologue and held in VGPRs for the whole kernel.
__device__ __forceinline__ float opaque_s(float x) {
  asm volatile("" : "+s"(x));
  return x;
}

// Paths per wave for a register/LDS budget of kWaves waves per SIMD: pool +
// launch parameters must fit 160 KB / (4 kWaves) of LDS, or the CU holds
// fewer waves than the register budget allows (round 1 lost 7% to an 8-byte
// LaunchParams growth that pushed the workgroup to 10248 bytes).  Derived from
// sizeof(LaunchParams): 64 LDS bytes per slot, 154 slots at 4 waves per SIMD,
// 122 at 5.  The pool size matters: lanes step only while the pool holds
// track-ready paths besides the events waiting for a batch (93 slots instead
// of 118 at 4 waves cost 13% on C2).
// LDS is handed to workgroups in 1280-byte granules (measured, tools/census.hip:
// one-wave workgroups of 7680 B fit 20 per CU, of 7936 / 8064 / 8192 B only 18,
// although the occupancy API answers 20 for all of them; 10240 B fit 16).  A
// budget of 163840 / 20 = 8192 B therefore ran 4.5 waves per SIMD, not 5.
constexpr int kLdsGranule = 1280;
template <int kWaves, int kExtra = 0, int kWpg = 1>
struct PoolSize {
  static_assert((4 * kWaves) % kWpg == 0, "a CU's waves split into whole workgroups");
  // LDS bytes per workgroup of kWpg waves (kExtra: bytes of it shared by its waves,
  // besides the launch parameters)
  static constexpr int kBudget = 163840 / (4 * kWaves / kWpg) / kLdsGranule * kLdsGranule;
  static constexpr int kParams = (int)((sizeof(LaunchParams) + 15) / 16 * 16);
  static constexpr int value = ((kBudget - kParams - kExtra) / kWpg - 24 - 4 * STAT_COUNT) / 64;
  static_assert(4 * STAT_COUNT + 8 + 12 + 4 <= 4 * STAT_COUNT + 24, "pool header exceeds its LDS reserve");
};
constexpr int kWpgSparse = CVR_WPOOL_SPARSE_WPG, kWpgDense = CVR_WPOOL_DENSE_WPG;
// waves per workgroup of an instance (kMedMk's low bits: the medium layout): kWpgSparse
// on sparse media (kWpgDense on dense ones) when a CU's 4 kWaves waves split into such
// workgroups, else 4 (sparse) or 1 (dense)
constexpr int wpg_of(int kMedMk, int kWaves) {
  return (kMedMk & 3) != 1 /* kMedSparse */ ? ((4 * kWaves) % kWpgDense == 0 ? kWpgDense : 1)
                                            : ((4 * kWaves) % kWpgSparse == 0 ? kWpgSparse : 4);
}
// Sparse media (C5) split the slot too and run 5 waves per SIMD: 142.7 ms vs
// 147.6 with the event part in LDS at 4 waves (round 3, once the global part's
// loads and stores stopped being flat instructions that LDS waits also waited
// for; round 2 measured 156.8 split at 4 waves, 153.7 at 5).

// One path per slot.  LDS holds what the track loop and the event code both
// need, as arrays of 16-byte blocks (ds_read_b128 / ds_write_b128):
//   a = (o.x, o.y, o.z, t)   b = (d.x, d.y, d.z, dist)   c = rng v0..v3
//   e = (rng v4, rng d)      meta: bits 0-2 normal code, bit 3 inside, bits 4.. segments
// The event-only part, (T.x, T.y, T.z, image_id), lives in global memory
// (L.pool_T, one float4 per slot of every wave: ~10 MB, L2-resident), read
// and written once per event; so a slot takes 64 LDS bytes instead of 84 and
// the pool holds 30% more paths, enough for 5 waves per SIMD (C2: 5.25 ms
// vs 5.40 at 4 waves with the whole slot in LDS).
// Sparse instances also stage the medium's empty-region mask (MediumParams::
// emask, kEmaskWords words; CVR_WPOOL_EMASK), once per workgroup beside the
// launch parameters (k_wpool's EM).
template <int kSlots>
struct WavePool {
  float4 a[kSlots], b[kSlots];
  uint4 c[kSlots];
  uint2 e[kSlots];
  uint32_t meta[kSlots];
  uint8_t ready[kSlots];   // ring of track-ready slots
  uint8_t lb[kSlots];      // stack of boundary events
  uint8_t lc[kSlots];      // stack of real collisions
  uint8_t ln[kSlots];      // stack of slots waiting for a new path
  uint32_t cnt[STAT_COUNT];  // the wave's event counters (lane 0 adds per batch)
  unsigned long long dead;   // queues this wave found empty (lane 0's dequeue skips them)
  // the wave's path cursor into the global work queues: next, end, q | home << 8 | exhausted << 16
  // (LDS, not SGPRs: only the regeneration code reads it, and the kernel has no scalar
  // registers to spare)
  uint32_t cur[3];
  // in-launch output (LaunchParams::frame_done): the last batch's ended paths, not yet
  // counted: ln stack entries [pend & 0xFF, + pend >> 8), each slot's meta holding its
  // pixel (image_id)
  uint32_t pend;
};
constexpr uint32_t kCurExhausted = 1u << 16;

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint32_t normal_code(V3 n) {
  return n.x > 0.f ? 1u : n.x < 0.f ? 2u : n.y > 0.f ? 3u : n.y < 0.f ? 4u : n.z > 0.f ? 5u : n.z < 0.f ? 6u : 0u;
}
__device__ __forceinline__ V3 normal_of(uint32_t c) {
  const float s = (c & 1u) ? 1.0f : -1.0f;
  return c == 0u ? mk3(0, 0, 0) : c <= 2u ? mk3(s, 0, 0) : c <= 4u ? mk3(0, s, 0) : mk3(0, 0, s);
}

template <class Pool>
__device__ __forceinline__ void store_full(Pool& S, float4* __restrict__ gT, uint32_t s,
                                           const PathState& ps, const Isect& is, uint32_t nseg,
                                           uint32_t wword) {
  S.a[s] = make_float4(ps.o.x, ps.o.y, ps.o.z, 0.0f);
  S.b[s] = make_float4(ps.d.x, ps.d.y, ps.d.z, is.dist);
  S.c[s] = make_uint4(ps.rng.v0, ps.rng.v1, ps.rng.v2, ps.rng.v3);
  S.e[s] = make_uint2(ps.rng.v4, ps.rng.d);
  S.meta[s] = normal_code(is.normal) | (is.inside ? 8u : 0u) | (nseg << 4);
  gstore4(gT + s, make_float4(ps.T.x, ps.T.y, ps.T.z, __uint_as_float(wword)));
}
template <class Pool>
__device__ __forceinline__ void load_full(const Pool& S, const float4* __restrict__ gT, uint32_t s,
                                          PathState& ps, Isect& is, uint32_t& nseg, float& t) {
  const float4 f = gload4(gT + s);
  const float4 a = S.a[s], b = S.b[s];
  const uint4 c = S.c[s];
  const uint2 e = S.e[s];
  const uint32_t meta = S.meta[s];
  ps.o = mk3(a.x, a.y, a.z);
  t = a.w;
  ps.d = mk3(b.x, b.y, b.z);
  is.dist = b.w;
  ps.T = mk3(f.x, f.y, f.z);
  ps.rng = Rng{c.x, c.y, c.z, c.w, e.x, e.y};
  ps.image_id = __float_as_uint(f.w);
  is.normal = normal_of(meta & 7u);
  is.inside = (meta & 8u) != 0u;
  nseg = meta >> 4;
}
template <class Pool>
__device__ __forceinline__ void store_track(Pool& S, uint32_t s, float t, const Rng& rng) {
  S.a[s].w = t;
  S.c[s] = make_uint4(rng.v0, rng.v1, rng.v2, rng.v3);
  S.e[s] = make_uint2(rng.v4, rng.d);
}
// Track state of a ready path: o, t, d, max_t, rng.
template <class Pool>
__device__ __forceinline__ void load_track(const Pool& S, uint32_t s, V3& o, V3& d, Rng& rng, float& t,
                                           float& max_t) {
  const float4 a = S.a[s], b = S.b[s];
  const uint4 c = S.c[s];
  const uint2 e = S.e[s];
  o = mk3(a.x, a.y, a.z);
  t = a.w;
  d = mk3(b.x, b.y, b.z);
  max_t = b.w;
  rng = Rng{c.x, c.y, c.z, c.w, e.x, e.y};
}

// The launch parameters as seen from code that runs rarely (the drain): the
// LDS address goes through an empty asm each time, so the compiler cannot
// hoist loads of L's fields out of the main loop and hold them in registers
// across the track loop (the dense kernel has no VGPR to spare at 5 waves).
typedef __attribute__((address_space(3))) const LaunchParams LdsParams;
__device__ __forceinline__ const LaunchParams& fresh(const LaunchParams& L) {
  LdsParams* p = (LdsParams*)&L;
  asm volatile("" : "+v"(p));
  return *(const LaunchParams*)p;
}

enum : uint32_t { K_BOUNDARY = 0, K_COLLIDE = 1, K_NEW = 2, K_NONE = 3 };

// The batch's escapes, combined per pixel before the framebuffer atomics
// (atomicVectorAdd, Utilities.cuh:15-22, once per escape in the reference).
// The framebuffer adds are performed at the memory side (the XCDs' L2s are not
// coherent), up to three float adds and the w swap per escape; with the units'
// samples innermost (unit_to_path) the escapes of one batch mostly share a few
// pixels.  Each escaping lane finds its pixel's leader (the lowest lane with
// that pixel: one ballot per distinct pixel), the others add their T into the
// leader's freed slot in LDS (ds_add_f32; the path has ended, its slot goes to
// the new-path stack and no later part of this batch touches it), and each
// leader issues one splat of its pixel's sum.  Only the order of the fp32
// additions changes, so the per-pixel bound of DESIGN.md §4 holds: a pixel's
// n contributions are still summed once each, in some order.  With no pixel
// escaped to twice the batch splats per lane as before.
template <bool kCombine, class Pool>
__device__ __forceinline__ void splat_wave(Pool& S, const LaunchParams& L, const PathState& ps, bool esc,
                                           uint32_t s, uint32_t lane) {
#if defined(CVR_DIAG_NO_SPLAT)  // diagnostic timing builds only (wrong images): no framebuffer writes
  (void)S; (void)L; (void)ps; (void)esc; (void)s; (void)lane;
  return;
#endif
  unsigned long long rest = __ballot(esc);
  if (rest == 0ull) return;
  if (!kCombine || !(fresh(L).wflags & kSplatCombine)) {  // (CVR_OPT_SAMPLE_ORDER 0: few shared pixels)
    if (esc) splat(L, ps);
    return;
  }
  uint32_t leader = lane;
  bool multi = false;  // wave-uniform: some pixel gets two or more escapes
  while (rest != 0ull) {
    const uint32_t l0 = (uint32_t)__builtin_ctzll(rest);
    const uint32_t id0 = __builtin_amdgcn_readlane(ps.image_id, l0);
    const unsigned long long g = __ballot(esc && ps.image_id == id0);
    if (esc && ps.image_id == id0) leader = l0;
    multi |= (g & (g - 1ull)) != 0ull;
    rest &= ~g;
  }
  if (!multi) {
    if (esc) splat(L, ps);
    return;
  }
  const uint32_t sl = (uint32_t)__shfl((int)s, (int)leader);  // the leader's slot
  float* acc = reinterpret_cast<float*>(&S.a[sl]);
  const bool lead = esc && leader == lane;
  if (lead) {
    acc[0] = ps.T.x;
    acc[1] = ps.T.y;
    acc[2] = ps.T.z;
  }
  // one wave: its LDS instructions are performed in order; the wait keeps the
  // compiler from moving the adds above the leaders' stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (esc && !lead) {
    __hip_atomic_fetch_add(acc + 0, ps.T.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(acc + 1, ps.T.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(acc + 2, ps.T.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lead) {
    PathState q{};
    q.image_id = ps.image_id;
    q.T = mk3(acc[0], acc[1], acc[2]);
    splat(L, q);
  }
}

// The wave's path cursor into the global work queues (as k_persistent).
// Debug records (LaunchParams::rec): a path's final state when it ends, in
// the oracle's per-path record layout (cvr_kernels.h PathRecord; steps and
// density counts are per lane here, so they stay 0).
template <int kSlots, int kWpg>
__device__ __forceinline__ uint32_t* rec_pids(const LaunchParams& L, uint32_t gw) {
  // the path-id array (grid * slots u32, grid in waves) sits just below the records
  return reinterpret_cast<uint32_t*>(L.rec) - (size_t)gridDim.x * kWpg * kSlots + (size_t)gw * kSlots;
}
template <int kSlots, int kWpg>
__device__ __forceinline__ void record_end(const LaunchParams& L, uint32_t gw, uint32_t s, const PathState& ps,
                                           uint32_t flags, uint32_t nseg) {
  const uint32_t pid = rec_pids<kSlots, kWpg>(L, gw)[s];
  PathRecord r = {};
  r.image_id = ps.image_id;
  r.flags = flags;
  r.T[0] = ps.T.x;
  r.T[1] = ps.T.y;
  r.T[2] = ps.T.z;
  r.n_segments = nseg;
  static_cast<PathRecord*>(L.rec)[pid - L.path_first] = r;
}



// ---- in-launch output (cvr_render_frame) -----------------------------------
// getImage (CudaVolPath.cpp:339-347, ImageBufferTransfer.cu:61-78: Scale, then
// the D->H copy) without a copy after the launch: each wave counts its ended
// paths per 8x8 tile block, and kFrameFlushers flusher waves store a block's
// normalised pixels into the pinned host image as soon as all 64 * samples of
// its paths have ended, while the launch goes on.
//
// Ordering: the framebuffer atomics (splat) and the block counts are agent-
// scope atomics, performed at the memory side.  A batch's ended paths are
// counted at the next batch (or at the wave's exit): it first waits for all of
// the wave's outstanding memory operations, so a full count means every splat
// of the block has been performed, and the flusher reads the pixels with
// atomics too.  Most of a batch's ended paths lie in lane 0's block (the wave's
// current chunk): their count is one atomic, issued at the end of the counting
// batch beside that batch's splats, so that no memory wait of the batch's own
// loads waits for it; the other lanes add 1 each at once.
constexpr unsigned kWaitVm0 = 0x0F70;   // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)
constexpr uint32_t kPendAgg = 0x80000000u;  // S.pend holds kPendAgg | block << 7 | count

template <class Pool>
__device__ __forceinline__ uint32_t count_ended(const Pool& S, const LaunchParams& L, uint32_t pend,
                                                uint32_t lane) {
#if defined(CVR_DIAG_NO_COUNT)  // diagnostic timing builds only: no block counts (flushers must give up)
  (void)S; (void)L; (void)pend; (void)lane;
  return 0u;
#endif
  const uint32_t base = pend & 0xFFu, n = pend >> 8;
#if !defined(CVR_DIAG_NO_COUNT_WAIT)  // diagnostic timing builds only (unordered counts)
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
#endif
  uint32_t blk = 0;
  if (lane < n) blk = tile_block_of(fresh(L), S.meta[S.ln[base + lane]]);
  const uint32_t b0 = __builtin_amdgcn_readfirstlane(blk);
  const unsigned long long same = __ballot(lane < n && blk == b0);
  // a second block (the wave's previous chunk) with one atomic too, the rest one per lane
  const bool rest = lane < n && blk != b0;
  const unsigned long long rm = __ballot(rest);
  if (rm != 0ull) {
    const uint32_t first = (uint32_t)__builtin_ctzll(rm);
    const uint32_t b1 = __builtin_amdgcn_readlane(blk, first);
    const unsigned long long s1 = __ballot(rest && blk == b1);
    if (lane == first || (rest && blk != b1))
      __hip_atomic_fetch_add(gmem(fresh(L).frame_done + kDoneStride * blk), lane == first ? (unsigned int)__popcll(s1) : 1u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return kPendAgg | b0 << 7 | (uint32_t)__popcll(same);
}
__device__ __forceinline__ void add_counted(const LaunchParams& L, uint32_t agg) {
#if defined(CVR_DIAG_NO_COUNT)
  (void)L; (void)agg;
  return;
#endif
  __hip_atomic_fetch_add(gmem(fresh(L).frame_done + kDoneStride * ((agg & ~kPendAgg) >> 7)), agg & 0x7Fu,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Up to 8 tile blocks' pixels (one per lane in each block), normalised, into the
// host image: all reads first (24 atomics in flight per lane), then the stores.
__device__ __forceinline__ void store_blocks(const LaunchParams& L, const FrameFlush& F, const uint32_t (&b)[8], uint32_t nb,
                                             uint32_t lane) {
  float v[8][3];
  size_t pix[8];
#pragma unroll
  for (uint32_t k = 0; k < 8u; ++k) {
    if (k < nb) {
      const uint32_t by = fastdiv(b[k], L.div_blocks_x), bx = b[k] - by * L.blocks_x;
      const uint32_t px = bx * 8u + (lane & 7u), py = by * 8u + (lane >> 3);
      pix[k] = (size_t)py * L.tile_w + px;
      gptr_t<float> src = gmem(reinterpret_cast<float*>(L.out + pix[k]));
#pragma unroll
      for (int c = 0; c < 3; ++c) v[k][c] = __hip_atomic_fetch_add(src + c, 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < 8u; ++k) {
    if (k < nb) {
      const float x = v[k][0], y = v[k][1], z = v[k][2];
      // w: splat's plain store of 1 (Utilities.cuh:21) may still sit in another XCD's L2.
      // It is 1 exactly when some path escaped to the pixel, and then the rgb sum is not
      // zero (or NaN): an escaping path's throughput has a positive component, since
      // roulette ends every path whose components are all zero (p = 0 < xi).
      const float w = (x != 0.0f || y != 0.0f || z != 0.0f) ? 1.0f : 0.0f;
      // the tile is the host image (cvr_render_frame: host_w = tile_w)
      float4* dst = F.host + pix[k];
      __builtin_nontemporal_store(x / F.scale, &dst->x);
      __builtin_nontemporal_store(y / F.scale, &dst->y);
      __builtin_nontemporal_store(z / F.scale, &dst->z);
      __builtin_nontemporal_store(w / F.scale, &dst->w);
    }
  }
}

// Flusher wave f follows queues f, f + 8, ..., f + 56 through their blocks in
// dequeue order: lane l looks at block cur + (l >> 3) of queue f + 8 (l & 7), so a
// pass polls a window of 8 blocks per queue and stores every block in it whose
// count is full (a block that ends late does not hold up the ones behind it);
// stored blocks are marked in their count (kFlushed) and each queue's cursor
// moves past its leading stored blocks.  A flusher that sees no block finish for
// a second gives up (status word kFrameFlushers): the host then normalises and
// copies the image after the launch.
constexpr unsigned long long kFlushPatience = 100000000ull;  // s_memrealtime ticks (100 MHz)
constexpr unsigned int kFlushed = 0x80000000u;
__device__ void frame_flusher(const LaunchParams& L, uint32_t f, uint32_t lane) {
  const FrameFlush F = *frame_header(L.frame_done);
  if (F.give_up) {  // test mode: exercise the host's fallback copy
    if (lane == 0) __hip_atomic_store(F.status + kFrameFlushers, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const uint32_t quota = 64u * L.samples, qi = lane & 7u, off = lane >> 3, q = f + kFrameFlushers * qi;
  uint32_t cur = 0, end = 0, stored = 0;  // this lane's queue (all 8 lanes of a queue agree)
  if (q < L.n_queues) {
    cur = queue_blocks_begin(L, q);
    end = queue_blocks_begin(L, q + 1u);
  }
  unsigned long long last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (__ballot(cur < end) == 0ull) break;
    const bool mine = cur + off < end;
    uint32_t tb = 0, v = 0;
    if (mine) {
      tb = launch_block_tile(L, cur + off);
      v = __hip_atomic_fetch_add(gmem(L.frame_done + kDoneStride * tb), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool ready = mine && v < kFlushed && v >= quota;
    unsigned long long rm = __ballot(ready);
    const unsigned long long settled = __ballot(mine && v >= quota);  // stored before or now
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const bool any_ready = rm != 0ull;
    while (rm != 0ull) {  // eight blocks per store_blocks call
      uint32_t bsel[8], nb = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8u; ++k) {
        if (rm != 0ull) {
          bsel[k] = __builtin_amdgcn_readlane(tb, (uint32_t)__builtin_ctzll(rm));
          rm &= rm - 1ull;
          ++nb;
        }
      }
      store_blocks(L, F, bsel, nb, lane);
      stored += nb;
    }
    if (ready) __hip_atomic_fetch_or(gmem(L.frame_done + kDoneStride * tb), kFlushed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // each queue's cursor moves past its leading settled blocks (window bits qi, qi + 8, ...)
    uint32_t lead = 0;
#pragma unroll
    for (uint32_t o = 0; o < 8u; ++o)
      if (lead == o && ((settled >> (qi + 8u * o)) & 1ull)) ++lead;
    cur += lead;
    if (any_ready) {
      last = now;
    } else if (__ballot(lead != 0u) == 0ull) {
      if (now - last > kFlushPatience) {
        if (lane == 0) __hip_atomic_store(F.status + kFrameFlushers, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(32);
    }
  }
  if (lane == 0) __hip_atomic_store(F.status + f, stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- the launch's drain: one path's Woodcock points across K lanes -----------
// Once every queue is exhausted a wave's pool only drains: fewer paths than lanes
// are left, and the last ones run one segment at a time, each Woodcock group a
// dependent brick-word load (round-6 tail stamps, tools/tail_wpool.py: half of a
// draining wave's time is its track loop).  The points of a segment depend on
// nothing but its RNG stream, so with few paths left each ready path gets K
// lanes (one group of a DPP row): lane p of the group takes the path's draws
// 2p + 1 and 2p + 2 (every lane steps the XORWOW sequence up to its own pair),
// the distances follow the sequential chain t_p = fma(-log xi_p, inv_sigma,
// t_{p-1}) in order (one row shift per point), and all K brick words (and the
// cells the bounds do not settle) load at once.  The first point of the group
// that ends the segment (past max_t, or a real collision) is found by a ballot;
// the points after it are dropped, as in the two-point lookahead, and the path's
// t and RNG are that point's (its lane stores them into the slot).  The same
// candidates in the same order: the same results, steps and fetch counts as one
// point at a time (Utilities.cuh:147-152, tests/test_gpu_records.py).  On exit
// lane 0 of each group holds its path's finished segment, filed by the next
// swap.  Groups past `ngroups` repeat group 0's path and write nothing.
template <int K, int kSlots, int kEm, class Pool, class EmWords>
__device__ __forceinline__ void wide_track(Pool& S, const EmWords& em, const MediumParams& m, uint32_t lane,
                                           uint32_t ready_head,
                                           uint32_t ngroups, int& slot, int& fst, V3& o, V3& d, Rng& rng,
                                           float& t, float& max_t, uint32_t& c_steps, uint32_t& c_fetch) {
  static_assert(K >= 2 && K <= 16 && (K & (K - 1)) == 0, "a group lies within one 16-lane DPP row");
  constexpr uint32_t kGroupMask = K == 32 ? 0xFFFFFFFFu : (1u << K) - 1u;
  // (through an empty asm: lane / K and lane % K are loop-invariant, and hoisted to the
  // prologue they would hold two VGPRs across the track loop)
  uint32_t ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t g = ln / K, p = ln % K;
  const bool real = g < ngroups;
  const uint32_t r = ready_head + (real ? g : 0u);
  const uint32_t s = S.ready[r >= (uint32_t)kSlots ? r - kSlots : r];
  V3 go, gd;
  Rng gr;
  float gt, gmax;
  load_track(S, s, go, gd, gr, gt, gmax);
  int res = 0;        // the group's segment result once it ended: 1 past max_t, 2 accepted
  bool open = real;   // group-uniform: the segment has not ended
  for (;;) {
    // lane p: draws 2p + 1, 2p + 2 of the group's stream (divergent loop, K rounds)
    Rng lr = gr;
    float xi = 0.0f, xt = 0.0f;
    for (uint32_t i = 0; i <= p; ++i) {
      xi = rng_float(lr);
      xt = rng_float(lr);
    }
    const float a = -det_logf_normal(__builtin_fmaxf(xi, CVR_EPSILON_F));
    // t_p = fma(a_p, inv_sigma, t_{p-1}) in order: woodcock_advance's chain, one row shift per point
    float tp = det_fmaf(a, m.inv_sigma, gt);
#pragma unroll
    for (int j = 1; j < K; ++j) {
      const float prev = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(tp), 0x111 /* row_shr:1 */,
                                                                    0xF, 0xF, false));
      const float tn = det_fmaf(a, m.inv_sigma, prev);
      tp = p == (uint32_t)j ? tn : tp;
    }
    WoodcockPoint P;
    if constexpr (kEm != 0)
      P = woodcock_point_em<kEm>(m, go, gd, tp, em);
    else
      P = woodcock_point(m, go, gd, tp);
    int rr = 0;
    bool fetched = false;
    if (!(tp <= gmax)) {
      rr = 1;
    } else if (!(P.qb < xt)) {
      fetched = true;
      const float rho = m.scale * woodcock_density(m, P);
      if (!(rho * m.inv_sigma < xt)) rr = 2;
    }
    const unsigned long long me = __ballot(rr != 0), m1 = __ballot(rr == 1);
    const uint32_t gb = (uint32_t)(me >> (g * K)) & kGroupMask;
    const uint32_t end = gb ? (uint32_t)__builtin_ctz(gb) : (uint32_t)K;
    if (open) {
      c_fetch += (fetched && p <= end) ? 1u : 0u;
      if (p == 0) c_steps += end < (uint32_t)K ? end + 1u : (uint32_t)K;
      // the group's new track state: the ending point's, or the last point's
      if (p == (end < (uint32_t)K ? end : (uint32_t)K - 1u)) store_track(S, s, tp, lr);
      if (end < (uint32_t)K) {
        res = ((m1 >> (g * K + end)) & 1ull) ? 1 : 2;
        open = false;
      }
    }
    if (__ballot(open) == 0ull) break;
    if (open) {  // the next K points from the state just stored (one wave: LDS in order)
      V3 o2, d2;
      load_track(S, s, o2, d2, gr, gt, gmax);
    }
  }
  if (real && p == 0) {
    slot = (int)s;
    fst = res;
    load_track(S, s, o, d, rng, t, max_t);
  }
}

}  // namespace

// kMed: the medium layout the instance is compiled for (kMedDense any dense medium,
// kMedSparse leaves + brick words, kMedDenseFull a dense medium with density cells
// and brick bounds, the defaults: its null checks fold away, C2 -0.6%, C3 -1.8%;
// kMedDenseFullUniform the same with a uniform albedo, MediumParams::albedo_uniform,
// whose check would otherwise cost the non-uniform instance 1.5% on C2).
// kFlush: the in-launch output instance (cvr_render_frame, CVR_OPT_FRAME_FLUSH);
// the other instances carry none of its code.
enum : int { kMedDense = 0, kMedSparse = 1, kMedDenseFull = 2, kMedDenseFullUniform = 3 };
#if CVR_WPOOL_TAILSTAMP
constexpr uint32_t kTailWaves = 16384;
__device__ unsigned long long g_tail[8 * kTailWaves];
#endif
// kMedMK (or-ed into kMed): naiveMK's walk (NaiveVolPTmk_kernel.cuh:20-151) on the wave
// pool, round 5: a new path runs d_init (camera ray on the (iteration, pixel, 0) stream,
// AABB, the GGX sample at the box, Q12) and every segment starts as d_extend does, with
// the RNG re-seeded from (iteration, pixel, depth) and three unused draws; the slot's
// event-only word holds the path id (iteration and pixel) instead of the pixel.
constexpr int kMedMK = 4;
// kMedCount (or-ed into kMed, sparse media only): the counting instance of
// CVR_OPT_COUNT_WORDS, which also counts the brick words its Woodcock points load
// (the empty-region mask skips the rest), so that the launch's algorithmic bytes are
// exact; the benchmarked instances carry no counter.
constexpr int kMedCount = 8;
template <bool kScatterEps, int kWaves, int kMedMk, bool kRecord, bool kFlush>
__global__ __launch_bounds__(64 * wpg_of(kMedMk, kWaves), kWaves) void k_wpool(MediumParams mk, LaunchParams Lk) {
  constexpr bool kMK = (kMedMk & kMedMK) != 0;
  constexpr bool kCountWords = (kMedMk & kMedCount) != 0;
  constexpr int kMed = kMedMk & 3;
  static_assert(!kMK || (kScatterEps && !kRecord && !kFlush), "naiveMK: scatter -eps, no records / in-launch output");
  constexpr bool kSparse = kMed == kMedSparse;
  // Sparse media defer their cell fetches to the end of the track iteration
  // (the lookahead below): C5 -3.0%; the dense instances lose 5-8% with it.
  constexpr bool kLookDefer = kSparse && CVR_WPOOL_SPARSE_DEFER;
  constexpr bool kFetchList = CVR_WPOOL_FETCH_LIST && !kMK && (kMed == kMedDenseFull || kMed == kMedDenseFullUniform);
  // (dense media: +7% C2, +6% C3 with a 16-word mask)
  constexpr int kEm = kSparse && CVR_WPOOL_EMASK ? kEmaskWords : 0;
  // waves per workgroup, each with a pool of its own (kWpgSparse on sparse media)
  constexpr int kWpg = wpg_of(kMedMk, kWaves);
  constexpr int kSlots = PoolSize<kWaves, 4 * kEm, kWpg>::value;
  if constexpr (kFlush && kWpg == 1) {
    if (Lk.frame_done != nullptr && blockIdx.x < kFrameFlushers) {
      frame_flusher(Lk, blockIdx.x, threadIdx.x);
      return;
    }
  }
  // the wave's index within its workgroup and within the launch (pool_T rows,
  // records, home sub-queue): one-wave workgroups number as before
  const uint32_t wv = kWpg > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;
  const uint32_t gw = blockIdx.x * (uint32_t)kWpg + wv;
  // Dense instances see the sparse pointers as constant null, so the sparse
  // branches of the walk code fold away and take no scalar registers.
  MediumParams m = mk;
  if constexpr (!kSparse) {
    m.leaves = nullptr;
    m.leaf_density = nullptr;
    m.leaf_albedo = nullptr;
    m.sbounds = nullptr;
    if constexpr (kMed == kMedDenseFull || kMed == kMedDenseFullUniform) {
      __builtin_assume(m.cells != nullptr);
      __builtin_assume(m.bounds != nullptr);
      m.albedo_uniform = kMed == kMedDenseFullUniform ? 1u : 0u;
    }
  } else {
    // and sparse instances see the dense pointers as constant null (a sparse medium
    // has leaves, brick words and no dense grids)
    m.density = nullptr;
    m.albedo = nullptr;
    m.bounds = nullptr;
    __builtin_assume(m.leaves != nullptr);
    __builtin_assume(m.sbounds != nullptr);
    m.albedo_uniform = 0u;
  }
#if CVR_WPOOL_TAILSTAMP
  const unsigned long long ts_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long ts_ex = 0, ts_ev = 0, ts_a = 0;
  uint32_t ts_live = 0, ts_batches = 0, ts_trk = 0, ts_steps0 = 0, ts_seg0 = 0;
#endif
  static_assert(kWpg * sizeof(WavePool<kSlots>) + 4 * kEm + sizeof(LaunchParams) <=
                    (size_t)PoolSize<kWaves, 0, kWpg>::kBudget,
                "wave pools exceed the LDS budget of kWaves waves per SIMD");
  static_assert(kSlots <= 256, "the pool's rings and stacks hold slot indices as uint8_t");
  static_assert(!kFetchList || kSlots <= 128, "fetch-pending ring entries carry bit 7");
  __shared__ WavePool<kSlots> Sw[kWpg];
  WavePool<kSlots>& S = Sw[wv];
  // the empty-region mask (sparse media), one copy per workgroup
  __shared__ uint32_t EM[kEm ? kEm : 1];
  // The launch parameters live in LDS: only the event code reads them, and
  // keeping them in SGPRs for the whole kernel spills the step loop's
  // scalars (v_readlane reloads in every Woodcock step).
  __shared__ LaunchParams L;
  const uint32_t lane = kWpg > 1 ? threadIdx.x & 63u : threadIdx.x;
  if (threadIdx.x == 0) L = Lk;
  if constexpr (kEm != 0) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)kEm; i += 64u * kWpg) EM[i] = m.emask ? m.emask[i] : ~0u;
  }
  __syncthreads();
  // (a multi-wave workgroup's flushers take part in the barrier above)
  if constexpr (kFlush && kWpg > 1) {
    if (Lk.frame_done != nullptr && gw < kFrameFlushers) {
      frame_flusher(Lk, gw, lane);
      return;
    }
  }
  // Counters.  Event counts are popcounts of ballots that lane 0 adds to the
  // pool's LDS counters once per batch (no per-lane registers, no SGPRs, live
  // across the track loop); the track loop counts steps and fetches per lane.
  uint32_t c_steps = 0, c_fetch = 0;
  uint32_t c_words = 0;  // kCountWords: brick words loaded
  if (lane < (uint32_t)STAT_COUNT) S.cnt[lane] = 0u;
  if (lane == 0) {
    S.dead = 0ull;
    S.pend = 0u;
  }
  uint32_t n_over = 0;  // wave-uniform: segments whose last Woodcock step passed max_t
  // home queue: the XCD's band, and within it sub-queue (the wave's number among
  // its XCD's waves) mod sub (workgroups are dealt round-robin over the 8 XCDs)
  if (lane == 0) {
    S.cur[0] = S.cur[1] = 0u;
    S.cur[2] = (((__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u) % (L.n_queues / L.sub)) * L.sub +
                ((blockIdx.x >> 3) * (uint32_t)kWpg + wv) % L.sub)
               << 8;
  }
  const uint32_t batch = L.batch;  // TRACK: swap finished segments once this many lanes are idle
  // wave-uniform list state
  uint32_t ready_head = 0, n_ready = 0, n_lb = 0, n_lc = 0;
  uint32_t n_ln = kSlots;  // slots waiting for a new path (all of them at the start)
  for (uint32_t i = lane; i < (uint32_t)kSlots; i += 64u) S.ln[i] = (uint8_t)i;

  for (;;) {
    // ================================================= TRACK ==============
    __builtin_amdgcn_s_setprio(kPrioTrack);
    // The track state is fresh per outer iteration and parked in the pool
    // before the event code runs, so nothing of it is live across that code
    // (keeps the step loop free of spills).
    int slot = -1;      // pool slot of the lane's path, -1 = none
    // woodcock_step_core result of the lane's segment: 0 still tracking,
    // 2 real collision, 1/3 boundary (1: the last step evaluated no
    // density); filed at the next swap.  The track loop sets 2 for every
    // accepted point; filing turns an acceptance at t == max_t into 3 (the
    // reference scatters iff t < max_t), so the step carries no compare for it.
    // 4 (sparse only): cell fetch pending, resolved to 0 or 2 before the next
    // swap check.
    int fst = 0;
    V3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
    Rng rng{0, 0, 0, 0, 0, 0};
    float t = 0.0f, max_t = 0.0f;
    const float4* pcp = nullptr;  // kLookDefer: the pending fetch's cell and test value
    float pxt = 0.0f;
    if constexpr (CVR_WPOOL_WIDE != 0) {
      // the drain (every queue exhausted) with at most 64 / K paths ready: K lanes per path
      // (wide_track); the segments end there and the first swap below files them
      if (n_ready != 0u && n_ready <= 64u / CVR_WPOOL_WIDE && (S.cur[2] & kCurExhausted)) {
        wide_track<CVR_WPOOL_WIDE, kSlots, kEm>(S, EM, m, lane, ready_head, n_ready, slot, fst, o, d, rng, t, max_t,
                                                c_steps, c_fetch);
        ready_head += n_ready;
        if (ready_head >= (uint32_t)kSlots) ready_head -= kSlots;
        n_ready = 0;
      }
    }
    for (;;) {
      const unsigned long long trk = (__ballot(slot >= 0) & __ballot(fst == 0));
      const uint32_t n_trk = (uint32_t)__popcll(trk);
      // ---- swap: file finished segments, pull track-ready paths ----------
      if (64u - n_trk >= batch || n_trk == 0u) {
        if (fst == 2 && !(t < max_t)) fst = 3;
        if (fst != 0) store_track(S, (uint32_t)slot, t, rng);
        const unsigned long long mc = __ballot(fst == 2), mb = __ballot(fst & 1);
        if (fst == 2) S.lc[n_lc + lane_rank(mc)] = (uint8_t)slot;
        if (fst & 1) S.lb[n_lb + lane_rank(mb)] = (uint8_t)slot;
        n_lc += (uint32_t)__popcll(mc);
        n_lb += (uint32_t)__popcll(mb);
        n_over += (uint32_t)__popcll(__ballot(fst == 1));
        if constexpr (kFetchList) {  // fetch pending: back to the ready ring, marked
          const unsigned long long mf = __ballot(fst == 4);
          if (fst == 4) S.ready[(ready_head + n_ready + lane_rank(mf)) % kSlots] = (uint8_t)(slot | 0x80);
          n_ready += (uint32_t)__popcll(mf);
        }
        if (fst != 0) {
          slot = -1;
          fst = 0;
        }
        const unsigned long long idle = __ballot(slot < 0);
        const uint32_t k = min((uint32_t)__popcll(idle), n_ready), rank = lane_rank(idle);
        bool pend = false;
        if (slot < 0 && rank < k) {
          const uint32_t r = ready_head + rank;
          uint32_t s = S.ready[r >= (uint32_t)kSlots ? r - kSlots : r];
          if constexpr (kFetchList) {
            pend = (s & 0x80u) != 0u;
            s &= 0x7Fu;
          }
          slot = (int)s;
          load_track(S, s, o, d, rng, t, max_t);
        }
        ready_head += k;
        if (ready_head >= (uint32_t)kSlots) ready_head -= kSlots;
        n_ready -= k;
        if constexpr (kFetchList) {
          if (pend) {  // the pending point's cell, fetched by every lane that pulled one
            ++c_fetch;
            WoodcockPoint P;
            woodcock_coords(m, o, d, t, P);
            const uint32_t x1 = (uint32_t)P.cx, y1 = (uint32_t)P.cy, z1 = (uint32_t)P.cz;
            P.cp = m.cells + 2 * (__umul24(z1, m.rxy) + __umul24(y1, m.rx) + x1);
            const float xt = det_fmaf((float)(rng.v4 + rng.d), 2.3283064e-10f, 1.1641532e-10f);  // its test draw
            const float rho = m.scale * woodcock_density(m, P);
            fst = !(rho * m.inv_sigma < xt) ? 2 : 0;
          }
        }
      }
      const uint32_t n_act = (uint32_t)__popcll((__ballot(slot >= 0) & __ballot(fst == 0)));
      const uint32_t n_fin = (uint32_t)__popcll(__ballot(fst != 0 && (!kFetchList || fst != 4)));
      // EVENT next: a full wave of waiting events, slots never filled, or
      // nothing left to track.  Park: tracking lanes return (t, rng) to the
      // pool, finished lanes are filed.  (Once the queues are empty n_ln is a
      // stand-in that lowers this threshold: see the end of the event batch.)
      if (n_lb + n_lc + n_ln + n_fin >= 64u || (n_act == 0u && n_ready == 0u)) {
        if (fst == 2 && !(t < max_t)) fst = 3;
        if (slot >= 0) store_track(S, (uint32_t)slot, t, rng);
        const unsigned long long mr = (__ballot(slot >= 0) & __ballot(fst == 0 || (kFetchList && fst == 4)));
        const unsigned long long mc = __ballot(fst == 2), mb = __ballot(fst & 1);
        if (slot >= 0 && (fst == 0 || (kFetchList && fst == 4)))
          S.ready[(ready_head + n_ready + lane_rank(mr)) % kSlots] = (uint8_t)(slot | (fst == 4 ? 0x80 : 0));
        if (fst == 2) S.lc[n_lc + lane_rank(mc)] = (uint8_t)slot;
        if (fst & 1) S.lb[n_lb + lane_rank(mb)] = (uint8_t)slot;
        n_over += (uint32_t)__popcll(__ballot(fst == 1));
        n_ready += (uint32_t)__popcll(mr);
        n_lc += (uint32_t)__popcll(mc);
        n_lb += (uint32_t)__popcll(mb);
        break;
      }
      // ---- Woodcock steps (Utilities.cuh:147-152), two points at a time ----
      // woodcock_step_core for two consecutive tentative points: a lane takes
      // all four draws and loads both brick words before it tests either, so
      // the wave waits for one brick-word latency per two steps, and the two
      // points' arithmetic interleaves.  The points after the one that ends
      // the segment (t > max_t or a real collision) are dropped: t is that
      // point's, and the RNG goes back to the state after its two draws.
      // XORWOW shifts its five words by one per draw, so that state is two
      // saved words plus three of the current ones.  A segment that ends
      // past max_t has drawn its test value too, as in the one-point step
      // (the boundary event takes that draw back, rng_undo).  Density
      // evaluations are steps minus the segments that ended past max_t
      // (counted when filed), so only steps are counted here.  Measured
      // (profiles/round4/lookahead.md): 2 points -3.5% C2, -3.4% C3, -2.6% C5
      // against one; 3 or 4 points, or loading the undecided points' cells
      // before testing, were slower.  kLookDefer (sparse media): a point the
      // bound does not settle parks its lane (fst 4, later points dropped as
      // for an end) and the lane fetches its cell once after the unrolled
      // groups, so the wave waits for one cell latency per iteration instead
      // of one per group that needs a cell; the parked lanes idle meanwhile.
#pragma unroll
      for (int u = 0; u < CVR_WPOOL_UNROLL / kLook; ++u) {
        if (slot >= 0 && fst == 0) {
          float tk[kLook], xtk[kLook];
          uint32_t sva[kLook], svb[kLook];  // draw-sequence words 2k+2, 2k+3 (S_{k+1}.v0, v1)
          WoodcockPoint Pk[kLook];
          float tt = t;
#pragma unroll
          for (int k = 0; k < kLook; ++k) {
            const float xi = rng_float(rng);
            xtk[k] = rng_float(rng);
            sva[k] = rng.v0;
            svb[k] = rng.v1;
            tt = woodcock_advance(m, xi, tt);
            tk[k] = tt;
          }
#pragma unroll
          for (int k = 0; k < kLook; ++k) {
            if constexpr (kEm != 0)
              Pk[k] = woodcock_point_em<kEm>(m, o, d, tk[k], EM, kCountWords ? &c_words : nullptr);
            else
              Pk[k] = woodcock_point(m, o, d, tk[k]);
          }
          int end = kLook;  // the first point that ends the segment
#pragma unroll
          for (int k = 0; k < kLook; ++k) {
            if (end == kLook) {
              if (!(tk[k] <= max_t)) {
                fst = 1;
                end = k;
              } else if (!(Pk[k].qb < xtk[k])) {
                if constexpr (kLookDefer) {
                  fst = 4;  // cell fetch pending (after the groups); the lane steps no further
                  end = k;
                  pcp = Pk[k].cp;
                  pxt = xtk[k];
                } else if constexpr (kFetchList) {
                  fst = 4;  // cell fetch pending: filed as marked track-ready work at the next swap
                  end = k;
                } else {
                  ++c_fetch;
                  const float rho = m.scale * woodcock_density(m, Pk[k]);
                  if (!(rho * m.inv_sigma < xtk[k])) {
                    fst = 2;
                    end = k;
                  }
                }
              }
            }
          }
          c_steps += end == kLook ? kLook : end + 1;
          t = tk[kLook - 1];
#pragma unroll
          for (int k = 0; k < kLook - 1; ++k)
            if (end == k) t = tk[k];
          if (end < kLook - 1) {
            uint32_t w[2 * kLook + 5];
#pragma unroll
            for (int k = 0; k < kLook - 1; ++k) {
              w[2 * k + 2] = sva[k];
              w[2 * k + 3] = svb[k];
            }
            w[2 * kLook] = rng.v0;
            w[2 * kLook + 1] = rng.v1;
            w[2 * kLook + 2] = rng.v2;
            w[2 * kLook + 3] = rng.v3;
            w[2 * kLook + 4] = rng.v4;
#pragma unroll
            for (int j = 1; j < kLook; ++j) {
              if (end + 1 == j) {
                rng.v0 = w[2 * j];
                rng.v1 = w[2 * j + 1];
                rng.v2 = w[2 * j + 2];
                rng.v3 = w[2 * j + 3];
                rng.v4 = w[2 * j + 4];
              }
            }
            rng.d -= (uint32_t)(2 * (kLook - 1 - end)) * 362437u;
          }
        }
      }
      if constexpr (kLookDefer) {
        if (fst == 4) {
          ++c_fetch;
          WoodcockPoint P;
          woodcock_coords(m, o, d, t, P);
          P.cp = pcp;
          const float rho = m.scale * woodcock_density(m, P);
          fst = !(rho * m.inv_sigma < pxt) ? 2 : 0;
        }
      }
    }
    // no path left (new-path slots only count while the queues have paths)
    if (n_lb + n_lc == 0u && n_ready == 0u && (n_ln == 0u || (S.cur[2] & kCurExhausted))) break;

    // ================================================= EVENT ==============
    __builtin_amdgcn_s_setprio(kPrioEvent);
#if CVR_WPOOL_TAILSTAMP
    if (ts_ex != 0) ts_a = __builtin_amdgcn_s_memrealtime();
#endif
    if constexpr (kFlush) {
      const uint32_t pend = S.pend;  // the last batch's ended paths (in-launch output)
      if (pend != 0u) {
        const uint32_t agg = count_ended(S, L, pend, lane);
        if (lane == 0) S.pend = agg;
      }
    }
    // Event-code view of the medium: its BSDF / box / albedo fields pass
    // through opaque_s per batch, so values derived from them (HG and box
    // constants) are recomputed in the batch instead of being hoisted to the
    // prologue and held in VGPRs across the track loop (4 waves: 127 -> 119
    // VGPRs).
    MediumParams me = m;
    me.g = opaque_s(m.g);
    me.ax = opaque_s(m.ax);
    me.ay = opaque_s(m.ay);
    me.eta = opaque_s(m.eta);
    me.inv_eta = opaque_s(m.inv_eta);
    me.bmin = mk3(opaque_s(m.bmin.x), opaque_s(m.bmin.y), opaque_s(m.bmin.z));
    me.bmax = mk3(opaque_s(m.bmax.x), opaque_s(m.bmax.y), opaque_s(m.bmax.z));
    me.albedo_bg = mk3(opaque_s(m.albedo_bg.x), opaque_s(m.albedo_bg.y), opaque_s(m.albedo_bg.z));
    if constexpr (kMed == kMedDense)  // a run-time flag only in the generic instance
      me.albedo_uniform = __float_as_uint(opaque_s(__uint_as_float(m.albedo_uniform)));
    // One batch of up to 64 items, [boundary | collision | new].  New items
    // are regenerated first: a camera path's first segment is an AABB test
    // and, when it hits the box from outside, a boundary event, which then
    // runs in this batch's boundary part together with the filed boundary
    // events.  Then the boundary part, the collision part (one kind of code
    // each on consecutive lanes), and the AABB test of every survivor.  No
    // item loops: a path that dies (roulette, escape, truncation) files its
    // slot in the new list for a later batch.
    {
// Kind-major batches: once 48 boundary (else 24 collision) events wait, the
// batch runs that kind alone, so its code runs on more lanes; otherwise
// [boundary | collision | new] as they come (C2: -1.5% at 40/40; 48/24 is
// a further -1.8% on C2 and -1.0% on C3, profiles/round2/ab_kindmin_*.log).
// New paths fill a
// boundary batch (a camera path's first event is its GGX entry into the box,
// the same code) but not a collision batch unless a whole wave of them waits:
// beside collisions they would run the whole boundary code on a few lanes
// (C2 -2.7%, C3 -3%).
#ifndef CVR_WPOOL_KIND_MIN
#define CVR_WPOOL_KIND_MIN 48
#endif
#ifndef CVR_WPOOL_KIND_MIN_C
#define CVR_WPOOL_KIND_MIN_C 24
#endif
      uint32_t tb, tc, tn;
      if (n_lb >= (uint32_t)CVR_WPOOL_KIND_MIN) {
        tb = min(n_lb, 64u);
        tc = 0;
        tn = min(n_ln, 64u - tb);
      } else if (n_lc >= (uint32_t)CVR_WPOOL_KIND_MIN_C) {
        tb = 0;
        tc = min(n_lc, 64u);
        tn = n_ln < 64u ? 0u : min(n_ln, 64u - tc);
      } else {
        tb = min(n_lb, 64u);
        tc = min(n_lc, 64u - tb);
        tn = min(n_ln, 64u - tb - tc);
      }
      uint32_t kind = K_NONE, s = 0;
      if (lane < tb) {
        kind = K_BOUNDARY;
        s = S.lb[n_lb - 1u - lane];
      } else if (lane < tb + tc) {
        kind = K_COLLIDE;
        s = S.lc[n_lc - 1u - (lane - tb)];
      } else if (lane < tb + tc + tn) {
        kind = K_NEW;
        s = S.ln[n_ln - 1u - (lane - tb - tc)];
      }
      n_lb -= tb;
      n_lc -= tc;
      n_ln -= tn;
      // zero-initialised: left undefined on the lanes that skip the event code,
      // their values merge into loop-carried phis and the dense kernel spills
      PathState ps{};
      Isect is{};
      uint32_t nseg = 0;
      uint32_t mk_pid = 0;  // naiveMK: the path id (its iteration and pixel seed every segment)
      float t_hit = 0.0f;
      bool to_ready = false, to_lb = false, to_ln = false;
      bool alive = false;
      bool truncated = false, escaped = false, seg_first = false, seg_next = false;  // counted by ballots
      // ---- regeneration (new items): the wave's cursor into the global queues
      const unsigned long long want = __ballot(kind == K_NEW);
      if (want != 0ull) {
        const uint32_t rank = lane_rank(want);
        bool got = false;
        uint32_t given = 0;  // new items [0, given) get a path
        uint32_t cnext = __builtin_amdgcn_readfirstlane(S.cur[0]), cend = __builtin_amdgcn_readfirstlane(S.cur[1]);
        uint32_t cqh = __builtin_amdgcn_readfirstlane(S.cur[2]);
        while (given < (uint32_t)__popcll(want) && !(cqh & kCurExhausted)) {
          if (cnext == cend) {
            // A queue found empty is never asked again (S.dead): once the
            // queues run dry one after another, a wave would otherwise walk
            // every empty head, one memory round trip each, per dequeue.
            uint32_t b = 0xFFFFFFFFu, qsel = 0;
            if (lane == 0) {
              unsigned long long dead = S.dead;
              for (uint32_t k = 0; k < L.n_queues; ++k) {
                const uint32_t q = ((cqh >> 8) + k) % L.n_queues;
                if ((dead >> q) & 1ull) continue;
                // (a generic atomic: its global form costs the dense kernel ~40 VGPRs of
                // pressure; lane 0 waits for its result right here anyway)
                const uint32_t g = atomicAdd(L.queue + 16 * q, L.chunk);
                if (g < queue_units(L, q)) {
                  b = g;
                  qsel = q;
                  break;
                }
                dead |= 1ull << q;
              }
              S.dead = dead;
            }
            b = __shfl(b, 0);
            qsel = __shfl(qsel, 0);
            if (b == 0xFFFFFFFFu) {
              cqh |= kCurExhausted;
              break;
            }
            cqh = qsel | qsel << 8;
            cnext = b;
            cend = min(b + L.chunk, queue_units(L, qsel));
          }
          const uint32_t take = min((uint32_t)__popcll(want) - given, cend - cnext);
          if (kind == K_NEW && rank >= given && rank < given + take) {
            const uint32_t pid = unit_to_path(L, cqh & 0xFFu, cnext + (rank - given));
            if constexpr (kMK) {
              mk_pid = pid;
            } else {
              path_begin(L, pid, ps);
            }
            if (kRecord) rec_pids<kSlots, kWpg>(L, gw)[s] = pid;
            is.normal = mk3(0, 0, 0);
            nseg = 0;
            got = true;
          }
          cnext += take;
          given += take;
        }
        if (lane == 0) {
          S.cur[0] = cnext;
          S.cur[1] = cend;
          S.cur[2] = cqh;
        }
        // first segment: AABB test (NaiveVolPTsk_kernel.cuh:33-47); a new item
        // that got no path (queues exhausted) files its slot as free again
        const uint32_t n_got = (uint32_t)__popcll(__ballot(got));
        if (lane == 0) S.cnt[STAT_PATHS] += n_got;
        if constexpr (kMK) {
          // d_init (NaiveVolPTmk_kernel.cuh:20-77, mk_init): a miss adds (1,1,1), a failed
          // GGX sample drops the path, else its first d_extend starts below (alive)
          if (got) {
            const uint32_t it = fastdiv(mk_pid, L.div_tile_px);
            nseg = 1;
            seg_first = true;
            const uint32_t r0 = mk_init(me, L, it, mk_pid - it * L.tile_px, ps);
            if (r0 == MK_MISSED) {
              escaped = true;
              to_ln = true;
            } else if (r0 == MK_DROPPED) {
              to_ln = true;
            } else {
              alive = true;
            }
          }
        } else if (got) {
          if (L.max_segments && nseg >= L.max_segments) {
            truncated = true;
            to_ln = true;
            if (kFlush) S.meta[s] = ps.image_id;  // the ended path's pixel (in-launch output)
            if (kRecord) record_end<kSlots, kWpg>(L, gw, s, ps, 2u, nseg);
          } else {
            ++nseg;
            seg_first = true;
            if (!aabb_intersect(me, ps.o, ps.d, is)) {
              escaped = true;  // splat below (splat_wave)
              to_ln = true;
              if (kFlush) S.meta[s] = ps.image_id;  // the ended path's pixel (in-launch output)
              if (kRecord) record_end<kSlots, kWpg>(L, gw, s, ps, 1u, nseg);
            } else if (is.inside) {
              store_full(S, L.pool_T + (size_t)(kWpg > 1 ? gw : blockIdx.x) * kSlots, s, ps, is, nseg, ps.image_id);
              to_ready = true;
            } else {
              kind = K_BOUNDARY;  // enters the box: boundary event in this batch
            }
          }
        }
      }
      float4* __restrict__ gT = L.pool_T + (size_t)(kWpg > 1 ? gw : blockIdx.x) * kSlots;  // this wave's event-only slot part
      if (lane < tb + tc) {
        load_full(S, gT, s, ps, is, nseg, t_hit);
        if constexpr (kMK) {  // the event-only word is the path id
          mk_pid = ps.image_id;
          ps.image_id = mk_pid - fastdiv(mk_pid, L.div_tile_px) * L.tile_px;
        }
      }
      // a filed boundary whose last step passed max_t drew one number too many
      if (lane < tb && !(t_hit <= is.dist)) rng_undo(ps.rng);
      if (kind == K_BOUNDARY) {
        boundary_event(me, ps, is);
        alive = roulette(ps);
      }
      if (kind == K_COLLIDE) {
        scatter_event<kScatterEps>(me, ps, t_hit);
        alive = roulette(ps);
      }
      const uint32_t n_alb = (uint32_t)__popcll(__ballot(kind == K_COLLIDE));
      if ((kind == K_BOUNDARY || kind == K_COLLIDE) && !alive) {  // the path died in roulette
        to_ln = true;
        if (kFlush) S.meta[s] = ps.image_id;  // the ended path's pixel (in-launch output)
        if (kRecord) record_end<kSlots, kWpg>(L, gw, s, ps, 0u, nseg);
      }
      // ---- next segment: AABB test of the survivors ----------------------
      if (alive) {
        if (L.max_segments && nseg >= L.max_segments) {
          truncated = true;
          to_ln = true;
          if (kFlush) S.meta[s] = ps.image_id;  // the ended path's pixel (in-launch output)
          if (kRecord) record_end<kSlots, kWpg>(L, gw, s, ps, 2u, nseg);
        } else {
          ++nseg;
          seg_next = true;
          if constexpr (kMK) {
            // d_extend(depth) (NaiveVolPTmk_kernel.cuh:79-151): re-seed from (iteration,
            // pixel, depth), three unused draws (Q12), a fresh SimpleIsect
            const uint32_t it = fastdiv(mk_pid, L.div_tile_px);
            rng_seeded(ps.rng, it, ps.image_id, nseg - 2u);
            (void)rng_float(ps.rng);
            (void)rng_float(ps.rng);
            (void)rng_float(ps.rng);
            is.dist = 0.0f;
            is.normal = mk3(0, 0, 0);
            is.inside = false;
          }
          if (!aabb_intersect(me, ps.o, ps.d, is)) {
            escaped = true;  // splat below (splat_wave)
            to_ln = true;
            if (kFlush) S.meta[s] = ps.image_id;  // the ended path's pixel (in-launch output)
            if (kRecord) record_end<kSlots, kWpg>(L, gw, s, ps, 1u, nseg);
          } else {
            store_full(S, gT, s, ps, is, nseg, kMK ? mk_pid : ps.image_id);
            to_ready = is.inside;  // medium: Woodcock from t = 0
            to_lb = !is.inside;    // no medium: boundary at isect.dist
          }
        }
      }
      // the batch's escapes (camera rays that miss the box, survivors leaving it), per pixel
      // (the in-launch output instance splats per lane: combining cost it 2 VGPR spills)
      splat_wave<!kFlush>(S, L, ps, escaped, s, lane);
      // a path's segments are the increments of its nseg (each counted once, as
      // the reference's per-iteration RAYS_STATISTICS count)
      {
        const uint32_t n_seg = (uint32_t)(__popcll(__ballot(seg_first)) + __popcll(__ballot(seg_next)));
        const uint32_t n_esc = (uint32_t)__popcll(__ballot(escaped)), n_tr = (uint32_t)__popcll(__ballot(truncated));
        if (lane == 0) {
          S.cnt[STAT_SEGMENTS] += n_seg;
          S.cnt[STAT_ALBEDO] += n_alb;
          S.cnt[STAT_ESCAPED] += n_esc;
          S.cnt[STAT_TRUNCATED] += n_tr;
        }
      }
      const unsigned long long mr = __ballot(to_ready), mb = __ballot(to_lb), mn = __ballot(to_ln);
      if (to_ready) S.ready[(ready_head + n_ready + lane_rank(mr)) % kSlots] = (uint8_t)s;
      if (to_lb) S.lb[n_lb + lane_rank(mb)] = (uint8_t)s;
      if (to_ln) S.ln[n_ln + lane_rank(mn)] = (uint8_t)s;
      if constexpr (kFlush) {
        // in-launch output: the ended paths (their slots' meta holds the pixel) are counted
        // at the next batch
        if (lane == 0) {
          const uint32_t agg = S.pend;  // lane 0's block count of the last batch, beside this batch's splats
          if (agg != 0u) add_counted(L, agg);
          if (agg != 0u || mn != 0ull)
            S.pend = mn != 0ull ? n_ln | (uint32_t)__popcll(mn) << 8 : 0u;
        }
      }
      n_ready += (uint32_t)__popcll(mr);
      n_lb += (uint32_t)__popcll(mb);
      n_ln += (uint32_t)__popcll(mn);
    }
    if (S.cur[2] & kCurExhausted) {
      const uint32_t n_live = n_ready + n_lb + n_lc;
#if CVR_WPOOL_TAILSTAMP
      if (ts_ex == 0) {
        ts_ex = __builtin_amdgcn_s_memrealtime();
        ts_live = n_live;
        ts_steps0 = c_steps;
        ts_seg0 = S.cnt[STAT_SEGMENTS];
      } else {
        ts_ev += __builtin_amdgcn_s_memrealtime() - ts_a;
      }
      ++ts_batches;
#endif
      // The launch's drain.  A wave's lanes cannot all be busy any more, and
      // a batch that waits for its slowest segment stretches the last paths'
      // lives: the batch should run once drain x waiting >= tracking paths.
      // n_ln (the new-path slots, which the empty queues cannot serve) stands
      // in for that rule at no register cost in the track loop: with no path
      // dying in between, tracking = n_live - waiting, so the event trigger
      // waiting + n_ln >= 64 holds exactly when waiting >= n_live d / (d + 1).
      // The batch's new items then get no path and run no code; their slot
      // indices (the stack's stale entries) are never used.
      {
        const uint32_t d = fresh(L).wflags & kDrainMask;
        n_ln = d ? 64u - min(64u, (n_live * d + d) / (d + 1u)) : 0u;
      }
    }
  }

#if CVR_WPOOL_TAILSTAMP
  {
    const unsigned long long ts_end = __builtin_amdgcn_s_memrealtime();
    uint32_t dsteps = c_steps - ts_steps0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsteps += __shfl_xor(dsteps, off);
    if (lane == 0 && gw < kTailWaves) {
      const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
      unsigned long long* g = g_tail + 8 * gw;
      g[0] = ts_start;
      g[1] = ts_ex;
      g[2] = ts_end;
      g[3] = (unsigned long long)ts_live | (unsigned long long)ts_batches << 16 | (unsigned long long)xcc << 40;
      g[4] = ts_ev;
      g[5] = dsteps;
      g[6] = S.cnt[STAT_SEGMENTS] - ts_seg0;
      g[7] = ts_trk;
    }
  }
#endif
  if constexpr (kFlush) {
    const uint32_t pend = S.pend;  // raw: the last batch's ended paths
    if (pend != 0u) {
      const uint32_t agg = count_ended(S, L, pend, lane);
      if (lane == 0) add_counted(L, agg);
    }
  }
  // ---- counters ------------------------------------------------------------
  {
    unsigned long long steps = c_steps, fetch = c_fetch;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      steps += __shfl_xor(steps, off);
      fetch += __shfl_xor(fetch, off);
    }
    // density evaluations: steps minus segments whose last step passed max_t
    const unsigned long long w[STAT_COUNT] = {S.cnt[STAT_PATHS], S.cnt[STAT_SEGMENTS], steps, steps - n_over,
                                              S.cnt[STAT_ALBEDO], S.cnt[STAT_ESCAPED], S.cnt[STAT_TRUNCATED], fetch};
    if (lane < (uint32_t)STAT_COUNT && w[lane])
      __hip_atomic_fetch_add(gmem(L.stats + lane), w[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (kCountWords) {
      unsigned long long words = c_words;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) words += __shfl_xor(words, off);
      if (lane == 0) __hip_atomic_fetch_add(gmem(L.stats + kStatWordsSlot), words, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

#if CVR_WPOOL_PAIR  // experiment build only: make variant-pair (round-6 verdict: 4.1x slower, not in libcvr.so)
// ---- workgroup-shared event lists (CVR_OPT_WAVE_PAIR 1, round 5) ------------
// The round-3/4 verdicts' "event list shared by the waves of a workgroup": two
// waves per workgroup, one unified slot array (2 x kPairSlots paths), each wave
// with its own track-ready ring, new-path stack and queue cursor (wave-uniform
// scalars, as k_wpool), but ONE boundary list and ONE collision list for both:
// 256-entry LDS rings that either wave files into (ds_add_rtn on the list's
// tail reserves the entries) and either wave takes a batch from (a CAS on the
// packed heads claims them; entries are 0xFF until written, so a taker that
// meets a reserved but unwritten entry waits for it).  A batch thus sees both
// waves' events, so kind-major batches (48 boundary / 24 collision events of
// one kind) fill twice as fast.  A path that a wave takes from the shared lists
// becomes that wave's: it goes to its ready ring, to the shared boundary list or
// to its new-path stack.  Dense media with cells and brick bounds only (C2 /
// C3), no in-launch output, no records.  The same walk, the same per-path
// results: only which wave runs which event changes.
template <int kWaves>
struct PairSize {
  // LDS bytes per two-wave workgroup: twice a one-wave workgroup's budget
  static constexpr int kBudget = 2 * (163840 / (4 * kWaves) / kLdsGranule * kLdsGranule);
  static constexpr int kParams = (int)((sizeof(LaunchParams) + 15) / 16 * 16);
  static constexpr int kHeader = 2 * (4 * STAT_COUNT + 8 + 12 + 4) + 16;
  // unified slots of the pair: 60 bytes of path state each + a ready-ring and a
  // new-path-stack entry per wave (a wave may come to own every slot)
  static constexpr int value = (kBudget - kParams - kHeader - 512) / 64;
  static_assert(value <= 254, "slot ids are u8 with 0xFF as the empty ring entry");
};
template <int kN>
struct PairPool {
  float4 a[kN], b[kN];
  uint4 c[kN];
  uint2 e[kN];
  uint32_t meta[kN];
  uint8_t ready[2][kN];  // each wave's ring of track-ready slots
  uint8_t ln[2][kN];     // each wave's stack of slots waiting for a new path
  uint8_t lb[256];       // shared ring of boundary events (0xFF: not written yet / taken)
  uint8_t lc[256];       // shared ring of real collisions
  uint32_t tail[2];      // lb, lc tails (entries reserved so far)
  uint32_t heads;        // lb head | lc head << 16 (mod 2^16; claimed by CAS)
  uint32_t cnt[2][STAT_COUNT];
  unsigned long long dead[2];
  uint32_t cur[2][3];
  uint32_t gone[2];      // the wave has left its loop (every queue was found empty)
};
// events of list k (0 boundary, 1 collision) reserved and not yet claimed
__device__ __forceinline__ uint32_t pair_avail(uint32_t heads, uint32_t tail, uint32_t k) {
  return (tail - (heads >> (16 * k))) & 0xFFFFu;
}

template <bool kScatterEps, int kWaves, int kMed>
__global__ __launch_bounds__(128, kWaves) void k_wpair(MediumParams mk, LaunchParams Lk) {
  static_assert(kMed == kMedDenseFull || kMed == kMedDenseFullUniform, "paired waves: dense media with cells and bounds");
  constexpr int kN = PairSize<kWaves>::value;  // unified slots of the pair
  MediumParams m = mk;
  m.leaves = nullptr;
  m.leaf_density = nullptr;
  m.leaf_albedo = nullptr;
  m.sbounds = nullptr;
  __builtin_assume(m.cells != nullptr);
  __builtin_assume(m.bounds != nullptr);
  m.albedo_uniform = kMed == kMedDenseFullUniform ? 1u : 0u;
  static_assert(sizeof(PairPool<kN>) + sizeof(LaunchParams) <= (size_t)PairSize<kWaves>::kBudget,
                "paired pool exceeds the LDS budget of kWaves waves per SIMD");
  __shared__ PairPool<kN> S;
  __shared__ LaunchParams L;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) {
    L = Lk;
    S.tail[0] = S.tail[1] = 0u;
    S.heads = 0u;
    S.gone[0] = S.gone[1] = 0u;
  }
  for (uint32_t i = threadIdx.x; i < 256u; i += 128u) {
    S.lb[i] = 0xFFu;
    S.lc[i] = 0xFFu;
  }
  uint32_t c_steps = 0, c_fetch = 0;
  if (lane < (uint32_t)STAT_COUNT) S.cnt[wv][lane] = 0u;
  if (lane == 0) {
    S.dead[wv] = 0ull;
    S.cur[wv][0] = S.cur[wv][1] = 0u;
  }
  __syncthreads();
  uint32_t n_over = 0;
  if (lane == 0) {
    const uint32_t vw = 2u * blockIdx.x + wv;  // the wave's index as a one-wave launch would number it
    S.cur[wv][2] = (((__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u) % (L.n_queues / L.sub)) * L.sub +
                    (vw >> 4) % L.sub)
                   << 8;
  }
  const uint32_t batch = L.batch;
  uint32_t ready_head = 0, n_ready = 0;
  // this wave's half of the slots starts free
  uint32_t n_ln = kN / 2;
  for (uint32_t i = lane; i < (uint32_t)kN / 2; i += 64u) S.ln[wv][i] = (uint8_t)(wv * (kN / 2) + i);
  float4* __restrict__ gT = L.pool_T + (size_t)blockIdx.x * kN;  // the pair's event-only slot part

  // File lanes' slots into the shared lists: mb boundary, mc collision lanes.
  // The slot's LDS state is written before: the release fence orders it (and
  // the wave's pool_T stores) before the list entries the other wave may read.
  // full: the entries follow global pool_T stores of this batch (vmcnt wait); from the
  // track loop only LDS state precedes them, and one wave's LDS operations are performed in
  // order, so a compiler barrier suffices.
  auto file_shared = [&](bool is_b, bool is_c, uint32_t s, bool full) {
    const unsigned long long mb = __ballot(is_b), mc = __ballot(is_c);
    const uint32_t kb = (uint32_t)__popcll(mb), kc = (uint32_t)__popcll(mc);
    if ((kb | kc) == 0u) return;
    uint32_t tb0 = 0, tc0 = 0;
    if (lane == 0) {
      if (kb) tb0 = __hip_atomic_fetch_add(&S.tail[0], kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (kc) tc0 = __hip_atomic_fetch_add(&S.tail[1], kc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    tb0 = __builtin_amdgcn_readfirstlane(tb0);
    tc0 = __builtin_amdgcn_readfirstlane(tc0);
    if (full) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    else __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // An entry is written only once the taker of the same ring position one lap earlier
    // has read it (it writes 0xFF back): a taker that claimed its entries but was kept from
    // reading them (its wave starved at a lower priority while the rings went round) would
    // otherwise read a later lap's entry and leave the later taker waiting for ever.
    if (is_b || is_c) {
      uint8_t* e = is_b ? &S.lb[(tb0 + lane_rank(mb)) & 255u] : &S.lc[(tc0 + lane_rank(mc)) & 255u];
      uint32_t spins = 0;
      while (__hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0xFFu && ++spins < (1u << 16)) {
      }
      if (spins >= (1u << 16)) atomicAdd(&S.cnt[wv][STAT_TRUNCATED], 1u);  // (bug report, as below)
      __hip_atomic_store(e, (uint8_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };

  // Watchdog (the variant is an experiment): a wave that runs more outer iterations than
  // any launch needs (C2: a wave runs ~10^3-10^4 batches) leaves its loop and reports
  // it in the truncated counter (+2^20 per wave), so a scheduling bug ends the launch
  // with wrong counters instead of hanging the GPU.
  uint32_t watchdog = 0;
  uint32_t n_mine = 0;  // events this wave filed since its last batch (its batch trigger)
  for (;;) {
    if (++watchdog > (1u << 22)) {
      if (lane == 0) {
        atomicAdd(&S.cnt[wv][STAT_TRUNCATED], 1u << 20);
        __hip_atomic_store(&S.gone[wv], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      break;
    }
    __builtin_amdgcn_s_setprio(kPrioTrack);
    int slot = -1;
    int fst = 0;
    V3 o = mk3(0, 0, 0), d = mk3(0, 0, 0);
    Rng rng{0, 0, 0, 0, 0, 0};
    float t = 0.0f, max_t = 0.0f;
    uint32_t tracks = 0;
    for (;;) {
      if (++tracks > (1u << 24)) {  // (watchdog, as above: no segment takes this long)
        if (lane == 0) atomicAdd(&S.cnt[wv][STAT_TRUNCATED], 1u << 20);
        watchdog = 1u << 22;
        break;
      }
      const unsigned long long trk = (__ballot(slot >= 0) & __ballot(fst == 0));
      const uint32_t n_trk = (uint32_t)__popcll(trk);
      if (64u - n_trk >= batch || n_trk == 0u) {
        if (fst == 2 && !(t < max_t)) fst = 3;
        if (fst != 0) store_track(S, (uint32_t)slot, t, rng);
        n_over += (uint32_t)__popcll(__ballot(fst == 1));
        n_mine += (uint32_t)__popcll(__ballot(fst != 0));
        file_shared((fst & 1) != 0, fst == 2, (uint32_t)slot, false);
        if (fst != 0) {
          slot = -1;
          fst = 0;
        }
        const unsigned long long idle = __ballot(slot < 0);
        const uint32_t k = min((uint32_t)__popcll(idle), n_ready), rank = lane_rank(idle);
        if (slot < 0 && rank < k) {
          const uint32_t r = ready_head + rank;
          const uint32_t s = S.ready[wv][r >= (uint32_t)kN ? r - kN : r];
          slot = (int)s;
          load_track(S, s, o, d, rng, t, max_t);
        }
        ready_head += k;
        if (ready_head >= (uint32_t)kN) ready_head -= kN;
        n_ready -= k;
      }
      const uint32_t n_act = (uint32_t)__popcll((__ballot(slot >= 0) & __ballot(fst == 0)));
      const uint32_t n_fin = (uint32_t)__popcll(__ballot(fst != 0));
      // the trigger counts this wave's own filings since its last batch (registers only, as
      // k_wpool); the batch then takes what both waves have filed
      if (n_mine + n_ln + n_fin >= 64u || (n_act == 0u && n_ready == 0u)) {
        if (fst == 2 && !(t < max_t)) fst = 3;
        if (slot >= 0) store_track(S, (uint32_t)slot, t, rng);
        const unsigned long long mr = (__ballot(slot >= 0) & __ballot(fst == 0));
        if (slot >= 0 && fst == 0) S.ready[wv][(ready_head + n_ready + lane_rank(mr)) % kN] = (uint8_t)slot;
        n_over += (uint32_t)__popcll(__ballot(fst == 1));
        n_ready += (uint32_t)__popcll(mr);
        file_shared((fst & 1) != 0, fst == 2, (uint32_t)slot, false);
        break;
      }
#pragma unroll
      for (int u = 0; u < CVR_WPOOL_UNROLL / kLook; ++u) {
        if (slot >= 0 && fst == 0) {
          float tk[kLook], xtk[kLook];
          uint32_t sva[kLook], svb[kLook];
          WoodcockPoint Pk[kLook];
          float tt = t;
#pragma unroll
          for (int k = 0; k < kLook; ++k) {
            const float xi = rng_float(rng);
            xtk[k] = rng_float(rng);
            sva[k] = rng.v0;
            svb[k] = rng.v1;
            tt = woodcock_advance(m, xi, tt);
            tk[k] = tt;
          }
#pragma unroll
          for (int k = 0; k < kLook; ++k) Pk[k] = woodcock_point(m, o, d, tk[k]);
          int end = kLook;
#pragma unroll
          for (int k = 0; k < kLook; ++k) {
            if (end == kLook) {
              if (!(tk[k] <= max_t)) {
                fst = 1;
                end = k;
              } else if (!(Pk[k].qb < xtk[k])) {
                ++c_fetch;
                const float rho = m.scale * woodcock_density(m, Pk[k]);
                if (!(rho * m.inv_sigma < xtk[k])) {
                  fst = 2;
                  end = k;
                }
              }
            }
          }
          c_steps += end == kLook ? kLook : end + 1;
          t = tk[kLook - 1];
#pragma unroll
          for (int k = 0; k < kLook - 1; ++k)
            if (end == k) t = tk[k];
          if (end < kLook - 1) {
            uint32_t w[2 * kLook + 5];
#pragma unroll
            for (int k = 0; k < kLook - 1; ++k) {
              w[2 * k + 2] = sva[k];
              w[2 * k + 3] = svb[k];
            }
            w[2 * kLook] = rng.v0;
            w[2 * kLook + 1] = rng.v1;
            w[2 * kLook + 2] = rng.v2;
            w[2 * kLook + 3] = rng.v3;
            w[2 * kLook + 4] = rng.v4;
#pragma unroll
            for (int j = 1; j < kLook; ++j) {
              if (end + 1 == j) {
                rng.v0 = w[2 * j];
                rng.v1 = w[2 * j + 1];
                rng.v2 = w[2 * j + 2];
                rng.v3 = w[2 * j + 3];
                rng.v4 = w[2 * j + 4];
              }
            }
            rng.d -= (uint32_t)(2 * (kLook - 1 - end)) * 362437u;
          }
        }
      }
    }
    // claim the batch's events from the shared lists (kind-major thresholds as k_wpool), at
    // the top priority until they are read (see file_shared)
    __builtin_amdgcn_s_setprio(3);
    uint32_t tb = 0, tc = 0, hb = 0, hc = 0;
    {
      uint32_t h = __builtin_amdgcn_readfirstlane(S.heads);
      for (;;) {
        const uint32_t ab = pair_avail(h, __builtin_amdgcn_readfirstlane(S.tail[0]), 0);
        const uint32_t ac = pair_avail(h, __builtin_amdgcn_readfirstlane(S.tail[1]), 1);
        if (ab >= (uint32_t)CVR_WPOOL_KIND_MIN) {
          tb = min(ab, 64u);
          tc = 0;
        } else if (ac >= (uint32_t)CVR_WPOOL_KIND_MIN_C) {
          tb = 0;
          tc = min(ac, 64u);
        } else {
          tb = min(ab, 64u);
          tc = min(ac, 64u - tb);
        }
        if ((tb | tc) == 0u) break;
        const uint32_t want = ((h + tb) & 0xFFFFu) | (((h >> 16) + tc) << 16);
        uint32_t got = 0;
        if (lane == 0) {
          got = h;
          __hip_atomic_compare_exchange_strong(&S.heads, &got, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        got = __builtin_amdgcn_readfirstlane(got);
        if (got == h) break;
        h = got;  // the other wave claimed first: retry with its heads
      }
      hb = h & 0xFFFFu;
      hc = h >> 16;
    }
    const bool any_event = (tb | tc) != 0u;
    if (!any_event && n_ready == 0u) {
      const uint32_t hs = __builtin_amdgcn_readfirstlane(S.heads);
      const bool shared_empty = pair_avail(hs, __builtin_amdgcn_readfirstlane(S.tail[0]), 0) +
                                    pair_avail(hs, __builtin_amdgcn_readfirstlane(S.tail[1]), 1) ==
                                0u;
      // no path left: nothing to track, nothing shared, no new path to start
      if (shared_empty && (S.cur[wv][2] & kCurExhausted)) {
        if (lane == 0) __hip_atomic_store(&S.gone[wv], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      // holding no slot at all while the other wave has left (with every slot free): this
      // wave takes all of them and goes on with its queue cursor
      if (shared_empty && n_ln == 0u &&
          __hip_atomic_load(&S.gone[wv ^ 1u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) {
        for (uint32_t i = lane; i < (uint32_t)kN; i += 64u) S.ln[wv][i] = (uint8_t)i;
        n_ln = kN;
        continue;
      }
      // the other wave holds every slot (this wave has none free and none ready): wait for
      // it to file events this wave can take, without taking its issue slots meanwhile
      if (n_ln == 0u) {
        __builtin_amdgcn_s_sleep(4);
        continue;
      }
    }
    MediumParams me = m;
    me.g = opaque_s(m.g);
    me.ax = opaque_s(m.ax);
    me.ay = opaque_s(m.ay);
    me.eta = opaque_s(m.eta);
    me.inv_eta = opaque_s(m.inv_eta);
    me.bmin = mk3(opaque_s(m.bmin.x), opaque_s(m.bmin.y), opaque_s(m.bmin.z));
    me.bmax = mk3(opaque_s(m.bmax.x), opaque_s(m.bmax.y), opaque_s(m.bmax.z));
    me.albedo_bg = mk3(opaque_s(m.albedo_bg.x), opaque_s(m.albedo_bg.y), opaque_s(m.albedo_bg.z));
    {
      uint32_t tn;
      if (tb >= (uint32_t)CVR_WPOOL_KIND_MIN) tn = min(n_ln, 64u - tb);
      else if (tc >= (uint32_t)CVR_WPOOL_KIND_MIN_C) tn = n_ln < 64u ? 0u : min(n_ln, 64u - tc);
      else tn = min(n_ln, 64u - tb - tc);
      uint32_t kind = K_NONE, s = 0;
      if (lane < tb + tc) {
        // a claimed entry may be reserved but not yet written by the other wave: wait for it
        uint8_t* q = lane < tb ? &S.lb[(hb + lane) & 255u] : &S.lc[(hc + lane - tb) & 255u];
        uint32_t v, spins = 0;
        do {
          v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } while (v == 0xFFu && ++spins < (1u << 16));
        // (a bounded wait: an entry that never appears would be a bug; the item is then
        // dropped and counted as truncated, so the launch ends and the counters differ)
        __hip_atomic_store(q, (uint8_t)0xFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        s = v;
        kind = v == 0xFFu ? K_NONE : lane < tb ? K_BOUNDARY : K_COLLIDE;
        if (v == 0xFFu) atomicAdd(&S.cnt[wv][STAT_TRUNCATED], 1u);
      } else if (lane < tb + tc + tn) {
        kind = K_NEW;
        s = S.ln[wv][n_ln - 1u - (lane - tb - tc)];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the filer's slot state and pool_T stores
      __builtin_amdgcn_s_setprio(kPrioEvent);
      n_ln -= tn;
      PathState ps{};
      Isect is{};
      uint32_t nseg = 0;
      float t_hit = 0.0f;
      bool to_ready = false, to_lb = false, to_ln = false;
      bool truncated = false, escaped = false, seg_first = false, seg_next = false;
      const unsigned long long want = __ballot(kind == K_NEW);
      if (want != 0ull) {
        const uint32_t rank = lane_rank(want);
        bool got = false;
        uint32_t given = 0;
        uint32_t cnext = __builtin_amdgcn_readfirstlane(S.cur[wv][0]), cend = __builtin_amdgcn_readfirstlane(S.cur[wv][1]);
        uint32_t cqh = __builtin_amdgcn_readfirstlane(S.cur[wv][2]);
        while (given < (uint32_t)__popcll(want) && !(cqh & kCurExhausted)) {
          if (cnext == cend) {
            uint32_t b = 0xFFFFFFFFu, qsel = 0;
            if (lane == 0) {
              unsigned long long dead = S.dead[wv];
              for (uint32_t k = 0; k < L.n_queues; ++k) {
                const uint32_t q = ((cqh >> 8) + k) % L.n_queues;
                if ((dead >> q) & 1ull) continue;
                const uint32_t g = atomicAdd(L.queue + 16 * q, L.chunk);
                if (g < queue_units(L, q)) {
                  b = g;
                  qsel = q;
                  break;
                }
                dead |= 1ull << q;
              }
              S.dead[wv] = dead;
            }
            b = __shfl(b, 0);
            qsel = __shfl(qsel, 0);
            if (b == 0xFFFFFFFFu) {
              cqh |= kCurExhausted;
              break;
            }
            cqh = qsel | qsel << 8;
            cnext = b;
            cend = min(b + L.chunk, queue_units(L, qsel));
          }
          const uint32_t take = min((uint32_t)__popcll(want) - given, cend - cnext);
          if (kind == K_NEW && rank >= given && rank < given + take) {
            const uint32_t pid = unit_to_path(L, cqh & 0xFFu, cnext + (rank - given));
            path_begin(L, pid, ps);
            is.normal = mk3(0, 0, 0);
            nseg = 0;
            got = true;
          }
          cnext += take;
          given += take;
        }
        if (lane == 0) {
          S.cur[wv][0] = cnext;
          S.cur[wv][1] = cend;
          S.cur[wv][2] = cqh;
        }
        const uint32_t n_got = (uint32_t)__popcll(__ballot(got));
        if (lane == 0) S.cnt[wv][STAT_PATHS] += n_got;
        if (got) {
          if (L.max_segments && nseg >= L.max_segments) {
            truncated = true;
            to_ln = true;
          } else {
            ++nseg;
            seg_first = true;
            if (!aabb_intersect(me, ps.o, ps.d, is)) {
              escaped = true;
              to_ln = true;
            } else if (is.inside) {
              store_full(S, gT, s, ps, is, nseg, ps.image_id);
              to_ready = true;
            } else {
              kind = K_BOUNDARY;
            }
          }
        }
      }
      const bool filed = lane < tb + tc && kind != K_NONE;  // (K_NONE: a dropped entry, see above)
      if (filed) load_full(S, gT, s, ps, is, nseg, t_hit);
      if (filed && lane < tb && !(t_hit <= is.dist)) rng_undo(ps.rng);
      bool alive = false;
      if (kind == K_BOUNDARY) {
        boundary_event(me, ps, is);
        alive = roulette(ps);
      }
      if (kind == K_COLLIDE) {
        scatter_event<kScatterEps>(me, ps, t_hit);
        alive = roulette(ps);
      }
      const uint32_t n_alb = (uint32_t)__popcll(__ballot(kind == K_COLLIDE));
      if ((kind == K_BOUNDARY || kind == K_COLLIDE) && !alive) to_ln = true;
      if (alive) {
        if (L.max_segments && nseg >= L.max_segments) {
          truncated = true;
          to_ln = true;
        } else {
          ++nseg;
          seg_next = true;
          if (!aabb_intersect(me, ps.o, ps.d, is)) {
            escaped = true;
            to_ln = true;
          } else {
            store_full(S, gT, s, ps, is, nseg, ps.image_id);
            to_ready = is.inside;
            to_lb = !is.inside;
          }
        }
      }
      splat_wave<true>(S, L, ps, escaped, s, lane);
      {
        const uint32_t n_seg = (uint32_t)(__popcll(__ballot(seg_first)) + __popcll(__ballot(seg_next)));
        const uint32_t n_esc = (uint32_t)__popcll(__ballot(escaped)), n_tr = (uint32_t)__popcll(__ballot(truncated));
        if (lane == 0) {
          S.cnt[wv][STAT_SEGMENTS] += n_seg;
          S.cnt[wv][STAT_ALBEDO] += n_alb;
          S.cnt[wv][STAT_ESCAPED] += n_esc;
          S.cnt[wv][STAT_TRUNCATED] += n_tr;
        }
      }
      const unsigned long long mr = __ballot(to_ready), mn = __ballot(to_ln);
      if (to_ready) S.ready[wv][(ready_head + n_ready + lane_rank(mr)) % kN] = (uint8_t)s;
      if (to_ln) S.ln[wv][n_ln + lane_rank(mn)] = (uint8_t)s;
      n_ready += (uint32_t)__popcll(mr);
      n_ln += (uint32_t)__popcll(mn);
      n_mine = (uint32_t)__popcll(__ballot(to_lb));
      file_shared(to_lb, false, s, true);
    }
    if (S.cur[wv][2] & kCurExhausted) {
      const uint32_t hs = __builtin_amdgcn_readfirstlane(S.heads);
      const uint32_t n_live = n_ready + pair_avail(hs, __builtin_amdgcn_readfirstlane(S.tail[0]), 0) +
                              pair_avail(hs, __builtin_amdgcn_readfirstlane(S.tail[1]), 1);
      const uint32_t dr = fresh(L).wflags & kDrainMask;
      n_ln = dr ? 64u - min(64u, (n_live * dr + dr) / (dr + 1u)) : 0u;
    }
  }
  {
    unsigned long long steps = c_steps, fetch = c_fetch;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      steps += __shfl_xor(steps, off);
      fetch += __shfl_xor(fetch, off);
    }
    const unsigned long long w[STAT_COUNT] = {S.cnt[wv][STAT_PATHS], S.cnt[wv][STAT_SEGMENTS], steps, steps - n_over,
                                              S.cnt[wv][STAT_ALBEDO], S.cnt[wv][STAT_ESCAPED], S.cnt[wv][STAT_TRUNCATED],
                                              fetch};
    if (lane < (uint32_t)STAT_COUNT && w[lane])
      __hip_atomic_fetch_add(gmem(L.stats + lane), w[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#endif  // CVR_WPOOL_PAIR

// Instances: 5 waves per SIMD (the default budget) for every medium layout, with and
// without the in-launch output; the other budgets for the generic layouts.
template <bool E>
static const void* wpool_fn(int waves, bool sparse, bool full, bool flush = false, bool uniform = false) {
#define CVR_WP(W, M, F) reinterpret_cast<const void*>(&k_wpool<E, W, M, false, F>)
  if (waves == 5) {
    if (sparse) return flush ? CVR_WP(5, kMedSparse, true) : CVR_WP(5, kMedSparse, false);
    if (full && uniform) return flush ? CVR_WP(5, kMedDenseFullUniform, true) : CVR_WP(5, kMedDenseFullUniform, false);
    if (full) return flush ? CVR_WP(5, kMedDenseFull, true) : CVR_WP(5, kMedDenseFull, false);
    return flush ? CVR_WP(5, kMedDense, true) : CVR_WP(5, kMedDense, false);
  }
  if (flush) return nullptr;
  if (sparse) return CVR_WP(4, kMedSparse, false);
  if (waves == 6) return CVR_WP(6, kMedDense, false);
  if (waves == 3) return CVR_WP(3, kMedDense, false);
  return CVR_WP(4, kMedDense, false);
#undef CVR_WP
}
// Record instances (cvr_trace_launch; debug only, so the production kernels
// carry none of the record code): the default register budgets, generic layouts.
template <bool E>
static const void* wpool_record_fn(int waves, bool sparse) {
  if (sparse) return waves == 5   ? reinterpret_cast<const void*>(&k_wpool<E, 5, kMedSparse, true, false>)
                    : waves == 4 ? reinterpret_cast<const void*>(&k_wpool<E, 4, kMedSparse, true, false>)
                                 : nullptr;
  return waves == 5 ? reinterpret_cast<const void*>(&k_wpool<E, 5, kMedDense, true, false>) : nullptr;
}

// naiveMK instances (kMedMK): 5 waves per SIMD, every medium layout, scatter -eps.
static const void* wpool_mk_fn(bool sparse, bool full, bool uniform) {
#define CVR_WPMK(M) reinterpret_cast<const void*>(&k_wpool<true, 5, (M) | kMedMK, false, false>)
  if (sparse) return CVR_WPMK(kMedSparse);
  if (full && uniform) return CVR_WPMK(kMedDenseFullUniform);
  if (full) return CVR_WPMK(kMedDenseFull);
  return CVR_WPMK(kMedDense);
#undef CVR_WPMK
}

hipError_t launch_wpool(const MediumParams& m, const LaunchParams& L, bool scatter_eps, int waves, uint32_t grid,
                        hipStream_t s, bool pair, bool naive_mk, bool count_words) {
  if (L.path_count == 0) return hipSuccess;
  const bool sparse = m.leaves != nullptr;
  const bool flush = L.frame_done != nullptr;
  const bool full = !sparse && m.cells != nullptr && m.bounds != nullptr;
  const bool uniform = m.albedo_uniform != 0u;
  if (L.rec && flush) return hipErrorInvalidValue;
  if (naive_mk) {
    if (waves != 5 || flush || L.rec) return hipErrorInvalidValue;
    if (grid % wpool_wpg(waves, sparse)) return hipErrorInvalidValue;
    MediumParams mm = m;
    LaunchParams ll = L;
    void* args[] = {&mm, &ll};
    return hipLaunchKernel(wpool_mk_fn(sparse, full, uniform), dim3(grid / wpool_wpg(waves, sparse)),
                           dim3(64 * wpool_wpg(waves, sparse)), args, 0, s);
  }
#if CVR_WPOOL_PAIR
  if (pair && waves == 5 && full && !flush && !L.rec && grid >= 2) {
    // paired waves (workgroup-shared event lists): two waves per workgroup
#define CVR_WPAIR(E, M) reinterpret_cast<const void*>(&k_wpair<E, 5, M>)
    const void* fn = scatter_eps ? (uniform ? CVR_WPAIR(true, kMedDenseFullUniform) : CVR_WPAIR(true, kMedDenseFull))
                                 : (uniform ? CVR_WPAIR(false, kMedDenseFullUniform) : CVR_WPAIR(false, kMedDenseFull));
#undef CVR_WPAIR
    MediumParams mm = m;
    LaunchParams ll = L;
    void* args[] = {&mm, &ll};
    return hipLaunchKernel(fn, dim3(grid / 2), dim3(128), args, 0, s);
  }
#else
  if (pair) return hipErrorInvalidValue;  // (cvr_set_option refuses it first)
#endif
  const void* fn = L.rec ? (scatter_eps ? wpool_record_fn<true>(waves, sparse) : wpool_record_fn<false>(waves, sparse))
                         : (scatter_eps ? wpool_fn<true>(waves, sparse, full, flush, uniform)
                                        : wpool_fn<false>(waves, sparse, full, flush, uniform));
  // the counting instances (CVR_OPT_COUNT_WORDS): sparse media, 5 waves per SIMD, no records
  // or in-launch output (other launches count nothing: cvr_stats.words stays 0)
  if (count_words && sparse && waves == 5 && !L.rec && !flush)
    fn = scatter_eps ? reinterpret_cast<const void*>(&k_wpool<true, 5, kMedSparse | kMedCount, false, false>)
                     : reinterpret_cast<const void*>(&k_wpool<false, 5, kMedSparse | kMedCount, false, false>);
  if (!fn) return hipErrorInvalidValue;  // no record / in-launch output instance for this register budget
  // (a grid of whole workgroups: pool_T and the record ids are sized for grid waves)
  if (grid % wpool_wpg(waves, sparse)) return hipErrorInvalidValue;
  MediumParams mm = m;
  LaunchParams ll = L;
  void* args[] = {&mm, &ll};
  return hipLaunchKernel(fn, dim3(grid / wpool_wpg(waves, sparse)), dim3(64 * wpool_wpg(waves, sparse)), args, 0, s);
}

bool wpool_pair_built() { return CVR_WPOOL_PAIR != 0; }

#if CVR_WPOOL_TAILSTAMP
// (diagnostic build) the per-wave stamps of the last launch, 8 u64 per wave
extern "C" int cvr_debug_tailstamps(unsigned long long* host, size_t n_waves) {
  if (n_waves > kTailWaves) n_waves = kTailWaves;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail), n_waves * 64, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
extern "C" int cvr_debug_tailstamps_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_tail)) != hipSuccess) return -2;
  return hipMemset(p, 0, sizeof(unsigned long long) * 8 * kTailWaves) == hipSuccess ? 0 : -2;
}
#endif

uint32_t wpool_wpg(int waves, bool sparse) { return (uint32_t)wpg_of(sparse ? kMedSparse : kMedDense, waves); }

uint32_t wpool_slots(int waves, bool sparse) {
  constexpr int kEmB = CVR_WPOOL_EMASK ? 4 * kEmaskWords : 0;
  if (sparse)
    return waves == 5 ? PoolSize<5, kEmB, wpg_of(kMedSparse, 5)>::value : PoolSize<4, kEmB, wpg_of(kMedSparse, 4)>::value;
  return waves == 5   ? PoolSize<5, 0, wpg_of(kMedDense, 5)>::value
         : waves == 6 ? PoolSize<6, 0, wpg_of(kMedDense, 6)>::value
         : waves == 3 ? PoolSize<3, 0, wpg_of(kMedDense, 3)>::value
                      : PoolSize<4, 0, wpg_of(kMedDense, 4)>::value;
}

hipError_t wpool_occupancy(bool scatter_eps, int waves, bool sparse, int* waves_per_cu) {
  const void* fn = scatter_eps ? wpool_fn<true>(waves, sparse, false) : wpool_fn<false>(waves, sparse, false);
  int blocks = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, 64 * wpool_wpg(waves, sparse), 0);
  *waves_per_cu = blocks * (int)wpool_wpg(waves, sparse);
  return e;
}

}  // namespace cvr
