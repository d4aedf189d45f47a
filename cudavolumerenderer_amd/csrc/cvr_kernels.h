// cvr_kernels.h - host-side launch entry points of cvr_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cvr_walk.h"

namespace cvr {

// Per-context work area (cvr_api.cpp d_work, zeroed per launch), in bytes:
// 16 u64 stats at 0, 16 u64 diagnostic counters at 128, up to 64 queue heads
// from 256 (one 64-byte line each, LaunchParams::queue).
constexpr size_t kWorkStats = 0, kWorkDebug = 128, kWorkQueues = 256, kMaxQueues = 64;
constexpr size_t kWorkBytesBase = kWorkQueues + kMaxQueues * 64;

// Per-path debug record; layout identical to cvr_path_record (include/cvr.h)
// and oracle_path (oracle/cvr_oracle.c).
struct PathRecord {
  uint32_t image_id;
  uint32_t flags;  // bit0 escaped (contributed), bit1 truncated
  float T[3];
  uint32_t n_segments, n_steps, n_density, n_albedo;
};

// Ray-slot pool of the wavefront scheduler (cvr_wavefront.hip), SoA in HBM.
struct WfPool {
  float *ox, *oy, *oz, *dx, *dy, *dz, *tx, *ty, *tz, *dist, *t;
  uint32_t *r0, *r1, *r2, *r3, *r4, *rd;
  uint32_t* img;
  uint32_t* meta;    // state | normal code << 2 | segments << 8
  uint32_t* cursor;  // per events-wave [q_next, q_end) into the path-id range
  unsigned int* head;  // global path-id dequeue head
  unsigned int* alive; // set by the events kernel when a slot needs tracking
  unsigned long long* stats_events;  // per events-wave rows of 8 counters
  unsigned long long* stats_track;   // per track-wave rows of 8 counters
  uint32_t n;        // slots
};

hipError_t wf_launch_events(const MediumParams& m, const LaunchParams& L, const WfPool& P, bool scatter_eps,
                            hipStream_t s);
hipError_t wf_launch_track(const MediumParams& m, const LaunchParams& L, const WfPool& P, uint32_t grid,
                           hipStream_t s);
hipError_t wf_track_occupancy(int* blocks_per_cu);
hipError_t wf_launch_reduce(const unsigned long long* rows, uint32_t nrows, unsigned long long* out, hipStream_t s);

hipError_t launch_naive(const MediumParams& m, const LaunchParams& L, bool scatter_eps, hipStream_t s);
hipError_t launch_persistent(const MediumParams& m, const LaunchParams& L, bool scatter_eps, int waves,
                             uint32_t grid, hipStream_t s);
hipError_t persistent_occupancy(bool scatter_eps, int waves, int* blocks_per_cu);
hipError_t launch_trace(const MediumParams& m, const LaunchParams& L, bool scatter_eps, PathRecord* rec,
                        hipStream_t s);
hipError_t launch_pool(const MediumParams& m, const LaunchParams& L, bool scatter_eps, uint32_t grid, hipStream_t s);
hipError_t pool_occupancy(bool scatter_eps, int* blocks_per_cu);
// whether this build carries k_wpair (CVR_WPOOL_PAIR; only `make variant-pair`)
bool wpool_pair_built();
// pair: two waves per workgroup sharing their event lists (k_wpair; dense media with
// cells and bounds, 5 waves per SIMD, no records / in-launch output; else k_wpool).
// naive_mk: naiveMK's walk on the wave pool (5 waves per SIMD, no records / in-launch output).
// count_words: sparse media, the counting instance (CVR_OPT_COUNT_WORDS: brick words loaded).
hipError_t launch_wpool(const MediumParams& m, const LaunchParams& L, bool scatter_eps, int waves, uint32_t grid,
                        hipStream_t s, bool pair = false, bool naive_mk = false, bool count_words = false);
// Resident waves per CU of the wave-pool instance (workgroups per CU x waves per workgroup).
hipError_t wpool_occupancy(bool scatter_eps, int waves, bool sparse, int* waves_per_cu);
// Pool slots per wave of the wave-pool kernel instance (LaunchParams::pool_T
// needs grid * slots float4).
uint32_t wpool_slots(int waves, bool sparse);
// Waves per workgroup of the wave-pool instance: 1 for dense media; sparse media run
// several wave-private pools per workgroup that share one LDS copy of the launch
// parameters and the empty-region mask.  A wave-pool grid (in waves) is a multiple.
uint32_t wpool_wpg(int waves, bool sparse);
// regenerationSK with the RNG bound to the persistent thread (CVR_OPT_RNG_BINDING 1):
// `grid` one-wave workgroups, path ids from the launch's single queue head.
hipError_t launch_regen_thread(const MediumParams& m, const LaunchParams& L, bool scatter_eps, uint32_t grid,
                               hipStream_t s);
// streamingSK / sortingSK with the thread-bound RNG (CVR_OPT_RNG_BINDING 1): blocks of 256 threads
hipError_t launch_stream_thread(const MediumParams& m, const LaunchParams& L, bool sorting, uint32_t grid,
                                hipStream_t s);
// streamingMK with the thread-bound RNG (CVR_OPT_RNG_BINDING 1): the reference's regenerate /
// extend pair per iteration of a host loop, 256-thread blocks, one slot per thread.
struct SmkSlots {
  float4* a;     // (o, image_id bits)
  float4* b;     // (d, segments bits)
  float4* t;     // (T, 0)
  uint8_t* act;  // path active
};
hipError_t launch_smk_regen(const LaunchParams& L, const SmkSlots& out, uint4* st0, uint2* st1, uint32_t* ctl,
                            uint32_t grid, hipStream_t s);
hipError_t launch_smk_extend(const MediumParams& m, const LaunchParams& L, const SmkSlots& in, const SmkSlots& out,
                             uint4* st0, uint2* st1, uint32_t* ctl, uint32_t grid, hipStream_t s);
hipError_t launch_naive_mk(const MediumParams& m, const LaunchParams& L, hipStream_t s);
// naiveMK with the reference's compaction count (CVR_OPT_MK_COMPACTION 1):
// d_init over the tile's pixels, then one d_extend launch per bounce; `st`
// holds 3 float4 per pixel, `live` one flag, `ctl` the bounce's survivors.
struct MkCtl {
  uint32_t count;   // live paths after the bounce
  uint32_t max_id;  // highest live pixel id (the one end - begin - 1 drops)
};
hipError_t launch_mk_init(const MediumParams& m, const LaunchParams& L, uint32_t iteration, float4* st,
                          uint32_t* live, hipStream_t s);
hipError_t launch_mk_extend(const MediumParams& m, const LaunchParams& L, uint32_t iteration, uint32_t depth,
                            float4* st, uint32_t* live, MkCtl* ctl, hipStream_t s);
hipError_t launch_image_to_host(const float* src, float* dst, size_t n, float scale, hipStream_t s);
hipError_t launch_blocks_to_host(const float* src, float* dst, uint32_t w, uint32_t h, uint32_t rank, uint32_t world,
                                 float scale, hipStream_t s);
hipError_t launch_build_bounds(const float* density, uint32_t rx, uint32_t ry, uint32_t rz, uint32_t bshift,
                               float max_density, uint8_t* bounds, hipStream_t s);
// Sparse medium: cell-leaf pool (`coords`: 3 u32 leaf coordinates per slot,
// slot 0 the zero leaf) and brick words (`cell_slot`: per leaf, its slot or 0).
// `m` carries the leaf table/pools and the brick geometry (bshift <= 3).
hipError_t launch_build_sparse(const MediumParams& m, const uint32_t* coords, size_t n_cell_leaves,
                               const uint32_t* cell_slot, uint32_t bnz, float max_density, int unbounded,
                               float4* cells, uint32_t* sbounds, hipStream_t s);
hipError_t launch_build_cells(const float* density, uint32_t rx, uint32_t ry, uint32_t rz, float4* cells,
                              hipStream_t s);
hipError_t launch_tile_to_image(const float4* tile, uint32_t tw, uint32_t th, float4* image, uint32_t iw,
                                uint32_t ox, uint32_t oy, float scale, hipStream_t s);

}  // namespace cvr
