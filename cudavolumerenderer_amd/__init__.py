"""MI355X-native volumetric path tracer (the hot path of Fe0437/CudaVolumeRenderer).

The renderer is libcvr.so (HIP for gfx950 behind the C ABI in include/cvr.h);
this package is its ctypes binding plus the multi-GPU driver.  There is no
CPU fallback: on a machine without a GPU, Context() raises.
"""
from ._lib import (  # noqa: F401
    KERNELS, NAIVE_SK, NAIVE_MK, REGENERATION_SK, STREAMING_MK, STREAMING_SK, SORTING_SK,
    OPT_MAX_SEGMENTS, OPT_CHUNK, OPT_EVENT_THRESHOLD, OPT_GRID, OPT_SCATTER_EPS,
    OPT_SCHEDULER, OPT_POOL, OPT_TIMING, OPT_CELLS, OPT_WAVES, OPT_ORDER, OPT_QUEUES, OPT_BOUNDS, OPT_TAIL, OPT_BATCH, OPT_RNG_BINDING, OPT_MORTON, OPT_WORLD_TO_AABB, OPT_MK_COMPACTION, OPT_SUBQUEUES, OPT_DRAIN, OPT_INFLIGHT, OPT_FRAME_FLUSH, OPT_UNIFORM_ALBEDO, OPT_WAVE_PAIR, OPT_SAMPLE_ORDER, OPT_EMPTY_MASK, OPT_COUNT_WORDS,
    PATH_RECORD_DTYPE, CvrError, Context, MediumDesc, PinnedImage, Scene, Stats, default_camera, load,
    medium_from_arrays, tile_origin, tiling, write_hdr, LIB_PATH,
)

__all__ = [
    "KERNELS", "Context", "Scene", "MediumDesc", "Stats", "CvrError", "PinnedImage", "default_camera", "tiling",
    "tile_origin", "write_hdr", "medium_from_arrays", "load", "LIB_PATH", "PATH_RECORD_DTYPE",
]
