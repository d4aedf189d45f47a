"""HIP path vs CPU oracle parity (run on the MI355X box: pytest -m gpu).

Contract:
  * per path: bit-exact (image_id, flags, T bits, segment/step/tap counts);
  * per pixel: the only difference is the order of fp32 atomic additions, so
    |gpu - cpu| <= 2 (n - 1) 2^-24 max(gpu, cpu) for a pixel that receives
    n <= iterations contributions (plus 1e-30 for zeros);
  * counters (segments, Woodcock steps, density/albedo taps, escapes): equal.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)


def make_ctx(cvr, scene, W, H, kernel, seed=0, cells=1):
    ctx = cvr.Context(0, kernel)
    ctx.set_option(cvr.OPT_CELLS, cells)
    ctx.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_seed(seed)
    ctx.init()
    return ctx, iv, r2v


def oracle_for(oracle_mod, scene):
    return oracle_mod.Oracle.from_medium_desc(scene.medium, scene.density, scene.albedo)


def oracle_image(oracle_mod, orc, iv, r2v, W, H, tiles, iters, kernel, seed=0):
    """The reference's tile loop restated with the oracle (CudaVolPath.cpp:249-347)."""
    tw, th = W // tiles[0], H // tiles[1]
    n_paths = tw * th * iters
    img = np.zeros((H, W, 4), np.float32)
    stats = {}
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * int(np.float32(k) / np.float32(tiles[0]))
        # per-tile seed advance of each launcher's reset() (RenderKernelLauncher.cu:359,480,573,664)
        sb = {2: seed + k * n_paths, 3: seed + k * n_paths, 4: seed + k, 5: seed + k}.get(kernel, seed) & 0xFFFFFFFF
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), kernel, sb)
        tile, st = orc.render(L, 0, n_paths, nthreads=NTHREADS)
        img[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        for key, v in st.as_dict().items():
            stats[key] = stats.get(key, 0) + v
    return img, stats


def assert_pixels_close(gpu, cpu, iters):
    # NaN pixels are reference behaviour: they must
    # coincide exactly; every other pixel obeys the summation-order bound.
    ng, nc = np.isnan(gpu), np.isnan(cpu)
    assert (ng == nc).all(), f"NaN pattern differs: gpu {ng.sum()} cpu {nc.sum()}"
    gpu = np.where(ng, 0, gpu)
    cpu = np.where(nc, 0, cpu)
    bound = 2.0 * max(iters - 1, 1) * 2.0 ** -24 * np.maximum(np.abs(gpu), np.abs(cpu)) + 1e-30
    diff = np.abs(gpu.astype(np.float64) - cpu.astype(np.float64))
    bad = diff > bound
    assert not bad.any(), (f"{bad.sum()} pixels out of tolerance; worst diff {diff.max()} "
                           f"at {np.unravel_index(np.argmax(diff - bound), diff.shape)}")


SCENES = {
    "bucky": dict(name="bucky"),
    "manix_small": dict(name="manix", dims=(64, 58, 64)),
    "hetvol": dict(name="hetvol"),
}


@pytest.fixture(scope="module")
def scenes(cvr):
    return {k: cvr.Scene.synthetic(v["name"], 0, v.get("dims")) for k, v in SCENES.items()}


@pytest.mark.parametrize("scene_key", list(SCENES))
@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "streamingSK", "naiveMK"])
@pytest.mark.parametrize("cells", [1, 0])
def test_per_path_bit_exact(cvr, oracle_mod, scenes, scene_key, kernel, cells):
    scene = scenes[scene_key]
    W = H = 64
    iters = 3
    ctx, iv, r2v = make_ctx(cvr, scene, W, H, kernel, seed=7, cells=cells)
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    n = W * H * iters
    g = ctx.trace_paths(0, n)
    orc = oracle_for(oracle_mod, scene)
    kid = cvr.KERNELS.index(kernel)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, 7), 0, n)
    for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
        mism = np.nonzero(g[f] != c[f])[0]
        assert mism.size == 0, f"{f} differs for {mism.size} paths, first path {mism[:5]}"
    tb, cb = g["T"].view(np.uint32), c["T"].view(np.uint32)
    mism = np.nonzero((tb != cb).any(axis=1))[0]
    assert mism.size == 0, f"T bits differ for {mism.size} paths, first {mism[:5]}"
    assert c["n_density"].sum() > 0 and (c["flags"] & 1).any()
    if kernel == "naiveMK":  # init misses (T = 1) and escapes after bounces both occur
        assert ((c["flags"] & 4) != 0).any() and ((c["flags"] & 5) == 1).any()


@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "streamingSK", "sortingSK", "streamingMK", "naiveMK"])
@pytest.mark.parametrize("tiles", [(1, 1), (4, 2), (3, 3)])
def test_render_image_matches_oracle(cvr, oracle_mod, scenes, kernel, tiles):
    scene = scenes["bucky"]
    W, H, iters = 96, 96, 4  # 96/3 = 32, 96/4 = 24, 96/2 = 48
    ctx, iv, r2v = make_ctx(cvr, scene, W, H, kernel)
    img, st = ctx.render_image(W, H, tiles, iters)
    ref, rst = oracle_image(oracle_mod, oracle_for(oracle_mod, scene), iv, r2v, W, H, tiles, iters,
                            cvr.KERNELS.index(kernel))
    assert_pixels_close(img, ref, iters)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "truncated"):
        assert getattr(st, k) == rst[k], k


@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "streamingSK", "streamingMK"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_render_tiles_sharded_sums_to_render_image(cvr, scenes, kernel, world):
    """C4's decomposition: tile k -> rank k mod world (cvr_render_tiles).  The
    ranks' images are disjoint and sum to the sequential tile loop's; every
    rank's seed ends where the full loop leaves it."""
    scene = scenes["manix_small"]
    W, H, iters, tiles = 128, 96, 3, (4, 2)
    ref, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=11)
    img0, st0 = ref.render_image(W, H, tiles, iters)
    total = np.zeros_like(img0)
    steps = paths = 0
    for r in range(world):
        ctx, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=11)
        img, st = ctx.render_tiles(W, H, tiles, iters, r, world)
        mine = np.zeros((H, W), bool)
        for k in range(r, 8, world):
            ox, oy = (W // 4) * (k % 4), (H // 2) * (k // 4)
            mine[oy:oy + H // 2, ox:ox + W // 4] = True
        assert not np.nan_to_num(img)[~mine].any()
        total += np.nan_to_num(img)
        steps += st.steps
        paths += st.paths
        assert ctx.get_seed() == ref.get_seed()
    assert steps == st0.steps and paths == st0.paths
    assert_pixels_close(total, np.nan_to_num(img0), iters)


@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK", "naiveSK"])
@pytest.mark.parametrize("world", [2, 3])
def test_tile_path_shards_sum_to_render_image(cvr, scenes, kernel, world):
    """bench.py --shard tilepaths: rank r renders path-id shard r of every
    tile (cvr_set_path_range + cvr_render_tiles, each tile with its own seed);
    the ranks' images sum to the sequential tile loop's (rgb; w is a plain
    store per render)."""
    from cudavolumerenderer_amd.distributed import shard_range
    scene = scenes["manix_small"]
    W, H, iters, tiles = 128, 96, 3, (4, 2)
    ref, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=5)
    img0, st0 = ref.render_image(W, H, tiles, iters)
    total = np.zeros_like(img0[..., :3])
    steps = paths = 0
    for r in range(world):
        ctx, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=5)
        ctx.set_path_range(*shard_range((W // 4) * (H // 2) * iters, r, world))
        img, st = ctx.render_tiles(W, H, tiles, iters, 0, 1)
        total += np.nan_to_num(img[..., :3])
        steps += st.steps
        paths += st.paths
    assert steps == st0.steps and paths == st0.paths
    assert_pixels_close(total, np.nan_to_num(img0[..., :3]), world * iters)


def test_c1_bucky_256_4it(cvr, oracle_mod, scenes):
    """BASELINE config C1 (bucky 32^3, 256x256, 4 iterations) through naiveSK."""
    scene = scenes["bucky"]
    ctx, iv, r2v = make_ctx(cvr, scene, 256, 256, "naiveSK")
    img, st = ctx.render_image(256, 256, (1, 1), 4)
    ref, rst = oracle_image(oracle_mod, oracle_for(oracle_mod, scene), iv, r2v, 256, 256, (1, 1), 4, 0)
    assert_pixels_close(img, ref, 4)
    assert st.paths == 256 * 256 * 4 and st.steps == rst["steps"]


def test_scheduler_knobs_do_not_change_results(cvr, scenes):
    scene = scenes["manix_small"]
    W = H = 128
    base = None
    # (chunk, event/refill threshold, grid, scheduler, pool): the single
    # persistent kernel and the wavefront scheduler with pools from 256 slots
    # (hundreds of events/track iterations) up must all give the same result.
    # sched 0 = persistent kernel (with work orders/queues), 1 = wavefront pair, 3 = wave pool, 4 = per item
    for chunk, thresh, grid, sched, pool, order, queues in [
            (128, 56, 0, 0, 1 << 21, 1, 8), (128, 16, 0, 0, 1 << 21, 0, 1), (64, 1, 0, 0, 1 << 21, 1, 3),
            (256, 64, 0, 0, 1 << 21, 1, 1), (32, 8, 7, 0, 1 << 21, 1, 8), (100, 30, 3, 0, 1 << 21, 0, 1),
            (128, 16, 0, 1, 1 << 21, 1, 8), (64, 1, 0, 1, 256, 1, 8), (256, 64, 0, 1, 4096, 1, 8),
            (32, 8, 7, 1, 1000, 1, 8),
            # round 5: sched 3 = the wave pool (every id's default), 4 = one path per work-item
            (128, 56, 0, 3, 1 << 21, 1, 8), (64, 56, 0, 3, 1 << 21, 0, 1), (256, 56, 0, 4, 1 << 21, 1, 8)]:
        ctx, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
        ctx.set_option(cvr.OPT_CHUNK, chunk)
        ctx.set_option(cvr.OPT_EVENT_THRESHOLD, thresh)
        ctx.set_option(cvr.OPT_GRID, grid)
        ctx.set_option(cvr.OPT_SCHEDULER, sched)
        ctx.set_option(cvr.OPT_POOL, pool)
        ctx.set_option(cvr.OPT_ORDER, order)
        ctx.set_option(cvr.OPT_QUEUES, queues)
        img, st = ctx.render_image(W, H, (1, 1), 4)
        key = (st.paths, st.segments, st.steps, st.density, st.albedo, st.escaped)
        if base is None:
            base = (img, key)
        else:
            assert key == base[1]
            assert_pixels_close(img, base[0], 4)


def test_naive_without_eps_equals_regeneration(cvr, scenes):
    """The two schedulers differ only by the scatter -eps."""
    scene = scenes["hetvol"]
    W = H = 96
    a, _, _ = make_ctx(cvr, scene, W, H, "naiveSK")
    a.set_option(cvr.OPT_SCATTER_EPS, 0)
    b, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
    ia, sa = a.render_image(W, H, (1, 1), 2)
    ib, sb = b.render_image(W, H, (1, 1), 2)
    assert (sa.steps, sa.escaped) == (sb.steps, sb.escaped)
    assert_pixels_close(ia, ib, 2)


@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK"])
def test_path_range_shards_sum_to_whole(cvr, scenes, kernel):
    scene = scenes["manix_small"]
    W = H = 128
    iters = 4
    n = W * H * iters
    whole, _, _ = make_ctx(cvr, scene, W, H, kernel)
    whole.set_resolution(W, H)
    whole.set_iterations(iters)
    whole.clear_output()
    whole.launch_render()
    sw = whole.stats()
    full = whole.copy_output(W, H)
    parts = np.zeros_like(full)
    tot = 0
    bounds = [0, n // 3, n // 2 + 17, n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        ctx, _, _ = make_ctx(cvr, scene, W, H, kernel)
        ctx.set_resolution(W, H)
        ctx.set_iterations(iters)
        ctx.set_path_range(a, b - a)
        ctx.clear_output()
        ctx.launch_render()
        tot += ctx.stats().steps
        parts[..., :3] += ctx.copy_output(W, H)[..., :3]
    assert tot == sw.steps
    assert_pixels_close(parts[..., :3], full[..., :3], 3 * iters)


def test_c2_manix_1024_full_size_vs_oracle(cvr, oracle_mod):
    """BASELINE config C2 at full size: manix proxy 256x230x256, 1024^2, 20 it,
    regenerationSK.  The oracle renders the same 20.97 M paths on the host."""
    scene = cvr.Scene.synthetic("manix")
    W = H = 1024
    ctx, iv, r2v = make_ctx(cvr, scene, W, H, "regenerationSK")
    img, st = ctx.render_image(W, H, (1, 1), 20)
    assert st.paths == W * H * 20 and st.truncated == 0
    ref, rst = oracle_image(oracle_mod, oracle_for(oracle_mod, scene), iv, r2v, W, H, (1, 1), 20, 2)
    for k in ("segments", "steps", "density", "albedo", "escaped"):
        assert getattr(st, k) == rst[k], k
    assert_pixels_close(img, ref, 20)


@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK"])
def test_c3_hetvol_1024_full_size_vs_oracle(cvr, oracle_mod, kernel):
    """BASELINE config C3 at full size: hetvol proxy 128x128x50 (seed 800),
    1024^2, Woodcock tracking through the regeneration and streaming
    schedulers; the oracle renders the same paths on the host."""
    scene = cvr.Scene.synthetic("hetvol")
    W = H = 1024
    iters = 8
    ctx, iv, r2v = make_ctx(cvr, scene, W, H, kernel)
    img, st = ctx.render_image(W, H, (1, 1), iters)
    assert st.paths == W * H * iters and st.truncated == 0
    ref, rst = oracle_image(oracle_mod, oracle_for(oracle_mod, scene), iv, r2v, W, H, (1, 1), iters,
                            cvr.KERNELS.index(kernel))
    for k in ("segments", "steps", "density", "albedo", "escaped"):
        assert getattr(st, k) == rst[k], k
    assert_pixels_close(img, ref, iters)


def test_c4_manix_2048_256it_tiles_full_size(cvr, oracle_mod):
    """BASELINE config C4 at full size: manix proxy, 2048^2, 256 iterations,
    --number-of-tiles 4 2 (1.07 G paths).  Size-independent checks: the
    8-way tile-sharded render (tile k -> rank k) sums to the sequential tile
    loop with identical counters, and sampled path ranges of every tile are
    bit-exact against the oracle with that tile's seed."""
    scene = cvr.Scene.synthetic("manix")
    W = H = 2048
    iters, tiles = 256, (4, 2)
    tw, th = W // 4, H // 2
    n_paths = tw * th * iters
    ref, iv, r2v = make_ctx(cvr, scene, W, H, "regenerationSK")
    img0, st0 = ref.render_image(W, H, tiles, iters)
    assert st0.paths == W * H * iters and st0.truncated == 0
    total = np.zeros_like(img0)
    steps = 0
    for r in range(8):
        ctx, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
        img, st = ctx.render_tiles(W, H, tiles, iters, r, 8)
        total += np.nan_to_num(img)
        steps += st.steps
        ctx.close()
    assert steps == st0.steps
    assert_pixels_close(total, np.nan_to_num(img0), iters)
    orc = oracle_for(oracle_mod, scene)
    ctx, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
    ctx.set_resolution(tw, th)
    ctx.set_iterations(iters)
    for k in range(8):
        ox, oy = tw * (k % 4), th * (k // 4)
        seed = (k * n_paths) & 0xFFFFFFFF
        ctx.set_offset(ox, oy)
        ctx.set_seed(seed)
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), 2, seed)
        for first in (0, n_paths // 2 + 12345, n_paths - 2048):
            g = ctx.trace_paths(first, 2048)
            c = orc.trace_paths(L, first, 2048)
            for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
                assert (g[f] == c[f]).all(), (k, first, f)
            assert (g["T"].view(np.uint32) == c["T"].view(np.uint32)).all(), (k, first)


def test_errors_are_reported_not_fatal(cvr, scenes):
    with pytest.raises(cvr.CvrError) as e:
        cvr.Context(0, 9)
    assert "unknown kernel" in str(e.value)
    ctx = cvr.Context(0, "regenerationSK")
    with pytest.raises(cvr.CvrError) as e:
        ctx.launch_render()
    assert "CVR_ERR_STATE" in str(e.value)
    with pytest.raises(cvr.CvrError):
        ctx.set_option(cvr.OPT_EVENT_THRESHOLD, 0)
    # n_paths must fit the reference's uint32 path ids whichever of
    # setNIterations / setResolution comes last
    ctx.set_resolution(16, 16)
    ctx.set_iterations(256)
    with pytest.raises(cvr.CvrError) as e:
        ctx.set_resolution(4096, 4096)
    assert "uint32" in str(e.value)
    with pytest.raises(cvr.CvrError):
        ctx.set_iterations(1 << 30)


@pytest.mark.parametrize("scene_key", ["manix_small", "hetvol"])
@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK"])
def test_brick_bounds_do_not_change_results(cvr, scenes, scene_key, kernel):
    """Brick bounds (MediumParams::bounds) only skip fetches whose test is
    decided anyway: per-path records are bit-identical for every brick size
    and with the bounds off; only the fetch count changes."""
    scene = scenes[scene_key]
    W = H = 64
    iters = 2
    iv, r2v = cvr.default_camera(W, H)
    want = None
    for bshift in [0, 1, 2, 3, 5]:
        ctx = cvr.Context(0, kernel)
        ctx.set_option(cvr.OPT_BOUNDS, bshift)
        ctx.set_medium(scene.medium)
        ctx.set_camera(iv, r2v, (W, H))
        ctx.init()
        ctx.set_resolution(W, H)
        ctx.set_iterations(iters)
        rec = ctx.trace_paths(0, W * H * iters)
        ctx.clear_output()
        ctx.launch_render()
        st = ctx.stats()
        assert st.density == rec["n_density"].sum()
        if bshift == 0:
            assert st.fetches == st.density
            want = rec
            continue
        assert st.fetches <= st.density
        if bshift <= 2:
            assert st.fetches < st.density
        for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
            assert np.array_equal(rec[f], want[f]), (bshift, f)
        assert np.array_equal(rec["T"].view(np.uint32), want["T"].view(np.uint32)), bshift


@pytest.mark.parametrize("scene_key", ["manix_small", "hetvol", "bucky"])
def test_pool_scheduler_matches_persistent(cvr, scenes, scene_key):
    """Scheduler 2 (workgroup path pool in LDS) renders exactly the paths of
    the persistent kernel: same counters, same pixels up to fp32 atomic
    order, for several tails, grids and chunk sizes."""
    scene = scenes[scene_key]
    W = H = 128
    ref, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
    ref.set_option(cvr.OPT_SCHEDULER, 0)  # the per-wave persistent kernel
    img0, st0 = ref.render_image(W, H, (1, 1), 4)
    key0 = (st0.paths, st0.segments, st0.steps, st0.density, st0.albedo, st0.escaped, st0.fetches)
    for tail, grid, chunk, order in [(16, 0, 256, 1), (0, 0, 64, 1), (48, 5, 256, 1), (64, 1, 7, 0),
                                     (16, 3, 1, 1)]:
        ctx, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
        ctx.set_option(cvr.OPT_SCHEDULER, 2)
        ctx.set_option(cvr.OPT_TAIL, tail)
        ctx.set_option(cvr.OPT_GRID, grid)
        ctx.set_option(cvr.OPT_CHUNK, chunk)
        ctx.set_option(cvr.OPT_ORDER, order)
        img, st = ctx.render_image(W, H, (1, 1), 4)
        key = (st.paths, st.segments, st.steps, st.density, st.albedo, st.escaped, st.fetches)
        assert key == key0, (tail, grid, chunk, order)
        assert_pixels_close(img, img0, 4)


@pytest.mark.parametrize("scene_key", ["manix_small", "hetvol", "bucky"])
def test_wave_pool_scheduler_matches_persistent(cvr, scenes, scene_key):
    """Scheduler 3 (wave-private path pool in LDS) renders exactly the paths
    of the persistent kernel for several swap batches, grids and chunks."""
    scene = scenes[scene_key]
    W = H = 128
    ref, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
    ref.set_option(cvr.OPT_SCHEDULER, 0)  # the per-wave persistent kernel
    img0, st0 = ref.render_image(W, H, (1, 1), 4)
    key0 = (st0.paths, st0.segments, st0.steps, st0.density, st0.albedo, st0.escaped, st0.fetches)
    # + the drain-time event rule (CVR_OPT_DRAIN 0 / 1 / 3), the in-flight grid rule
    # (CVR_OPT_INFLIGHT) and the sub-queues per XCD band (CVR_OPT_SUBQUEUES)
    for batch, grid, chunk, order, drain, inflight, sub in [
            (8, 0, 256, 1, 1, 1, 8), (1, 0, 64, 1, 0, 1, 8), (64, 5, 256, 1, 3, 1, 1), (16, 1, 7, 0, 1, 1, 8),
            (32, 3, 1, 1, 0, 1, 3), (8, 0, None, 2, 1, 3, 8), (8, 0, None, 2, 2, 64, 2)]:
        ctx, _, _ = make_ctx(cvr, scene, W, H, "regenerationSK")
        ctx.set_option(cvr.OPT_SCHEDULER, 3)
        ctx.set_option(cvr.OPT_BATCH, batch)
        ctx.set_option(cvr.OPT_GRID, grid)
        if chunk is not None:  # None: the automatic chunk
            ctx.set_option(cvr.OPT_CHUNK, chunk)
        ctx.set_option(cvr.OPT_ORDER, order)
        ctx.set_option(cvr.OPT_DRAIN, drain)
        ctx.set_option(cvr.OPT_INFLIGHT, inflight)
        ctx.set_option(cvr.OPT_SUBQUEUES, sub)
        img, st = ctx.render_image(W, H, (1, 1), 4)
        key = (st.paths, st.segments, st.steps, st.density, st.albedo, st.escaped, st.fetches)
        assert key == key0, (batch, grid, chunk, order, drain, inflight, sub)
        assert_pixels_close(img, img0, 4)
    with pytest.raises(cvr.CvrError):
        ctx.set_option(cvr.OPT_DRAIN, 65)
    with pytest.raises(cvr.CvrError):
        ctx.set_option(cvr.OPT_INFLIGHT, 0)


@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK", "naiveSK"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_block_shards_sum_to_whole_render(cvr, scenes, kernel, world):
    """cvr_set_block_shard (bench.py's strong-scaling shards): the world
    shards of a launch render exactly its paths (counters add up) and their
    framebuffers sum to the unsharded one; on a tile whose sides are not
    multiples of 8 the shards are contiguous path ranges."""
    scene = scenes["manix_small"]
    for W, H in ((128, 96), (100, 60)):
        iters = 3
        whole, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=3)
        whole.set_resolution(W, H)
        whole.set_iterations(iters)
        whole.clear_output()
        whole.launch_render()
        s0 = whole.stats()
        full = whole.copy_output(W, H)
        total = np.zeros_like(full)
        acc = dict(paths=0, steps=0, density=0, albedo=0, escaped=0, segments=0)
        for r in range(world):
            ctx, _, _ = make_ctx(cvr, scene, W, H, kernel, seed=3)
            ctx.set_resolution(W, H)
            ctx.set_iterations(iters)
            ctx.set_block_shard(r, world)
            ctx.clear_output()
            ctx.launch_render()
            st = ctx.stats()
            for k in acc:
                acc[k] += getattr(st, k)
            total[..., :3] += ctx.copy_output(W, H)[..., :3]
            ctx.close()
        for k in acc:
            assert acc[k] == getattr(s0, k), (W, k)
        assert_pixels_close(total[..., :3], full[..., :3], iters)
