"""CVR_OPT_RNG_BINDING = 1: regenerationSK, streamingSK and sortingSK with the reference's thread-bound
RNG (RegenerationVolPTsk_kernel.cuh:146-232): Rng(seed + tid) per
persistent thread, a roulette draw after an escape, the isect kept across a
thread's paths.

The oracle restates it for lockstep threads taking path ids in thread order
(oracle_render_thread_bound); a one-wave launch of k_regen_thread produces
exactly that order, so it is compared with the oracle pixel by pixel and
counter by counter.  Larger launches assign paths to threads by timing (as the
reference does): checked for completeness and against the path-bound image
statistically.
"""
import numpy as np
import pytest

from parity_util import NTHREADS, assert_pixels_close


def _bucky_oracle(cvr, oracle_mod):
    s = cvr.Scene.synthetic("bucky")
    return s, oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)


@pytest.mark.parametrize("seed", [0, 77])
def test_oracle_thread_bound_with_a_thread_per_path_is_path_bound(cvr, oracle_mod, seed):
    """With at least as many threads as paths every thread takes one path at
    the first iteration, path i on thread i, so Rng(seed + tid) is the
    path-bound stream: the thread-bound restatement equals the path-bound
    regenerationSK walk (the extra roulette draw after an escape and the
    carried isect cannot show)."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H * 2
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, seed)
    a, sa = orc.render_thread_bound(L, n, 0, n)
    b, sb = orc.render(L, 0, n, nthreads=NTHREADS)
    assert sa.as_dict() == sb.as_dict()
    assert_pixels_close(a, b, 2)


def test_oracle_thread_bound_differs_from_path_bound_with_few_threads(cvr, oracle_mod):
    """With 64 threads each thread walks many paths from one stream: the
    image differs from the path-bound one (same paths rendered, other random
    numbers), the path count and the pixel coverage do not."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H * 2
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    a, sa = orc.render_thread_bound(L, 64, 0, n)
    b, sb = orc.render(L, 0, n, nthreads=NTHREADS)
    assert sa.paths == sb.paths == n and sa.truncated == 0
    assert sa.steps != sb.steps
    assert not np.array_equal(a, b)
    assert abs(a[..., :3].mean() - b[..., :3].mean()) < 0.1 * b[..., :3].mean()


def _ctx(cvr, scene, W, H, grid):
    ctx = cvr.Context(0, "regenerationSK")
    ctx.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_option(cvr.OPT_RNG_BINDING, 1)
    if grid:
        ctx.set_option(cvr.OPT_GRID, grid)
    ctx.init()
    return ctx, iv, r2v


@pytest.mark.gpu
@pytest.mark.parametrize("scene_name,seed,tiles", [("bucky", 0, (1, 1)), ("hetvol", 5, (1, 1)), ("bucky", 3, (2, 2))])
def test_one_wave_thread_bound_launch_matches_oracle(cvr, oracle_mod, scene_name, seed, tiles):
    s = cvr.Scene.synthetic(scene_name)
    orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    W = H = 48
    iters = 3
    ctx, iv, r2v = _ctx(cvr, s, W, H, grid=1)
    ctx.set_seed(seed)
    img, st = ctx.render_image(W, H, tiles, iters)
    tw, th = W // tiles[0], H // tiles[1]
    n = tw * th * iters
    ref = np.zeros((H, W, 4), np.float32)
    tot = dict(paths=0, segments=0, steps=0, density=0, albedo=0, escaped=0)
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * (k // tiles[0])
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), 2, (seed + k * n) & 0xFFFFFFFF)
        tile, rst = orc.render_thread_bound(L, 64, 0, n)
        ref[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        for key in tot:
            tot[key] += getattr(rst, key)
    for key, v in tot.items():
        assert getattr(st, key) == v, key
    assert_pixels_close(img, ref, iters, f"thread-bound {scene_name}")
    assert st.albedo > 0


@pytest.mark.gpu
def test_full_grid_thread_bound_renders_every_path(cvr):
    """The default grid (16 waves per CU): every path is rendered exactly
    once and the image agrees with the path-bound render in the mean (the
    thread-bound streams are other random numbers, so only statistically)."""
    s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    W = H = 128
    iters = 16
    tb, _, _ = _ctx(cvr, s, W, H, grid=0)
    img, st = tb.render_image(W, H, (1, 1), iters)
    assert st.paths == W * H * iters and st.truncated == 0
    pb = cvr.Context(0, "regenerationSK")
    pb.set_medium(s.medium)
    iv, r2v = cvr.default_camera(W, H)
    pb.set_camera(iv, r2v, (W, H))
    pb.init()
    ref, sr = pb.render_image(W, H, (1, 1), iters)
    a, b = np.nanmean(img[..., :3]), np.nanmean(ref[..., :3])
    assert abs(a - b) < 0.02 * b, (a, b)
    assert abs(st.steps - sr.steps) < 0.02 * sr.steps


@pytest.mark.gpu
def test_thread_bound_is_for_the_persistent_and_block_kernels(cvr):
    s = cvr.Scene.synthetic("bucky")
    ctx = cvr.Context(0, "naiveSK")
    ctx.set_medium(s.medium)
    iv, r2v = cvr.default_camera(32, 32)
    ctx.set_camera(iv, r2v, (32, 32))
    ctx.set_option(cvr.OPT_RNG_BINDING, 1)
    with pytest.raises(cvr.CvrError) as e:
        ctx.render_image(32, 32, (1, 1), 1)
    assert "regenerationSK" in str(e.value) and "streamingMK" in str(e.value)


# ---- streamingSK / sortingSK with the thread-bound RNG ------------------------------
@pytest.mark.parametrize("sorting", [False, True])
def test_oracle_stream_thread_bound_renders_every_path_once(cvr, oracle_mod, sorting):
    """One block of 256 lockstep threads (StreamingVolPTsk_kernel.cuh:328-349): every path id
    is taken exactly once and ends (escape or roulette), the image differs from the path-bound
    render only by which random numbers each path draws, and sortingSK's deferred albedo and
    drain-mode extend give yet another image with the same path count."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H * 2
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    a, sa = orc.render_stream_thread_bound(L, 256, 0, n, sorting)
    b, sb = orc.render(L, 0, n, nthreads=NTHREADS)
    assert sa.paths == sb.paths == n and sa.truncated == 0
    assert sa.segments > n
    assert not np.array_equal(a, b)
    assert abs(a[..., :3].mean() - b[..., :3].mean()) < 0.1 * b[..., :3].mean()
    other, so = orc.render_stream_thread_bound(L, 256, 0, n, not sorting)
    assert so.paths == n and not np.array_equal(a, other)


def test_oracle_stream_thread_bound_is_seeded_per_thread(cvr, oracle_mod):
    """Rng(seed + tid): seed s with thread t draws the stream of seed s + 1 with thread t - 1,
    so shifting the seed changes the image (the reference's seed++ per tile,
    RenderKernelLauncher.cu:567-575) and the same seed reproduces it bit for bit."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H
    iv, r2v = cvr.default_camera(W, H)
    a, _ = orc.render_stream_thread_bound(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 7), 256, 0, n)
    b, _ = orc.render_stream_thread_bound(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 7), 256, 0, n)
    c, _ = orc.render_stream_thread_bound(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 8), 256, 0, n)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)


def _stream_ctx(cvr, scene, kernel, W, H, grid):
    ctx = cvr.Context(0, kernel)
    ctx.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_option(cvr.OPT_RNG_BINDING, 1)
    if grid:
        ctx.set_option(cvr.OPT_GRID, grid)
    ctx.init()
    return ctx, iv, r2v


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,scene_name,seed,tiles", [("streamingSK", "bucky", 0, (1, 1)),
                                                         ("sortingSK", "bucky", 0, (1, 1)),
                                                         ("streamingSK", "hetvol", 5, (1, 1)),
                                                         ("sortingSK", "hetvol", 5, (2, 1)),
                                                         ("streamingSK", "manix", 3, (2, 2))])
def test_one_block_stream_thread_bound_launch_matches_oracle(cvr, oracle_mod, kernel, scene_name, seed, tiles):
    """A one-block launch of k_stream_thread (CVR_OPT_GRID 1) is the oracle's lockstep block:
    same counters, same pixels up to the order of the fp32 atomic adds; each tile with the
    streaming kernels' seed + 1 per tile (RenderKernelLauncher.cu:567-575)."""
    if scene_name == "manix":
        s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    else:
        s = cvr.Scene.synthetic(scene_name)
    orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    W = H = 48
    iters = 2
    ctx, iv, r2v = _stream_ctx(cvr, s, kernel, W, H, grid=1)
    ctx.set_seed(seed)
    img, st = ctx.render_image(W, H, tiles, iters)
    tw, th = W // tiles[0], H // tiles[1]
    n = tw * th * iters
    ref = np.zeros((H, W, 4), np.float32)
    tot = dict(paths=0, segments=0, steps=0, density=0, albedo=0, escaped=0)
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * (k // tiles[0])
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), 2, (seed + k) & 0xFFFFFFFF)
        tile, rst = orc.render_stream_thread_bound(L, 256, 0, n, kernel == "sortingSK")
        ref[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        for key in tot:
            tot[key] += getattr(rst, key)
    for key, v in tot.items():
        assert getattr(st, key) == v, key
    assert_pixels_close(img, ref, iters, f"thread-bound {kernel} {scene_name}")
    assert st.albedo > 0
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["streamingSK", "sortingSK"])
def test_full_grid_stream_thread_bound_renders_every_path(cvr, kernel):
    """The default grid (2 blocks per CU): every path is rendered exactly once and the image
    agrees with the path-bound render in the mean (other random numbers, so statistically)."""
    s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    W = H = 128
    iters = 16
    tb, iv, r2v = _stream_ctx(cvr, s, kernel, W, H, grid=0)
    img, st = tb.render_image(W, H, (1, 1), iters)
    assert st.paths == W * H * iters and st.truncated == 0
    pb = cvr.Context(0, kernel)
    pb.set_medium(s.medium)
    pb.set_camera(iv, r2v, (W, H))
    pb.init()
    ref, sr = pb.render_image(W, H, (1, 1), iters)
    a, b = np.nanmean(img[..., :3]), np.nanmean(ref[..., :3])
    assert abs(a - b) < 0.03 * b, (a, b)
    tb.close()
    pb.close()


# ---- streamingMK with the thread-bound RNG --------------------------------------------
def test_oracle_smk_thread_bound_with_a_slot_per_path_is_path_bound(cvr, oracle_mod):
    """One block of 256 threads: every path id is taken exactly once and ends; a new path starts
    from Rng(seed + path_id) as in the path-bound walk, but once compaction moves it to another
    slot it draws from that slot's thread state, so the image differs from the path-bound one
    (same paths, other random numbers after the first segment) while its mean agrees; the
    lockstep restatement is deterministic."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H * 2
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    a, sa = orc.render_smk_thread_bound(L, 256, 0, n)
    b, sb = orc.render(L, 0, n, nthreads=NTHREADS)
    assert sa.paths == sb.paths == n and sa.truncated == 0
    assert sa.segments > n
    assert not np.array_equal(a, b)
    assert abs(a[..., :3].mean() - b[..., :3].mean()) < 0.1 * b[..., :3].mean()
    a2, sa2 = orc.render_smk_thread_bound(L, 256, 0, n)
    assert np.array_equal(a, a2) and sa.as_dict() == sa2.as_dict()


def test_oracle_smk_thread_bound_differs_from_streaming_sk(cvr, oracle_mod):
    """streamingMK seeds a new path's RNG from its path id and keeps the states with the
    threads; streamingSK seeds the threads once (Rng(seed + tid)): other numbers, other image."""
    s, orc = _bucky_oracle(cvr, oracle_mod)
    W = H = 32
    n = W * H
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 3)
    a, sa = orc.render_smk_thread_bound(L, 256, 0, n)
    b, sb = orc.render_stream_thread_bound(L, 256, 0, n)
    assert sa.paths == sb.paths == n
    assert not np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("scene_name,seed,tiles", [("bucky", 0, (1, 1)), ("hetvol", 5, (2, 1)),
                                                   ("manix", 3, (2, 2))])
def test_one_block_smk_thread_bound_launch_matches_oracle(cvr, oracle_mod, scene_name, seed, tiles):
    """A one-block thread-bound streamingMK render (CVR_OPT_GRID 1: k_smk_regen / k_smk_extend
    per iteration of the host loop) is the oracle's lockstep block: same counters, same pixels
    up to the order of the fp32 atomic adds; tile k with seed + k * n_paths (reset(),
    RenderKernelLauncher.cu:475-482)."""
    if scene_name == "manix":
        s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    else:
        s = cvr.Scene.synthetic(scene_name)
    orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    W = H = 48
    iters = 2
    ctx, iv, r2v = _stream_ctx(cvr, s, "streamingMK", W, H, grid=1)
    ctx.set_seed(seed)
    img, st = ctx.render_image(W, H, tiles, iters)
    tw, th = W // tiles[0], H // tiles[1]
    n = tw * th * iters
    ref = np.zeros((H, W, 4), np.float32)
    tot = dict(paths=0, segments=0, steps=0, density=0, albedo=0, escaped=0)
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * (k // tiles[0])
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), 2, (seed + k * n) & 0xFFFFFFFF)
        tile, rst = orc.render_smk_thread_bound(L, 256, 0, n)
        ref[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        for key in tot:
            tot[key] += getattr(rst, key)
    for key, v in tot.items():
        assert getattr(st, key) == v, key
    assert_pixels_close(img, ref, iters, f"thread-bound streamingMK {scene_name}")
    assert st.albedo > 0
    ctx.close()


@pytest.mark.gpu
def test_full_grid_smk_thread_bound_renders_every_path(cvr):
    """The default grid (2 blocks per CU): every path is rendered exactly once and the image
    agrees with the path-bound streamingMK render in the mean (other random numbers)."""
    s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    W = H = 128
    iters = 8
    tb, iv, r2v = _stream_ctx(cvr, s, "streamingMK", W, H, grid=0)
    img, st = tb.render_image(W, H, (1, 1), iters)
    assert st.paths == W * H * iters and st.truncated == 0
    pb = cvr.Context(0, "streamingMK")
    pb.set_medium(s.medium)
    pb.set_camera(iv, r2v, (W, H))
    pb.init()
    ref, sr = pb.render_image(W, H, (1, 1), iters)
    a, b = np.nanmean(img[..., :3]), np.nanmean(ref[..., :3])
    assert abs(a - b) < 0.03 * b, (a, b)
    tb.close()
    pb.close()
