"""Several renders in flight on one GPU (bench.py's pipelined mode): contexts
that share one device medium (cvr_share_medium), the pixel-block work order's
permutation (cvr_set_block_order) and the wave pool's automatic dequeue chunk
for small launches (block shards).  All are scheduling only: the RNG is bound
to the path id, so counters are equal and pixels agree up to fp32 summation
order (tests/parity_util.py), here against the CPU oracle and against the
plain single-context render."""
import numpy as np
import pytest

from parity_util import assert_counters_equal, assert_pixels_close, oracle_for_scene

pytestmark = pytest.mark.gpu

W = H = 256
ITERS = 6


def _owner(cvr, scene):
    c = cvr.Context(0, "regenerationSK")
    if scene.is_sparse:
        c.set_medium_sparse(scene.sparse_medium)
    else:
        c.set_medium(scene.medium)
    return c


def _setup(cvr, c):
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    c.init()
    c.set_resolution(W, H)
    c.set_iterations(ITERS)
    return iv, r2v


def _render(c):
    c.clear_output()
    c.launch_render()
    st = c.stats()
    return c.copy_output(W, H), st


@pytest.mark.parametrize("name", ["manix", "hetvol"])
def test_shared_medium_contexts_render_like_the_owner_and_the_oracle(cvr, oracle_mod, name):
    scene = cvr.Scene.synthetic(name)
    a = _owner(cvr, scene)
    iv, r2v = _setup(cvr, a)
    b = cvr.Context(0, "regenerationSK")
    b.share_medium(a)
    _setup(cvr, b)
    b.use_own_stream()
    ia, sa = _render(a)
    ib, sb = _render(b)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "fetches"):
        assert getattr(sa, k) == getattr(sb, k), k
    assert_pixels_close(ib, ia, ITERS, "shared medium")
    orc = oracle_for_scene(oracle_mod, scene)
    ref, rst = orc.render(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0), 0, W * H * ITERS, nthreads=8)
    assert_counters_equal(sb, rst, "shared medium vs oracle")
    assert_pixels_close(ib, ref, ITERS, "shared medium vs oracle")
    b.close()
    a.close()


def test_renders_in_flight_on_two_streams_match(cvr):
    """Launch on three contexts (own streams) back to back without syncs, as
    bench.py's pipelined step does; every image equals the serial one."""
    scene = cvr.Scene.synthetic("manix")
    a = _owner(cvr, scene)
    _setup(cvr, a)
    ref, rs = _render(a)
    ctxs = [a]
    for _ in range(2):
        c = cvr.Context(0, "regenerationSK")
        c.share_medium(a)
        _setup(cvr, c)
        c.use_own_stream()
        ctxs.append(c)
    a.use_own_stream()
    for c in ctxs:
        c.clear_output()
        c.launch_render()
    for c in ctxs:
        c.synchronize()
        img, st = c.copy_output(W, H), c.stats()
        assert st.steps == rs.steps and st.escaped == rs.escaped
        assert_pixels_close(img, ref, ITERS, "in flight")
    for c in reversed(ctxs):
        c.close()


@pytest.mark.parametrize("world", [1, 3])
def test_block_order_permutation_changes_nothing(cvr, oracle_mod, world):
    scene = cvr.Scene.synthetic("manix")
    c = _owner(cvr, scene)
    iv, r2v = _setup(cvr, c)
    c.set_path_range(0, W * H * ITERS)
    c.set_block_shard(world - 1, world)
    nat, sn = _render(c)
    nb, nq, qbeg = c.launch_blocks()
    assert nb == len(range(world - 1, (W // 8) * (H // 8), world)) and qbeg[-1] == nb
    perm = np.random.default_rng(7).permutation(nb).astype(np.uint32)
    c.set_block_order(perm)
    per, sp = _render(c)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "fetches"):
        assert getattr(sn, k) == getattr(sp, k), k
    assert_pixels_close(per, nat, ITERS, "block order")
    with pytest.raises(cvr.CvrError):
        c.set_block_order(np.zeros(nb, np.uint32))  # not a permutation
    c.set_block_order(None)
    again, _ = _render(c)
    assert_pixels_close(again, nat, ITERS, "natural again")
    c.close()


def test_small_shard_auto_chunk_vs_oracle(cvr, oracle_mod):
    """A C2-sized block shard 7 of 8 (the per-rank launch of an 8-GPU
    strong-scaling render, where the wave pool's dequeue chunk drops to 64): pixels and
    counters vs the oracle's render of the same path ids."""
    from cudavolumerenderer_amd.distributed import block_shard_path_ids
    scene = cvr.Scene.synthetic("manix")
    Wc = Hc = 1024
    iters = 4  # 131 K paths per shard: about 26 per wave, chunk 64
    c = cvr.Context(0, "regenerationSK")
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(Wc, Hc)
    c.set_camera(iv, r2v, (Wc, Hc))
    c.init()
    c.set_resolution(Wc, Hc)
    c.set_iterations(iters)
    c.set_path_range(0, Wc * Hc * iters)
    c.set_block_shard(7, 8)
    c.clear_output()
    c.launch_render()
    st = c.stats()
    img = c.copy_output(Wc, Hc)
    ids = block_shard_path_ids(Wc, Hc, iters, 7, 8)
    orc = oracle_for_scene(oracle_mod, scene)
    L = orc.launch(iv, r2v, (Wc, Hc), (Wc, Hc), (0, 0), 2, 0)
    # the shard's path ids are runs of 8 consecutive ids (one block row of one sample)
    ref = np.zeros((Hc, Wc, 4), np.float32)
    steps = esc = 0
    for start in ids[::8]:
        rec = orc.trace_paths(L, int(start), 8)
        steps += int(rec["n_steps"].sum())
        e = rec[(rec["flags"] & 1) != 0]
        np.add.at(ref.reshape(-1, 4)[:, :3], e["image_id"], e["T"])
        ref.reshape(-1, 4)[e["image_id"], 3] = 1.0
        esc += len(e)
    assert st.paths == len(ids) and st.steps == steps and st.escaped == esc
    assert_pixels_close(img, ref, iters, "shard 7/8")
    c.close()


@pytest.mark.parametrize("name", ["manix", "hetvol"])
def test_morton_sorted_track_order_vs_oracle(cvr, oracle_mod, name):
    """streamingSK with the reference's Morton ray order (CVR_OPT_MORTON 1,
    StreamingVolPTsk_kernel.cuh:188-216) on the pool scheduler: counters equal
    and pixels within the summation bound against the oracle's streamingSK
    render (scatter -eps, kernel id 4) and the unsorted run."""
    scene = cvr.Scene.synthetic(name)
    imgs = []
    for morton in (0, 1):
        c = cvr.Context(0, "streamingSK")
        c.set_option(cvr.OPT_SCHEDULER, 2)  # the workgroup pool (streamingSK's default is the wave pool)
        c.set_option(cvr.OPT_MORTON, morton)
        c.set_medium(scene.medium)
        iv, r2v = _setup(cvr, c)
        imgs.append(_render(c))
        c.close()
    (i0, s0), (i1, s1) = imgs
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "fetches"):
        assert getattr(s0, k) == getattr(s1, k), k
    orc = oracle_for_scene(oracle_mod, scene)
    ref, rst = orc.render(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 4, 0), 0, W * H * ITERS, nthreads=8)
    assert_counters_equal(s1, rst, "morton vs oracle")
    assert_pixels_close(i1, ref, ITERS, "morton vs oracle")
    assert_pixels_close(i1, i0, ITERS, "morton vs unsorted")


def test_image_to_host_matches_division(cvr):
    """cvr_image_to_host: the kernel's x / scale into pinned memory equals
    IEEE fp32 division, including a ragged tail and an unaligned interior
    offset.  (HIP through ctypes: in this process libcvr loaded the HIP
    runtime before torch could.)"""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")
    P = C.c_void_p
    rng = np.random.default_rng(3)
    for n in (1, 7, 4096, (1 << 20) | 3):
        a = (rng.standard_normal(n) * 1e3).astype(np.float32)
        d_src, h_buf = P(), P()
        assert hip.hipMalloc(C.byref(d_src), C.c_size_t(n * 4)) == 0
        assert hip.hipHostMalloc(C.byref(h_buf), C.c_size_t((n + 8) * 4), 0) == 0
        try:
            assert hip.hipMemcpy(d_src, a.ctypes.data_as(P), C.c_size_t(n * 4), 1) == 0  # H2D
            host = np.ctypeslib.as_array(C.cast(h_buf, C.POINTER(C.c_float)), shape=(n + 8,))
            host[:] = 0
            cvr._lib.image_to_host(d_src.value, h_buf.value + 20, n, 20.0, None)  # 5 floats in: unaligned
            assert hip.hipDeviceSynchronize() == 0
            assert np.array_equal(host[5:5 + n], a / np.float32(20.0))
            assert (host[:5] == 0).all() and (host[5 + n:] == 0).all()
        finally:
            hip.hipFree(d_src)
            hip.hipHostFree(h_buf)


@pytest.mark.parametrize("w,h,world", [(64, 48, 1), (64, 48, 3), (1024, 1024, 8), (24, 8, 5)])
def test_blocks_to_host_writes_own_blocks(cvr, w, h, world):
    """cvr_blocks_to_host: every rank's kernel stores exactly its block
    shard's pixels (distributed.block_pixel_index), x / scale bit for bit,
    and leaves the other pixels alone; the world's ranks together fill the
    image (the multi-GPU output step without a reduction)."""
    import ctypes as C
    from cudavolumerenderer_amd.distributed import block_pixel_index
    hip = C.CDLL("libamdhip64.so.7")
    P = C.c_void_p
    n = w * h * 4
    a = (np.random.default_rng(w + world).standard_normal(n) * 1e3).astype(np.float32)
    d_src, h_buf = P(), P()
    assert hip.hipMalloc(C.byref(d_src), C.c_size_t(n * 4)) == 0
    assert hip.hipHostMalloc(C.byref(h_buf), C.c_size_t(n * 4), 0) == 0
    try:
        assert hip.hipMemcpy(d_src, a.ctypes.data_as(P), C.c_size_t(n * 4), 1) == 0  # H2D
        host = np.ctypeslib.as_array(C.cast(h_buf, C.POINTER(C.c_float)), shape=(n,))
        host[:] = np.nan
        want = np.full(n, np.nan, np.float32).reshape(-1, 4)
        for r in range(world):
            cvr._lib.blocks_to_host(d_src.value, h_buf.value, w, h, r, world, 20.0, None)
            assert hip.hipDeviceSynchronize() == 0
            idx = block_pixel_index(w, h, r, world)
            want[idx] = a.reshape(-1, 4)[idx] / np.float32(20.0)
            got = host.reshape(-1, 4)
            assert np.array_equal(np.isnan(got), np.isnan(want)), f"rank {r}: wrong pixels written"
            assert np.array_equal(got[idx], want[idx]), f"rank {r}"
        assert not np.isnan(host).any()
        with pytest.raises(cvr.CvrError):
            cvr._lib.blocks_to_host(d_src.value, h_buf.value, w + 4, h, 0, world, 1.0, None)
    finally:
        hip.hipFree(d_src)
        hip.hipHostFree(h_buf)


def test_shared_sparse_medium_in_flight(cvr):
    """A small sparse cloud (leaves, cell-leaf pool, brick words) shared by a
    second context on its own stream: both launched back to back without a
    sync render the same counters and pixels."""
    from test_sparse import CLOUD_SMALL
    scene = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    a = _owner(cvr, scene)
    _setup(cvr, a)
    b = cvr.Context(0, "regenerationSK")
    b.share_medium(a)
    _setup(cvr, b)
    a.use_own_stream()
    b.use_own_stream()
    for c in (a, b):
        c.clear_output()
        c.launch_render()
    ia, sa = c_out(a)
    ib, sb = c_out(b)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "fetches"):
        assert getattr(sa, k) == getattr(sb, k), k
    assert sa.fetches < sa.density and sa.albedo > 0
    assert_pixels_close(ib, ia, ITERS, "shared sparse medium")
    b.close()
    a.close()


def c_out(c):
    c.synchronize()
    return c.copy_output(W, H), c.stats()


def _launch_copy(c, w, h):
    """The launcher-level render (clear, cvr_launch_render, cvr_copy_output / ITERS),
    with the seed render_image's tile 0 has: a path independent of cvr_render_frame
    (render_image of one tile into host memory goes through cvr_render_frame)."""
    c.set_resolution(w, h)
    c.set_iterations(ITERS)
    c.set_offset(0, 0)
    c.set_seed(0)
    c.clear_output()
    c.launch_render()
    c.synchronize()
    img = c.copy_output(w, h, float(ITERS))
    st = c.stats()
    c.set_seed(0)
    return img, st


@pytest.mark.parametrize("kernel,parts,res", [("regenerationSK", 3, (256, 256)), ("regenerationSK", 2, (256, 200)),
                                              ("sortingSK", 3, (256, 256)), ("regenerationSK", 1, (256, 256)),
                                              ("regenerationSK", 3, (250, 256)), ("naiveSK", 3, (256, 256)),
                                              ("regenerationSK", 3, (64, 16))])
def test_render_frame_equals_render_image(cvr, kernel, parts, res):
    """cvr_render_frame (one synchronous render, the launch split into bands
    of block rows on helper contexts, each band's normalise + copy overlapping
    the later bands; one part: the in-launch output) leaves the same image in
    host memory as a plain launch + copy, with the same counters; kernels and
    sizes that cannot take bands (naiveSK, a side that is not a multiple of 8)
    render as one part.  Repeated calls reuse the helpers; a second medium
    loaded into the owner is what the helpers render next.  render_frame(None)
    sizes its array from the library's resolution, which render_image sets to
    its tile size."""
    w, h = res
    scene = cvr.Scene.synthetic("manix")
    c = cvr.Context(0, kernel)
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(w, h)
    c.set_camera(iv, r2v, (w, h))
    c.init()
    c.set_resolution(16, 8)
    c.set_iterations(ITERS)
    small, _ = c.render_image(w, h, (1, 1), ITERS)  # leaves the context at the w x h tile
    assert c.resolution == (w, h) and small.shape == (h, w, 4)
    ref, rst = _launch_copy(c, w, h)
    for rep in range(2):
        c.set_seed(0)  # render_image's tile 0 seed; both calls advance it as reset() does
        img, st = c.render_frame(None, parts)
        assert c.get_seed() == {"regenerationSK": w * h * ITERS, "sortingSK": 1}.get(kernel, 0)
        for k in ("paths", "segments", "steps", "density", "albedo", "escaped", "fetches"):
            assert getattr(st, k) == getattr(rst, k), (k, rep)
        assert_pixels_close(img[..., :3], ref[..., :3], ITERS, f"render_frame {kernel} {parts} parts")
        assert st.kernel_ms > 0
    # another medium in the owner: the helpers follow it
    other = cvr.Scene.synthetic("hetvol")
    c.set_medium(other.medium)
    ref2, rst2 = _launch_copy(c, w, h)
    img2, st2 = c.render_frame(None, parts)
    assert st2.steps == rst2.steps and st2.escaped == rst2.escaped
    assert_pixels_close(img2[..., :3], ref2[..., :3], ITERS, "render_frame after a new medium")
    c.close()


def test_framebuffer_growth_keeps_work_order_tables(cvr):
    """growing the owned framebuffer (cvr_set_resolution to a
    larger tile after renders with the Morton work order and a block order)
    must neither free nor reuse the work-order tables: the next render at the
    new size equals a fresh context's, and destroying the context is clean."""
    scene = cvr.Scene.synthetic("manix")
    c = cvr.Context(0, "regenerationSK")
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(256, 256)
    c.set_camera(iv, r2v, (256, 256))
    c.init()
    c.set_resolution(64, 64)
    c.set_iterations(2)
    c.clear_output()
    c.launch_render()
    c.synchronize()
    nb, _, _ = c.launch_blocks()
    c.set_block_order(np.arange(nb, dtype=np.uint32)[::-1].copy())
    c.clear_output()
    c.launch_render()
    c.synchronize()
    c.set_resolution(256, 256)  # the owned framebuffer grows
    c.set_iterations(ITERS)
    big, sb = _render(c)
    f = cvr.Context(0, "regenerationSK")
    f.share_medium(c)
    f.set_camera(iv, r2v, (256, 256))
    f.init()
    f.set_resolution(256, 256)
    f.set_iterations(ITERS)
    ref, sr = _render(f)
    for k in ("paths", "segments", "steps", "escaped", "fetches"):
        assert getattr(sb, k) == getattr(sr, k), k
    assert_pixels_close(big, ref, ITERS, "after framebuffer growth")
    f.close()
    c.close()
