"""cvr_render_frame's in-launch output (CVR_OPT_FRAME_FLUSH): the wave-pool
launch's flusher waves store each 8x8 block, normalised, into the pinned host
image as soon as all of the block's paths have ended (getImage's Scale + D->H
copy, ImageBufferTransfer.cu:61-78, without a copy after the launch).

Checked against the copy path of the same call (rgb within the summation-order
tolerance, w bit for bit, equal counters), against the oracle's image, and for
the bookkeeping: every block stored once, no fallback; a pageable host image
takes the copy path.
"""
import ctypes as C

import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene, oracle_image

pytestmark = pytest.mark.gpu


class Pinned:
    """A pinned host float4 image (hipHostMalloc) and its numpy view."""

    def __init__(self, w, h):
        self.hip = C.CDLL("libamdhip64.so.7")
        self.ptr = C.c_void_p()
        assert self.hip.hipHostMalloc(C.byref(self.ptr), C.c_size_t(w * h * 16), 0) == 0
        self.img = np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_float)), shape=(h, w, 4))

    def close(self):
        self.hip.hipHostFree(self.ptr)


def _scene(cvr, name):
    if name == "cloud":
        from test_sparse import CLOUD_SMALL
        return cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    return cvr.Scene.synthetic(name)


def _context(cvr, scene, w, h, iters):
    c = cvr.Context(0, "regenerationSK")
    if scene.is_sparse:
        c.set_medium_sparse(scene.sparse_medium)
    else:
        c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(w, h)
    c.set_camera(iv, r2v, (w, h))
    c.init()
    c.set_resolution(w, h)
    c.set_iterations(iters)
    c.set_option(cvr.OPT_FRAME_FLUSH, 1)
    return c, iv, r2v


@pytest.mark.parametrize("name,res,iters", [("manix", (256, 256), 4), ("hetvol", (136, 72), 3),
                                            ("bucky", (64, 64), 2), ("cloud", (128, 96), 2),
                                            ("manix", (1024, 1024), 2)])
def test_flush_equals_copy_and_oracle(cvr, oracle_mod, name, res, iters):
    w, h = res
    scene = _scene(cvr, name)
    c, iv, r2v = _context(cvr, scene, w, h, iters)
    buf = Pinned(w, h)
    try:
        buf.img[:] = np.nan
        c.set_seed(0)
        _, st = c.render_frame(buf.ptr.value, 1, host_floats=buf.img.size)
        blocks, fallbacks = c.frame_flush_info()
        assert (blocks, fallbacks) == ((w // 8) * (h // 8), 0)
        assert c.get_seed() == w * h * iters  # reset() as the copy path advances it
        flushed = buf.img.copy()
        assert not np.isnan(flushed[..., 3]).any(), "a pixel was not stored"

        c.set_option(cvr.OPT_FRAME_FLUSH, 0)
        buf.img[:] = np.nan
        c.set_seed(0)
        _, st0 = c.render_frame(buf.ptr.value, 1, host_floats=buf.img.size)
        assert c.frame_flush_info() == (0, 0)
        copied = buf.img.copy()
        for k in COUNTERS:
            assert getattr(st, k) == getattr(st0, k), k
        assert np.array_equal(flushed[..., 3], copied[..., 3]), "w differs from the copy path"
        assert_pixels_close(flushed[..., :3], copied[..., :3], iters, f"{name}: flush vs copy")

        if w * h * iters <= 256 * 256 * 4:
            orc = oracle_for_scene(oracle_mod, scene)
            ref, rst = oracle_image(orc, iv, r2v, w, h, (1, 1), iters, 2)
            for k in COUNTERS:
                assert getattr(st, k) == rst[k], k
            assert np.array_equal(flushed[..., 3], ref[..., 3]), "w differs from the oracle"
            assert_pixels_close(flushed[..., :3], ref[..., :3], iters, f"{name}: flush vs oracle")

        # a pageable host image: the copy after the launch
        c.set_option(cvr.OPT_FRAME_FLUSH, 1)
        c.set_seed(0)
        img, _ = c.render_frame(None, 1)
        assert c.frame_flush_info() == (0, 0)
        assert np.array_equal(img[..., 3], copied[..., 3])
        assert_pixels_close(img[..., :3], copied[..., :3], iters, f"{name}: pageable vs copy")
    finally:
        buf.close()
        c.close()


def test_flush_repeated_frames_and_bands(cvr):
    """Back-to-back flushed frames reuse the counts and the status words; a
    multi-band call (parts 2) takes the copy path; a tile whose side is not a
    multiple of 8 (no pixel-block order) takes the copy path."""
    scene = _scene(cvr, "manix")
    c, _, _ = _context(cvr, scene, 128, 128, 3)
    buf = Pinned(128, 128)
    try:
        imgs = []
        for _ in range(3):
            c.set_seed(7)
            c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
            assert c.frame_flush_info() == (256, 0)
            imgs.append(buf.img.copy())
        for im in imgs[1:]:
            assert np.array_equal(im[..., 3], imgs[0][..., 3])
            assert_pixels_close(im[..., :3], imgs[0][..., :3], 3, "repeat")
        c.set_seed(7)
        c.render_frame(buf.ptr.value, 2, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info()[0] == 0
        assert_pixels_close(buf.img[..., :3], imgs[0][..., :3], 3, "two bands")
    finally:
        buf.close()
        c.close()
    c, _, _ = _context(cvr, scene, 100, 64, 2)
    buf = Pinned(100, 64)
    try:
        c.set_seed(0)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info()[0] == 0
    finally:
        buf.close()
        c.close()


def test_flush_with_block_order_and_other_budgets(cvr):
    """A caller's block order (cvr_set_block_order) is followed by the flushers
    too; a register budget without an in-launch output instance (4 waves per
    SIMD) takes the copy path.  Same image as the copy path throughout."""
    scene = _scene(cvr, "manix")
    c, _, _ = _context(cvr, scene, 128, 128, 3)
    buf = Pinned(128, 128)
    try:
        c.set_option(cvr.OPT_FRAME_FLUSH, 0)
        c.set_seed(3)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        ref = buf.img.copy()
        c.set_option(cvr.OPT_FRAME_FLUSH, 1)
        nb, _, _ = c.launch_blocks()
        c.set_block_order(np.random.default_rng(5).permutation(nb).astype(np.uint32))
        buf.img[:] = np.nan
        c.set_seed(3)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info() == (256, 0)
        assert np.array_equal(buf.img[..., 3], ref[..., 3])
        assert_pixels_close(buf.img[..., :3], ref[..., :3], 3, "block order")
        c.set_option(cvr.OPT_WAVES, 4)
        buf.img[:] = np.nan
        c.set_seed(3)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info()[0] == 0
        assert np.array_equal(buf.img[..., 3], ref[..., 3])
        assert_pixels_close(buf.img[..., :3], ref[..., :3], 3, "4 waves")
    finally:
        buf.close()
        c.close()


def test_flush_fallback_copy(cvr):
    """CVR_OPT_FRAME_FLUSH 2 (test mode): the flushers give up at once and the
    call copies the image after the launch instead; same image, the fallback
    counted, and the next flushed frame works again."""
    scene = _scene(cvr, "hetvol")
    c, _, _ = _context(cvr, scene, 96, 64, 3)
    buf = Pinned(96, 64)
    try:
        c.set_seed(1)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info() == (96, 0)
        ref = buf.img.copy()
        c.set_option(cvr.OPT_FRAME_FLUSH, 2)
        buf.img[:] = np.nan
        c.set_seed(1)
        _, st = c.render_frame(buf.ptr.value, 1, host_floats=buf.img.size)
        assert c.frame_flush_info() == (0, 1)
        assert st.paths == 96 * 64 * 3
        assert np.array_equal(buf.img[..., 3], ref[..., 3])
        assert_pixels_close(buf.img[..., :3], ref[..., :3], 3, "fallback")
        c.set_option(cvr.OPT_FRAME_FLUSH, 1)
        c.set_seed(1)
        c.render_frame(buf.ptr.value, 1, stats=False, host_floats=buf.img.size)
        assert c.frame_flush_info() == (96, 1)
        assert_pixels_close(buf.img[..., :3], ref[..., :3], 3, "flush after fallback")
    finally:
        buf.close()
        c.close()


def test_short_host_buffer_rejected(cvr):
    """ABI 3: cvr_render_frame takes the host buffer's size and rejects one
    shorter than the tile (CVR_ERR_INVALID) before anything runs: the seed
    does not advance and the buffer is not written."""
    scene = cvr.Scene.synthetic("bucky")
    c, _, _ = _context(cvr, scene, 64, 64, 1)
    buf = Pinned(64, 64)
    try:
        buf.img[:] = -7.0
        c.set_seed(5)
        with pytest.raises(cvr.CvrError) as e:
            c.render_frame(buf.ptr.value, 1, host_floats=64 * 64 * 4 - 1)
        assert e.value.code == -1 and "floats" in str(e.value)
        assert c.get_seed() == 5
        assert (buf.img == -7.0).all()
        c.render_frame(buf.ptr.value, 1, host_floats=64 * 64 * 4)  # exactly the tile
        assert c.get_seed() == 5 + 64 * 64
    finally:
        buf.close()
        c.close()
