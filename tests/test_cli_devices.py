"""The CLI's multi-device render (cvr --devices, SURVEY §8(e) from the drop-in
surface): one context per device, each on its own host thread, storing its
pixel-disjoint share (tile k -> context k mod N with --number-of-tiles, else
8x8-block shards of the one tile) straight into one pinned host image through
cvr_render_share_to_host, with no reduction and no torch.

The leased box has one GPU, so the contexts share device 0 (`--devices
0,0,0`): each still has its own stream, work queues and wave-pool scratch, and
the shares are exactly the ones N devices would render.  The image (written as
a float .pfm) must equal cvr_render_image's single-context render within the
summation-order bound."""
import os
import subprocess

import numpy as np
import pytest

from parity_util import assert_pixels_close

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cudavolumerenderer_amd", "cvr")


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        assert scale < 0  # little-endian
        a = np.frombuffer(f.read(), dtype="<f4").reshape(h, w, 3)
    return a[::-1]  # rows bottom to top


def run_cli(tmp_path, name, *args):
    out = str(tmp_path / name)
    r = subprocess.run([CLI, "--interactive", "0", "--pfm", "-o", out, *args], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return read_pfm(out + ".pfm"), r.stdout


def reference_image(cvr, scene_name, W, H, tiles, iters, kernel="regenerationSK"):
    scene = cvr.Scene.synthetic(scene_name)
    c = cvr.Context(0, kernel)
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    c.init()
    img, _ = c.render_image(W, H, tiles, iters)
    c.close()
    return img[..., :3]


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_cli_block_shards_equal_one_context(cvr, tmp_path, devices):
    W, H, iters = 256, 192, 4
    img, out = run_cli(tmp_path, "blk", "--synthetic", "manix", "-r", str(W), str(H), "-i", str(iters),
                       "--devices", devices)
    n = len(devices.split(","))
    assert f"[Devices] {n} contexts" in out and "block shards" in out
    ref = reference_image(cvr, "manix", W, H, (1, 1), iters)
    assert ref.max() > 0
    assert_pixels_close(img, ref, iters, f"CLI --devices {devices} vs one context")


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK"])
def test_cli_tile_shards_equal_tile_loop(cvr, tmp_path, kernel):
    """--number-of-tiles 4 2 over three contexts: tiles 0, 3, 6 / 1, 4, 7 / 2, 5,
    each with its sequential-loop seed (regenerationSK +n_paths, streamingSK +1
    per tile), against the one-context tile loop."""
    W, H, iters = 256, 128, 3
    img, out = run_cli(tmp_path, "tiles", "--synthetic", "hetvol", "-r", str(W), str(H), "-i", str(iters),
                       "--number-of-tiles", "4", "2", "-k", kernel, "--devices", "0,0,0")
    assert "tile k -> context k mod N" in out
    ref = reference_image(cvr, "hetvol", W, H, (4, 2), iters, kernel)
    assert_pixels_close(img, ref, iters, f"CLI tiles x3 {kernel} vs tile loop")


@pytest.mark.gpu
def test_cli_ragged_tiles_leave_remainder_black(cvr, tmp_path):
    """Q1 on the multi-device path: 3 x 2 tiles of a 100 x 70 image render
    tiles of 33 x 35, pixels x >= 99 are never written (zero), the rest equal
    the one-context tile loop; a one-tile image whose sides are not multiples
    of 8 cannot be block-sharded and renders on the first device."""
    img, _ = run_cli(tmp_path, "ragged", "--synthetic", "bucky", "-r", "100", "70", "-i", "2",
                     "--number-of-tiles", "3", "2", "--devices", "0,0")
    ref = reference_image(cvr, "bucky", 100, 70, (3, 2), 2)
    assert (img[:, 99:] == 0).all()
    assert_pixels_close(img, ref, 2, "ragged tiles x2")
    img1, out = run_cli(tmp_path, "one", "--synthetic", "bucky", "-r", "100", "70", "-i", "2", "--devices", "0,0")
    assert "rendering on device 0" in out
    assert_pixels_close(img1, reference_image(cvr, "bucky", 100, 70, (1, 1), 2), 2, "fallback single device")


@pytest.mark.parametrize("devices", ["0", "1,", ",1", "a,b", "0,,1", "2x", "-1,0"])
def test_cli_rejects_bad_devices(tmp_path, devices):
    """Host-only: a zero count, an empty entry or a non-numeric one is a usage error
    (exit 2) before any scene or device is touched (not silently device 0)."""
    r = subprocess.run([CLI, "--synthetic", "bucky", "--devices", devices, "--interactive", "0", "-o",
                        str(tmp_path / "x")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "--devices" in r.stderr, (devices, r.returncode, r.stderr)


@pytest.mark.gpu
def test_cli_thread_binding_does_not_block_shard(cvr, tmp_path):
    """--rng-binding thread has no 8x8-block work order: the CLI renders on one
    device instead of writing part-sums of other pixels (round-5 advisor), and the
    library refuses such a block-shard share outright."""
    W, H, iters = 64, 64, 2
    img, out = run_cli(tmp_path, "thr", "--synthetic", "bucky", "-r", str(W), str(H), "-i", str(iters),
                       "--rng-binding", "thread", "--devices", "0,0")
    assert "rendering on device 0" in out and "block shards of the image" not in out
    assert np.isfinite(img).any() and img.max() > 0
    scene = cvr.Scene.synthetic("bucky")
    c = cvr.Context(0, "regenerationSK")
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    c.set_option(cvr.OPT_RNG_BINDING, 1)
    c.init()
    c.set_block_shard(0, 2)
    pim = cvr.PinnedImage(W, H)
    try:
        with pytest.raises(RuntimeError, match="UNSUPPORTED"):
            c.render_share_to_host(pim.ptr.value, pim.floats, W, H, (1, 1), iters)
    finally:
        pim.close()
        c.close()


@pytest.mark.gpu
def test_share_to_host_from_python_threads(cvr):
    """The same multi-device path through the Python binding: three contexts
    (sharing one device medium), one Python thread each (ctypes releases the
    GIL), block shards of one tile into one PinnedImage."""
    import threading
    W, H, iters = 128, 128, 3
    scene = cvr.Scene.synthetic("hetvol")
    iv, r2v = cvr.default_camera(W, H)
    ctxs = []
    for k in range(3):
        c = cvr.Context(0, "regenerationSK")
        if k == 0:
            c.set_medium(scene.medium)
        else:
            c.share_medium(ctxs[0])
        c.set_camera(iv, r2v, (W, H))
        c.init()
        c.set_block_shard(k, 3)
        ctxs.append(c)
    img = cvr.PinnedImage(W, H)
    try:
        img.array[:] = -1.0
        errs = []

        def work(k):
            try:
                ctxs[k].render_share_to_host(img.ptr.value, img.floats, W, H, (1, 1), iters)
            except Exception as e:  # noqa: BLE001 (reported below)
                errs.append(e)
        th = [threading.Thread(target=work, args=(k,)) for k in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        out = img.array.copy()
    finally:
        img.close()
    assert (out != -1.0).all(), "a pixel no share wrote"
    for c in reversed(ctxs):
        c.close()
    ref = reference_image(cvr, "hetvol", W, H, (1, 1), iters)
    assert_pixels_close(out[..., :3], ref, iters, "python threads x3 vs one context")
