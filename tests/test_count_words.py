"""The brick-word counting instance (CVR_OPT_COUNT_WORDS, round 6): one more launch of
the benchmark's workload counts the brick words the sparse wave pool's Woodcock points
load (the empty-region mask skips the rest), so that bench.py's algorithmic bytes on a
sparse medium are exact instead of one word per density evaluation.  The counting
instance renders exactly what the benchmarked one does (same counters, same pixels up to
the summation order); its word count lies below the evaluations, and rises with the mask
off (every in-grid point loads its word)."""
import pytest

from parity_util import COUNTERS, assert_pixels_close
from test_gpu_records import _ctx

CLOUD_SMALL = (512, 256, 512)


def test_stats_struct_has_words(cvr):
    assert "words" in dict(cvr.Stats._fields_)
    assert cvr.load().cvr_abi_version() >= 4


def _render(cvr, scene, W, H, iters, count, mask=1):
    c, _, _ = _ctx(cvr, scene, W, H)
    c.set_option(cvr.OPT_EMPTY_MASK, mask)
    c.set_option(cvr.OPT_COUNT_WORDS, count)
    img, st = c.render_image(W, H, (1, 1), iters)
    c.close()
    return img, st


@pytest.mark.gpu
def test_counting_instance_renders_the_same(cvr):
    scene = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    W, H, iters = 128, 96, 3
    i0, s0 = _render(cvr, scene, W, H, iters, 0)
    i1, s1 = _render(cvr, scene, W, H, iters, 1)
    for k in COUNTERS + ("fetches",):
        assert getattr(s1, k) == getattr(s0, k), k
    assert_pixels_close(i1, i0, iters, "counting instance vs benchmarked instance")
    assert s0.words == 0, "only the counting instance counts"
    assert 0 < s1.words < s1.density
    _, s2 = _render(cvr, scene, W, H, iters, 1, mask=0)
    assert s2.density == s1.density and s2.words > s1.words, (s1.words, s2.words)


@pytest.mark.gpu
def test_dense_media_count_nothing(cvr):
    scene = cvr.Scene.synthetic("bucky")
    c, _, _ = _ctx(cvr, scene, 64, 64)
    c.set_option(cvr.OPT_COUNT_WORDS, 1)
    _, st = c.render_image(64, 64, (1, 1), 2)
    c.close()
    assert st.words == 0 and st.density > 0


@pytest.mark.gpu
def test_bench_line_counts_sparse_words(tmp_path):
    """bench.py on a sparse scene reports the words its counting launch found
    (counts_per_launch.brick_words_loaded) and builds its algorithmic bytes from
    them, so the bytes are exact rather than one word per density evaluation."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--scene", "cloud", "--resolution", "256", "256",
                        "--iterations", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--no-shard-emulation"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    roof = line["roofline"]
    counts = roof["counts_per_launch"]
    words = counts["brick_words_loaded"]
    assert 0 < words < counts["density_evals"]
    # 32 B per fetched cell + 4 B per word + 12 B per escape (the cloud's albedo is a constant)
    assert roof["algorithmic_bytes_per_launch"] == 32 * counts["cell_fetches"] + 4 * words + 12 * counts["escaped"]
