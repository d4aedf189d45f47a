#!/usr/bin/env python3
"""Generates tests/golden/*.npz: frozen outputs of the CPU oracle on small
seeded inputs (per-path records, RNG streams, scene checksums).

They pin the oracle against drift (tests/test_golden.py) and give the GPU
tests a fixed expectation that does not need the oracle at run time.  The
reference's own tests hold no vectors for this path and
the reference cannot be built here, so these are oracle outputs, not
reference outputs; DESIGN.md §Parity says what that pins and what it does
not.

    python tools/make_golden.py          # rewrites tests/golden/
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import cudavolumerenderer_amd as cvr  # noqa: E402
import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# (fixture name, synthetic scene, dims, image W, H, iterations, seed)
CASES = [
    ("bucky", "bucky", None, 16, 16, 2, 0),
    ("manix_small", "manix", (64, 58, 64), 16, 16, 2, 3),
    ("hetvol", "hetvol", None, 16, 16, 2, 0),
]
RNG_SEEDS = [0, 1, 12345, 2 ** 31 - 1, -1]


def scene_digest(s):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(s.density).tobytes())
    h.update(np.ascontiguousarray(s.albedo).tobytes())
    return h.hexdigest()


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, scene, dims, W, H, iters, seed in CASES:
        s = cvr.Scene.synthetic(scene, 0, dims)
        orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
        iv, r2v = cvr.default_camera(W, H)
        arrays = {"meta": np.array([W, H, iters, seed], np.int64),
                  "scene_sha256": np.frombuffer(bytes.fromhex(scene_digest(s)), np.uint8)}
        for kid in (0, 1, 2):
            L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, seed)
            rec = orc.trace_paths(L, 0, W * H * iters)
            arrays[f"paths_k{kid}"] = rec
            img, _ = orc.render(L, 0, W * H * iters)
            arrays[f"image_k{kid}"] = img
        np.savez_compressed(os.path.join(OUT, f"oracle_{name}.npz"), **arrays)
    u = np.stack([oracle.rng_stream(sd, 64)[0] for sd in RNG_SEEDS])
    f = np.stack([oracle.rng_stream(sd, 64)[1] for sd in RNG_SEEDS])
    np.savez_compressed(os.path.join(OUT, "rng_xorwow.npz"), seeds=np.array(RNG_SEEDS, np.int64), u32=u, f32=f)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
