"""Generate the committed golden vectors (tests/golden/*.npz + manifest.json).

Inputs come from the product's deterministic generator (mdx_synth_pair) and
from a few hand-built scenes; expected outputs come from the C oracle and are cross-checked
against the independent numpy restatement (tests/np_reference.py) before being written --
a fixture is only emitted when both restatements agree bit for bit.

The reference repository ships no tests or fixtures and OpenCV 2.4 is not
available here, so these vectors pin the oracle to the restated OpenCV semantics, not to
an OpenCV binary ("parity unpinned" w.r.t. real OpenCV).

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import motion_detection_amd as m  # noqa: E402  (generator only; libmdx.so loads without a GPU)
import np_reference as npr  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def scenes():
    a, b, H = m.synth_pair(20141105, 160, 120, 1)
    yield "synth_160x120_gray", a, b, dict(pixel_step=10, min_vector_size=1.0)
    a, b, H = m.synth_pair(20141106, 320, 240, 1)
    yield "synth_320x240_gray_ps7", a, b, dict(pixel_step=7, min_vector_size=1.0)
    a, b, H = m.synth_pair(20141107, 160, 120, 3)
    yield "synth_160x120_rgb", a, b, dict(pixel_step=10, min_vector_size=0.4)
    big, _, _ = m.synth_pair(99, 240, 180, 1)
    a = np.ascontiguousarray(big[10:130, 10:170]); b = np.ascontiguousarray(big[8:128, 6:166])
    yield "translate_4_2", a, b, dict(pixel_step=10, min_vector_size=1.0)
    flat = np.full((96, 128), 77, np.uint8)
    yield "flat", flat, flat.copy(), dict(pixel_step=8, min_vector_size=1.0)


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    manifest = {}
    for name, a, b, prm in scenes():
        ref = po.calculate_optical_flow(a, b, **prm)
        chk = npr.calculate_optical_flow(a, b, pixel_step=prm["pixel_step"], min_vector_size=prm["min_vector_size"])
        assert ref["num_vectors"] == chk["num_vectors"], name
        assert np.array_equal(ref["status"], chk["status"]), name
        assert np.array_equal(ref["next_pts"].view(np.uint32), chk["next_pts"].view(np.uint32)), name
        assert np.array_equal(ref["vectors"], chk["vectors"]), name
        assert np.array_equal(ref["H"], chk["H"]), name
        assert np.array_equal(ref["mask"], chk["mask"]), name
        out = dict(img1=a, img2=b, next_pts=ref["next_pts"], status=ref["status"], vectors=ref["vectors"],
                   mask=ref["mask"], H=ref["H"], Hinv=ref["Hinv"], num_vectors=np.int32(ref["num_vectors"]),
                   pixel_step=np.int32(prm["pixel_step"]), min_vector_size=np.float64(prm["min_vector_size"]))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        manifest[name] = dict(shape=list(a.shape), num_vectors=int(ref["num_vectors"]), inputs_sha256=sha(a, b),
                              outputs_sha256=sha(ref["next_pts"], ref["status"], ref["vectors"], ref["mask"], ref["H"]),
                              **prm)
        print(f"{name}: {ref['num_vectors']} vectors, fit_status {ref['fit_status']}")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
