#!/usr/bin/env python3
"""Post-processing band diagnostic on the GPU: raw bands (smoothing off) and smoothed bands against
the reference golden (app_post.npz default), per frame."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
from oracle import omega_ref as R  # noqa: E402


def main():
    from omega_gpu.app_post import SpectrumPostProcessor
    g = np.load(os.path.join(REPO, "tests", "golden", "app_post.npz"))
    comb, freqs, gb = g["default/combined"], g["default/freqs"], g["default/bands"]
    _, raw_dev, _ = SpectrumPostProcessor(freqs, smoothing_enabled=False).process(comb)
    _, raw_ref, _ = R.app_post_sequence(comb, freqs, smoothing=False)
    print("raw equal", np.array_equal(raw_dev, raw_ref), "mismatch per frame", (raw_dev != raw_ref).sum(axis=1).tolist())
    _, b, _ = SpectrumPostProcessor(freqs).process(comb)
    print("smoothed mismatch per frame", (b != gb).sum(axis=1).tolist())
    d = np.argwhere(b != gb)
    for fi, i in d[:5]:
        print(fi, i, repr(b[fi, i]), repr(gb[fi, i]), repr(raw_ref[fi, i]), repr(b[fi - 1, i]), repr(gb[fi - 1, i]))


if __name__ == "__main__":
    main()
