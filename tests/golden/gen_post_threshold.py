"""Makes tests/golden/post_threshold.npz: combined-spectrum frames whose bass-energy ratio sits within a
few float32 ulps of update_content_type's 0.6 threshold (omega4_main.py:805-840), chosen so that float64
range sums classify them differently from numpy's float32 pairwise np.mean -- the content type the
reference computes is the oracle's (np.mean, as the reference calls it). Run from the repo root:
python tests/golden/gen_post_threshold.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import omega_ref as R  # noqa: E402


def content_f64(s):
    """The classification with float64 range sums (what a naive device reduction computes)."""
    n = len(s)
    w = 48000 / (2 * n)
    be, vs, ve, hs = int(250 / w), int(200 / w), int(4000 / w), int(6000 / w)
    m = lambda a: np.float32(np.sum(a.astype(np.float64)) / len(a))  # noqa: E731
    eb, ev, eh, et = m(s[:be]), m(s[vs:ve]), m(s[hs:]), m(s)
    br, vr = eb / et, ev / et
    if br > np.float32(0.6):
        return 2
    if (vr > np.float32(0.4) and br < np.float32(0.4)) or (vr > np.float32(0.3) and eh < ev * np.float32(0.5)):
        return 1
    return 0


def main():
    rng = np.random.default_rng(0)
    found = []
    while len(found) < 3:
        s = (rng.random(512) * rng.random()).astype(np.float32)
        v = 0.6 * float(s[5:].astype(np.float64).sum()) / 509  # bass mean at 0.6 of the total mean
        s[:5] = (v * (1 + rng.standard_normal(5) * 1e-3)).astype(np.float32)
        for k in range(-40, 40):
            t = s.copy()
            t[0] = t[0] + np.float32(k) * np.spacing(t[0])
            if R.app_content_type(t) != content_f64(t):
                found.append(t)
                break
    x = np.stack(found)
    content = np.array([R.app_content_type(t) for t in x], np.int32)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "post_threshold.npz"),
                        combined=x, content=content, content_f64=np.array([content_f64(t) for t in x], np.int32))
    print(content)


if __name__ == "__main__":
    main()
