"""Lane model of post_frame_kernel's top-16 percentile select (csrc/post.hip: lane_xor, cas_lane,
sort128, wave_top16, merge_top64): the same compare-exchange network over 64-lane numpy vectors, so the
index algebra (key 2l + h on lane l, the runs read reversed, the rank-to-lane map T - 64 + l) is checked
against np.sort on the CPU."""
import numpy as np

L = np.arange(64)


def cas(x, m, asc):
    """compare-exchange with lane l ^ m; the lower lane keeps the smaller key where asc"""
    y = x[L ^ m]
    return np.where(((L & m) == 0) == asc, np.minimum(x, y), np.maximum(x, y))


def sort128(x0, x1):
    k = 2
    while k <= 128:
        asc = ((2 * L) & k) == 0
        j = k // 2
        while j >= 1:
            if j == 1:
                lo, hi = np.minimum(x0, x1), np.maximum(x0, x1)
                x0, x1 = np.where(asc, lo, hi), np.where(asc, hi, lo)
            else:
                x0, x1 = cas(x0, j // 2, asc), cas(x1, j // 2, asc)
            j //= 2
        k *= 2
    return x0, x1


def wave_top16(keys, w):
    t = len(keys)
    i = 128 * w + 2 * L
    x0 = np.where(i < t, keys[np.minimum(i, t - 1)], 0)
    x1 = np.where(i + 1 < t, keys[np.minimum(i + 1, t - 1)], 0)
    x0, x1 = sort128(x0, x1)
    e = np.stack([x0, x1], 1).reshape(-1)  # key 2l + h
    return e, e[112:]


def merge_top64(top):
    x = top[np.where(L & 16, (L | 15) - (L & 15), L)]
    for m in (16, 8, 4, 2, 1):
        x = cas(x, m, L < 32)
    for m in (32, 16, 8, 4, 2, 1):
        x = cas(x, m, np.ones(64, bool))
    return x


def select(keys, r):
    """key of sorted rank r (len(keys) <= 512, r in the top 16)"""
    t = len(keys)
    assert t <= 512 and t - 1 - r <= 15
    top = np.concatenate([wave_top16(keys, w)[1] for w in range(4)])
    return merge_top64(top)[64 - t + r]
