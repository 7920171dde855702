"""Lane model of post_frame_kernel's top-16 percentile select (csrc/post.hip: lane_xor, cas_lane,
bitonic16_merge, bitonic16_sort, wave_top16, merge_top16): the same compare-exchange network and folds
over 64-lane numpy vectors, so the index algebra (the two keys of lane l, the runs' directions, the
folds by lane xor 16 / 32, the runs read reversed, the rank-to-lane map T - 16 + l % 16) is checked
against np.sort on the CPU."""
import numpy as np

L = np.arange(64)
ALL = np.ones(64, bool)


def cas(x, m, asc):
    """compare-exchange with lane l ^ m; the lower lane keeps the smaller key where asc"""
    y = x[L ^ m]
    return np.where(((L & m) == 0) == asc, np.minimum(x, y), np.maximum(x, y))


def bitonic16_merge(x, up):
    for m in (8, 4, 2, 1):
        x = cas(x, m, up)
    return x


def bitonic16_sort(x, up):
    x = cas(x, 1, ((L & 2) == 0) == up)
    a = ((L & 4) == 0) == up
    x = cas(cas(x, 2, a), 1, a)
    a = ((L & 8) == 0) == up
    x = cas(cas(cas(x, 4, a), 2, a), 1, a)
    return bitonic16_merge(x, up)


def wave_top16(keys, w):
    t = len(keys)
    i = 128 * w + L
    x0 = np.where(i < t, keys[np.minimum(i, t - 1)], 0)
    x1 = np.where(i + 64 < t, keys[np.minimum(i + 64, t - 1)], 0)
    y = np.maximum(bitonic16_sort(x0, ALL), bitonic16_sort(x1, ~ALL))
    y = bitonic16_merge(y, (L & 16) == 0)
    y = bitonic16_merge(np.maximum(y, y[L ^ 16]), (L & 32) == 0)
    y = bitonic16_merge(np.maximum(y, y[L ^ 32]), ALL)
    return y[:16]


def merge_top16(top):
    y = top[np.where(L & 16, (L | 15) - (L & 15), L)]
    y = bitonic16_merge(np.maximum(y, y[L ^ 16]), (L & 32) == 0)
    return bitonic16_merge(np.maximum(y, y[L ^ 32]), ALL)


def select(keys, r):
    """key of sorted rank r (len(keys) <= 512, r in the top 16)"""
    t = len(keys)
    assert t <= 512 and t - 1 - r <= 15
    top = np.concatenate([wave_top16(keys, w) for w in range(4)])
    return merge_top16(top)[16 - t + r]
