#!/usr/bin/env python3
"""MEASURED AND REJECTED (round 4): the variant this models was built, parity-green
and slower on MI355X (profiles/r04_ab_paired_tp_cfg3_post.txt); the product kernels keep the
natural-order exchange. Kept as the record of the index algebra.

Model of the cfg3 transform in the paired role map (K = 4096, L = 16; csrc/regfft.hpp prow,
csrc/rfkern.hip spectra_rf_body): wave w's pass-2/3 threads hold rows {2w, 16 - 2w, 2w + 1, 15 - 2w}
(wave 0: {0, 1, 8, 15}), lane bits 4-5 choosing the row; output register m of lane l is frequency
n = k1 + 16 k2 + 256 m (k2 = l & 15). The mirror K - n is register 15 - m of lane l ^ 47 (row 8:
l ^ 15; row 0: lane 16 - l, and lane 0 of wave 0 its own register 16 - m), so the rfft magnitudes
need no natural-order exchange. Checks: the transform, the mirrors, |rfft| and exchange conflicts."""
import numpy as np

K, NTH, L = 4096, 256, 16
P1 = P2R = 272
P2C = 17


def prow(t):
    # (rows 2w and 2w + 1 share a 32-lane half: their exchange slots differ by an odd multiple of 272,
    # i.e. 16 banks -- no conflicts; the mirror rows 16 - 2w, 15 - 2w are the other half)
    w, j = t >> 6, (t >> 4) & 3
    return (2 * w, 2 * w + 1, 8 if w == 0 else 16 - 2 * w, 15 - 2 * w)[j]


def out_index(t, m):
    return prow(t) + 16 * (t & 15) + 256 * m


def a1(t, k1):
    return P1 * k1 + t


def a2(u, k2, k1):
    return P2R * k1 + P2C * k2 + u


W = np.exp(-2j * np.pi / K)


def dif(x):
    lds = {}
    for t in range(NTH):
        A = np.fft.fft(x[t + NTH * np.arange(16)]) * W ** (t * np.arange(16))
        for k1 in range(16):
            lds[a1(t, k1)] = A[k1]
    lds2 = {}
    for t in range(NTH):
        u, k1 = t % L, prow(t)
        b = np.array([lds[a1(u + L * v, k1)] for v in range(16)])
        C = np.fft.fft(b) * W ** (16 * u * np.arange(16))
        for k2 in range(16):
            lds2[a2(u, k2, k1)] = C[k2]
    out = np.zeros((NTH, 16), complex)
    for t in range(NTH):
        k2, k1 = t & 15, prow(t)
        out[t] = np.fft.fft(np.array([lds2[a2(u, k2, k1)] for u in range(16)]))
    return out


def mirror_src(t, m):
    w, l = t >> 6, t & 63
    k1, k2 = prow(t), t & 15
    if k1 not in (0, 8):
        return 64 * w + (l ^ 47), 15 - m
    if k1 == 8:
        return 64 * w + (l ^ 15), 15 - m
    if k2 >= 1:
        return 64 * w + (16 - l), 15 - m
    return None if m == 0 else (t, 16 - m)


def check():
    rng = np.random.default_rng(0)
    z = rng.standard_normal(K) + 1j * rng.standard_normal(K)
    Z = dif(z)
    F = np.fft.fft(z)
    err = max(abs(Z[t, m] - F[out_index(t, m)]) for t in range(NTH) for m in range(16)) / np.max(np.abs(F))
    bad = 0
    for t in range(NTH):
        for m in range(16):
            s = mirror_src(t, m)
            n = out_index(t, m)
            if s is None:
                bad += n != 0
            else:
                bad += out_index(*s) != (K - n) % K or (s[0] >> 6) != (t >> 6)
    x = rng.standard_normal(2 * K)
    Zx = dif(x[0::2] + 1j * x[1::2])
    X = np.fft.rfft(x)
    merr = 0.0
    for t in range(NTH):
        for m in range(16):
            n = out_index(t, m)
            s = mirror_src(t, m)
            a = Zx[t, m]
            if s is None:
                mag = abs(a.real + a.imag)
                merr = max(merr, abs(abs(a.real - a.imag) - abs(X[K])))
            else:
                b = Zx[s]
                e = (a + np.conj(b)) / 2
                o = -1j * (a - np.conj(b)) / 2
                mag = abs(e + np.exp(-2j * np.pi * n / (2 * K)) * o)
            merr = max(merr, abs(mag - abs(X[n])))
    return err, bad, merr / np.max(np.abs(X))


def conflicts():
    def rd(addrs):
        extra = 0
        for g0 in (0, 32):
            banks = {}
            for a in addrs[g0:g0 + 32]:
                banks.setdefault(a % 32, set()).add(a)
            extra += max(len(s) for s in banks.values()) - 1
        return extra

    def wr(addrs):
        extra = 0
        for g0 in range(0, 64, 16):
            banks = {}
            for a in addrs[g0:g0 + 16]:
                banks.setdefault(a % 16, set()).add(a)
            extra += max(len(s) for s in banks.values()) - 1
        return extra
    worst = {}
    for w in range(NTH // 64):
        lanes = range(64 * w, 64 * w + 64)
        for r in range(16):
            for k, v in (("x1r", rd([a1(t % L + L * r, prow(t)) for t in lanes])),
                         ("x2w", wr([a2(t % L, r, prow(t)) for t in lanes])),
                         ("x2r", rd([a2(r, t & 15, prow(t)) for t in lanes]))):
                worst[k] = max(worst.get(k, 0), v)
    return worst


if __name__ == "__main__":
    print("fft err, mirror errors, |rfft| err:", check())
    print("conflicts", conflicts())
