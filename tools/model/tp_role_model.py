#!/usr/bin/env python3
"""MEASURED AND REJECTED (round 4): the variant this models was built, parity-green
and slower on MI355X (profiles/r04_ab_paired_tp_cfg3_post.txt); the product kernels keep the
natural-order exchange. Kept as the record of the index algebra.

Model of the true peak on the register FFT without the natural-order exchange (csrc/regfft.hpp
run2 with the paired role map, run_dit; csrc/rfkern.hip truepeak_rf_body): checks the index algebra
against numpy / the oracle and counts LDS bank conflicts of the new exchange patterns (K = 8192).

  forward (DIF, run2): pass-1 column t1 = tp_column(tid), passes 2/3 in the PAIRED role map: wave w
    holds rows k1 in {a_w, 16 - a_w} (a_0 = 0 with 8), lane l: u = l % 32 (pass 2), q = l & 1,
    k2 = (l >> 1) & 15 (pass 3), j = l >> 5 selects the row; output register m of lane l is
    frequency n = k1 + 16 k2 + 256 (m + 16 q)
  untangle: Z_{K-n} is register 15 - m of the mirror lane (lane ^ 63; wave 0: 95 - lane for the row
    k1 = 8, 33 - lane for row 0, lanes 0 / 1 of row 0 read register 16 - m of lane ^ 1)
  phases: y = X rho^p, the packed inverse input from the mirror lane's values (same map), then the
    transposed (DIT) pipeline of the forward: pass 3^T (lane-pair butterfly, odd lanes * w32^m,
    DFT16), exchange 2^T (wave-local), pass 2^T (twiddle, DFT16), exchange 1^T, pass 1^T (twiddle,
    DFT16) -> y at t1 + NTH r: max |.| only.
"""
import sys

import numpy as np

K, NTH, L = 8192, 512, 32
P1 = P2R = 544
P2C = 34


def tp_column(tid):
    w, l = tid >> 6, tid & 63
    if l < 32:
        return 32 * w + l
    a = 32 * w + (63 - l)
    return NTH // 2 if a == 0 else NTH - a


def row_of(w, j):
    if w == 0:
        return 0 if j == 0 else 8
    return w if j == 0 else 16 - w


def p2(tid):  # (u, k1)
    w, l = tid >> 6, tid & 63
    return l & 31, row_of(w, l >> 5)


def p3(tid):  # (q, k2, k1)
    w, l = tid >> 6, tid & 63
    return l & 1, (l >> 1) & 15, row_of(w, l >> 5)


def out_index(tid, m):
    q, k2, k1 = p3(tid)
    return k1 + 16 * k2 + 256 * (m + 16 * q)


def a1(t, k1):
    return P1 * k1 + t


def a2(u, k2, k1):
    return P2R * k1 + P2C * k2 + u


W = np.exp(-2j * np.pi / K)
w32 = np.exp(-2j * np.pi / 32) ** np.arange(16)


def dif(x):
    """run2: x natural -> out[tid, m] = X[out_index(tid, m)]"""
    lds = {}
    for tid in range(NTH):
        t1 = tp_column(tid)
        A = np.fft.fft(x[t1 + NTH * np.arange(16)]) * W ** (t1 * np.arange(16))
        for k1 in range(16):
            lds[a1(t1, k1)] = A[k1]
    C = {}
    for tid in range(NTH):
        u, k1 = p2(tid)
        b = np.array([lds[a1(u + L * v, k1)] for v in range(16)])
        C[tid] = np.fft.fft(b) * W ** (16 * u * np.arange(16))
    lds2 = {}
    for tid in range(NTH):
        u, k1 = p2(tid)
        for k2 in range(16):
            lds2[a2(u, k2, k1)] = C[tid][k2]
    out = np.zeros((NTH, 16), complex)
    for tid in range(NTH):
        q, k2, k1 = p3(tid)
        c = np.array([lds2[a2(q + 2 * up, k2, k1)] for up in range(16)])
        out[tid] = np.fft.fft(c)
    F = out.copy()
    for tid in range(NTH):
        if tid & 1:
            F[tid] *= w32
    for tid in range(NTH):
        own, par = F[tid], F[tid ^ 1]
        out[tid] = own + par if not (tid & 1) else par - own
    return out


def dit(v):
    """run_dit: v[tid, m] = D[out_index(tid, m)] -> y[tid, r] = (FFT D)[tp_column(tid) + NTH r]"""
    G = np.zeros((NTH, 16), complex)
    for tid in range(NTH):  # lane-pair butterfly (its own transpose), odd lanes * w32^m, DFT16
        own, par = v[tid], v[tid ^ 1]
        g = own + par if not (tid & 1) else par - own
        if tid & 1:
            g = g * w32
        G[tid] = np.fft.fft(g)  # register u' -> element u = q + 2 u'
    lds2 = {}
    for tid in range(NTH):
        q, k2, k1 = p3(tid)
        for up in range(16):
            lds2[a2(q + 2 * up, k2, k1)] = G[tid][up]
    lds = {}
    for tid in range(NTH):
        u, k1 = p2(tid)
        b = np.array([lds2[a2(u, k2, k1)] for k2 in range(16)]) * W ** (16 * u * np.arange(16))
        B = np.fft.fft(b)  # register v -> element t = u + L v
        for vv in range(16):
            lds[a1(u + L * vv, k1)] = B[vv]
    y = np.zeros((NTH, 16), complex)
    for tid in range(NTH):
        t1 = tp_column(tid)
        a = np.array([lds[a1(t1, k1)] for k1 in range(16)]) * W ** (t1 * np.arange(16))
        y[tid] = np.fft.fft(a)  # register r -> t1 + NTH r
    return y


def mirror_src(tid, m):
    """(lane, register) holding Z_{K - n} for n = out_index(tid, m); None for the self-mirrored n = 0."""
    w, l = tid >> 6, tid & 63
    q, k2, k1 = p3(tid)
    if k1 not in (0, 8):
        return 64 * w + (l ^ 63), 15 - m
    if k1 == 8:
        return 64 * w + (95 - l), 15 - m
    if k2 >= 1:
        return 64 * w + (33 - l), 15 - m
    if m == 0:
        return None if q == 0 else (tid, 0)  # n = 0 (DC / Nyquist) and n = K / 2 (its own mirror)
    return 64 * w + (l ^ 1), 16 - m


def check_mirrors():
    bad = 0
    for tid in range(NTH):
        for m in range(16):
            n = out_index(tid, m)
            src = mirror_src(tid, m)
            if src is None:
                bad += n != 0
                continue
            bad += out_index(src[0], src[1]) != (K - n) % K
            bad += (src[0] >> 6) != (tid >> 6)  # same wave (ds_bpermute)
    return bad


def truepeak(x):
    M = len(x)
    z = x[0::2] + 1j * x[1::2]
    Z = dif(z)  # Z[tid, m] = FFT(z)[n]
    X = np.zeros((NTH, 16), complex)
    XN = None
    for tid in range(NTH):
        for m in range(16):
            n = out_index(tid, m)
            src = mirror_src(tid, m)
            a = Z[tid, m]
            if src is None:
                X[tid, m] = a.real + a.imag
                XN = a.real - a.imag
                continue
            b = Z[src]
            e = (a + np.conj(b)) / 2
            o = -1j * (a - np.conj(b)) / 2
            X[tid, m] = e + np.exp(-2j * np.pi * n / M) * o
    nn = np.array([[out_index(tid, m) for m in range(16)] for tid in range(NTH)])
    rho = np.exp(2j * np.pi * nn / (4 * M))
    alpha = (1 + 1j * np.exp(2j * np.pi * nn / M)) / 2
    mx = np.max(np.abs(x))
    Y = X.copy()
    for p in range(1, 4):
        Y = Y * rho
        Yp = np.zeros_like(Y)
        for tid in range(NTH):
            for m in range(16):
                src = mirror_src(tid, m)
                Yp[tid, m] = XN * np.cos(np.pi * p / 4) if src is None else np.conj(Y[src])
        v = np.conj(Yp + alpha * (Y - Yp))
        y = dit(v)
        mx = max(mx, max(np.max(np.abs(y.real)), np.max(np.abs(y.imag))) / K)
    return mx


def rd(addrs):  # ds_read_b64: 2 x 32 lanes, float2 index mod 32
    extra = 0
    for g0 in (0, 32):
        banks = {}
        for a in addrs[g0:g0 + 32]:
            banks.setdefault(a % 32, set()).add(a)
        extra += max(len(s) for s in banks.values()) - 1
    return extra


def wr(addrs):  # ds_write_b64: 4 x 16 lanes, float2 index mod 16
    extra = 0
    for g0 in range(0, 64, 16):
        banks = {}
        for a in addrs[g0:g0 + 16]:
            banks.setdefault(a % 16, set()).add(a)
        extra += max(len(s) for s in banks.values()) - 1
    return extra


def conflicts():
    worst = {}

    def upd(k, v):
        worst[k] = max(worst.get(k, 0), v)
    for w in range(NTH // 64):
        lanes = range(64 * w, 64 * w + 64)
        for r in range(16):
            upd("x1w", wr([a1(tp_column(t), r) for t in lanes]))
            upd("x1r", rd([a1(p2(t)[0] + L * r, p2(t)[1]) for t in lanes]))
            upd("x2w", wr([a2(p2(t)[0], r, p2(t)[1]) for t in lanes]))
            upd("x2r", rd([a2(p3(t)[0] + 2 * r, p3(t)[1], p3(t)[2]) for t in lanes]))
            # the transposed exchanges: 2^T writes with the pass-3 pattern, reads with the pass-2 one;
            # 1^T writes with the pass-2 read pattern, reads with the pass-1 write pattern
            upd("x2Tw", wr([a2(p3(t)[0] + 2 * r, p3(t)[1], p3(t)[2]) for t in lanes]))
            upd("x2Tr", rd([a2(p2(t)[0], r, p2(t)[1]) for t in lanes]))
            upd("x1Tw", wr([a1(p2(t)[0] + L * r, p2(t)[1]) for t in lanes]))
            upd("x1Tr", rd([a1(tp_column(t), r) for t in lanes]))
    return worst


def wave_local():
    """exchange 2 / 2^T touch only the wave's own exchange-1 rows"""
    bad = 0
    for w in range(NTH // 64):
        rows = {p2(t)[1] for t in range(64 * w, 64 * w + 64)}
        bad += len(rows) != 2
        for t in range(64 * w, 64 * w + 64):
            bad += p3(t)[2] not in rows
    return bad


if __name__ == "__main__":
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    from oracle import omega_ref as R
    rng = np.random.default_rng(0)
    z = rng.standard_normal(K) + 1j * rng.standard_normal(K)
    Zo = dif(z)
    F = np.fft.fft(z)
    print("dif err", max(abs(Zo[t, m] - F[out_index(t, m)]) for t in range(NTH) for m in range(16)) / np.max(np.abs(F)))
    D = rng.standard_normal(K) + 1j * rng.standard_normal(K)
    v = np.array([[D[out_index(t, m)] for m in range(16)] for t in range(NTH)])
    y = dit(v)
    FD = np.fft.fft(D)
    print("dit err", max(abs(y[t, r] - FD[tp_column(t) + NTH * r]) for t in range(NTH) for r in range(16)) / np.max(np.abs(FD)))
    print("mirror errors", check_mirrors(), "wave-local violations", wave_local())
    print("conflicts", conflicts())
    x = (0.25 * np.sin(2 * np.pi * 440 * np.arange(2 * K) / 48000) + 0.05 * rng.standard_normal(2 * K))
    tp = truepeak(x)
    print("true peak model", 20 * np.log10(tp), "oracle", R.true_peak(x.astype(np.float32)))
