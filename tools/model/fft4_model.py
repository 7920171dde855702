#!/usr/bin/env python3
"""Numpy model of the wave-decomposed block FFT (fft4.hpp): checks the index algebra against
np.fft and counts LDS bank conflicts of every exchange, for each (K, NTH) plan.

K = E * NTH (E = 16 or 8 elements per thread), NW = NTH / 64 waves.
  stage 0 (registers): radix E over n0, n = t + NTH*n0, twiddle W_K^{t k0}
  block exchange (NW > 1): wave w takes sub-FFTs k0 in [wQ, wQ+Q), Q = E/NW; lane l reads
      n1 = 0..NW-1 at 64 n1 + l
  stage 1 (registers, NW > 1): radix NW over n1, twiddle W_S^{l k1} (S = NTH)
  64-point part on lane l = 8a + b: exchange A, radix 8 over a (twiddle W_64^{b c}),
      exchange B, radix 8 over b -> d
  output k = k0 + E (k1 + NW (c + 8 d))
"""
import itertools
import sys

import numpy as np


def brev(m, r):
    bits = r.bit_length() - 1
    return int(format(m, f"0{bits}b")[::-1], 2) if bits else 0


def dft(v):
    return np.fft.fft(v)


def conflicts_read_b64(addrs):
    """addrs: float2 indices of 64 lanes (None = inactive). ds_read_b64: 2 groups of 32 lanes, bank of
    dword address (2e) mod 64 -> e mod 32 (each access covers banks 2e, 2e+1). Returns extra cycles."""
    extra = 0
    for g in (range(0, 32), range(32, 64)):
        banks = {}
        for l in g:
            e = addrs[l]
            if e is None:
                continue
            banks.setdefault(e % 32, set()).add(e)
        if banks:
            extra += max(len(s) for s in banks.values()) - 1
    return extra


def conflicts_write_b64(addrs):
    """ds_write_b64: 4 groups of 16 contiguous lanes, bank (dword) mod 32 -> e mod 16."""
    extra = 0
    for g0 in range(0, 64, 16):
        banks = {}
        for l in range(g0, g0 + 16):
            e = addrs[l]
            if e is None:
                continue
            banks.setdefault(e % 16, set()).add(e)
        if banks:
            extra += max(len(s) for s in banks.values()) - 1
    return extra


def swz_a(s, l):
    """exchange A layout: (s, l) -> s*64 + (l ^ hA(s))."""
    return s * 64 + (l ^ (((s & 3) << 3) | ((s >> 2) & 1)))


E_CUR = [16]


def swz_b(s, c, b):
    """exchange B layout: (s, c, b) -> s*64 + ((8c + b) ^ hB(s, c)); the mask touches bits 0-3 and
    depends only on s and bit 5 (c2), so each row stays a permutation."""
    return s * 64 + ((8 * c + b) ^ hB(s, c))


def hB(s, c):
    c2 = (c >> 2) & 1
    if E_CUR[0] == 16:
        return (s & 1) | (((s >> 2) & 1) << 1) | (c2 << 2) | (((s >> 1) & 1) << 3)
    return (s & 1) | (((s >> 1) & 1) << 1) | (c2 << 2) | ((s & 1) << 3)


def swz_out(k):
    return k ^ OUT_SWZ[0](k)


OUT_SWZ = [lambda k: 0]


def model(K, NTH, verbose=False):
    E = K // NTH
    E_CUR[0] = E
    NW = NTH // 64
    S = NTH
    x = (np.random.default_rng(K).standard_normal(K) + 1j * np.random.default_rng(K + 1).standard_normal(K))
    ref = np.fft.fft(x)
    WK = np.exp(-2j * np.pi / K)
    # stage 0
    Y = np.zeros((E, NTH), complex)   # Y[k0][t]
    for t in range(NTH):
        v = np.array([x[t + NTH * n0] for n0 in range(E)])
        out = dft(v)
        for k0 in range(E):
            Y[k0, t] = out[k0] * WK ** (t * k0)
    report = {}
    # block exchange: LDS[k0*S + t]
    Q = E // NW if NW > 1 else E
    waves = []
    if NW > 1:
        wr = 0
        for k0 in range(E):           # one store per k0 per thread; check per wave-instruction
            for w in range(NW):
                wr += conflicts_write_b64([k0 * S + w * 64 + l for l in range(64)])
        rd = 0
        for w in range(NW):
            for q in range(Q):
                for n1 in range(NW):
                    rd += conflicts_read_b64([(w * Q + q) * S + 64 * n1 + l for l in range(64)])
        report["block_w"], report["block_r"] = wr, rd
        WS = np.exp(-2j * np.pi / S)
        for w in range(NW):
            Z = {}   # Z[(s)][l], s = q*NW + k1 ; also keep (k0, k1)
            meta = {}
            for q in range(Q):
                k0 = w * Q + q
                for l in range(64):
                    u = np.array([Y[k0, 64 * n1 + l] for n1 in range(NW)])
                    o = dft(u)
                    for k1 in range(NW):
                        s = q * NW + k1
                        Z.setdefault(s, np.zeros(64, complex))[l] = o[k1] * WS ** (l * k1)
                        meta[s] = (k0, k1)
            waves.append((Z, meta))
    else:
        Z = {k0: Y[k0].copy() for k0 in range(E)}
        meta = {k0: (k0, 0) for k0 in range(E)}
        waves.append((Z, meta))
    X = np.zeros(K, complex)
    W64 = np.exp(-2j * np.pi / 64)
    G = E // 8
    ca_w = ca_r = cb_w = cb_r = 0
    co_w = [0]
    for Z, meta in waves:
        # exchange A: write (s, l) at swz_a
        for s in range(E):
            ca_w += conflicts_write_b64([swz_a(s, l) for l in range(64)])
        for i in range(G):
            for a in range(8):
                addrs = []
                for L in range(64):
                    g = L * G + i
                    s, b = g >> 3, g & 7
                    addrs.append(swz_a(s, 8 * a + b))
                ca_r += conflicts_read_b64(addrs)
        T = {}
        for L in range(64):
            for i in range(G):
                g = L * G + i
                s, b = g >> 3, g & 7
                v = np.array([Z[s][8 * a + b] for a in range(8)])
                o = dft(v)
                for c in range(8):
                    T[(s, c, b)] = o[c] * W64 ** (b * c)
        # exchange B writes: lane L (groups (s,b)) writes c = 0..7
        for i in range(G):
            for c in range(8):
                addrs = []
                for L in range(64):
                    g = L * G + i
                    s, b = g >> 3, g & 7
                    addrs.append(swz_b(s, c, b))
                cb_w += conflicts_write_b64(addrs)
        for i in range(G):
            for b in range(8):
                addrs = []
                for L in range(64):
                    g = L * G + i
                    s, c = g >> 3, g & 7
                    addrs.append(swz_b(s, c, b))
                cb_r += conflicts_read_b64(addrs)
        for i in range(G):
            for d in range(8):
                addrs = []
                for L in range(64):
                    g = L * G + i
                    s, c = g >> 3, g & 7
                    k0, k1 = meta[s]
                    k = k0 + E * (k1 + NW * (c + 8 * d)) if NW > 1 else k0 + E * (c + 8 * d)
                    addrs.append(swz_out(k))
                co_w[0] += conflicts_write_b64(addrs)
        for L in range(64):
            for i in range(G):
                g = L * G + i
                s, c = g >> 3, g & 7
                v = np.array([T[(s, c, b)] for b in range(8)])
                o = dft(v)
                k0, k1 = meta[s]
                for d in range(8):
                    k = k0 + E * (k1 + NW * (c + 8 * d)) if NW > 1 else k0 + E * (c + 8 * d)
                    X[k] = o[d]
    # swizzle bijectivity
    assert sorted(swz_a(s, l) for s in range(E) for l in range(64)) == list(range(E * 64))
    assert sorted(swz_b(s, c, b) for s in range(E) for c in range(8) for b in range(8)) == list(range(E * 64))
    err = np.max(np.abs(X - ref)) / np.max(np.abs(ref))
    # untangle-style reads of the output: k = tid + j*NTH (j-th round) and K - k
    ur = 0
    for j in range((K // 2 + NTH - 1) // NTH):
        for w in range(NW if NW else 1):
            ks = [w * 64 + l + j * NTH for l in range(64)]
            ur += conflicts_read_b64([swz_out(k) if k < K // 2 else None for k in ks])
            ur += conflicts_read_b64([swz_out(K - k) if 0 < k < K // 2 else None for k in ks])
    assert sorted(swz_out(k) for k in range(K)) == list(range(K))
    report.update(A_w=ca_w, A_r=ca_r, B_w=cb_w, B_r=cb_r, out_w=co_w[0], untangle_r=ur)
    return err, report


if __name__ == "__main__":
    if len(sys.argv) > 1:
        OUT_SWZ[0] = eval(sys.argv[1])
    for K, NTH in ((8192, 512), (4096, 256), (2048, 128), (1024, 64), (512, 64)):
        err, rep = model(K, NTH)
        print(K, NTH, f"err {err:.2e}", rep)
