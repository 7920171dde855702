#!/usr/bin/env python3
"""Numpy model of the register-resident block FFT (csrc/regfft.hpp) and the true-peak flow built on
it: checks the index algebra against np.fft / the oracle and counts LDS bank conflicts of every
exchange, for K = 8192 (512 threads, L = 32) and K = 4096 (256 threads, L = 16).

  pass 1 (thread t):           a[r] = x[t + NTH r]      DFT16 over r -> k1, twiddle W_K^{t k1}
  exchange 1 -> (u, k1):       b[v] = B_{u + L v}[k1]   DFT16 over v -> k2, twiddle W_K^{16 u k2}
  exchange 2 -> pass 3:
     L = 16, thread (k2, k1):  c[u] = C_u[k2][k1]       DFT16 over u -> m; X[k1 + 16 k2 + 256 m]
     L = 32, thread (q, k2, k1), q = lane bit 0: c[u'] = C_{q + 2u'}; DFT16 over u' -> m;
        odd lanes * w32^m; lane pair butterfly -> X[k1 + 16 k2 + 256 (m + 16 q)]
"""
import sys

import numpy as np


def conflicts(addrs, group, mod):
    """extra LDS cycles: lanes split in groups of `group` consecutive lanes; bank = addr % mod
    (float2 units). Identical addresses broadcast."""
    extra = 0
    for g0 in range(0, 64, group):
        banks = {}
        for l in range(g0, g0 + group):
            banks.setdefault(addrs[l] % mod, set()).add(addrs[l])
        extra += max(len(s) for s in banks.values()) - 1
    return extra


def rd(addrs):  # ds_read_b64: 2 x 32 lanes, float2 index mod 32
    return conflicts(addrs, 32, 32)


def wr(addrs):  # ds_write_b64: 4 x 16 lanes, float2 index mod 16
    return conflicts(addrs, 16, 16)


class Plan:
    def __init__(self, K):
        self.K = K
        self.NTH = K // 16
        self.L = K // 256

    # ---- swizzles (float2 index -> LDS slot) ----
    # padded layouts: every slot is a per-thread base plus a compile-time offset per register
    def a1(self, t, k1):
        return k1 * (544 if self.L == 32 else 272) + t  # the same row stride as a2 (wave-local exchange 2)

    def a2(self, u, k2, k1):
        if self.L == 32:
            return k1 * 544 + 34 * k2 + u
        return k1 * 272 + 17 * k2 + u

    def a3(self, n):
        if self.K == 8192:
            return n + (n >> 4) + ((n >> 12) << 3)
        return n ^ ((n >> 4) & 15)  # (round 4: the padded n + n / 16 left the untangle's reads 2-way)

    # ---- thread maps ----
    def p2(self, tau):
        return tau % self.L, tau // self.L  # u, k1

    def p3(self, s):
        if self.L == 32:
            return s & 1, (s >> 1) & 15, s >> 5  # q, k2, k1
        return 0, s & 15, s >> 4

    def out_index(self, s, m):
        q, k2, k1 = self.p3(s)
        return k1 + 16 * k2 + 256 * (m + 16 * q)

    def fft(self, x):
        K, NTH, L = self.K, self.NTH, self.L
        W = np.exp(-2j * np.pi / K)
        lds = np.zeros(K + K // 16 + 16, complex)
        # pass 1
        B = np.zeros((NTH, 16), complex)
        for t in range(NTH):
            A = np.fft.fft(x[t + NTH * np.arange(16)])
            B[t] = A * W ** (t * np.arange(16))
            for k1 in range(16):
                lds[self.a1(t, k1)] = B[t, k1]
        # pass 2
        C = np.zeros((NTH, 16), complex)
        for tau in range(NTH):
            u, k1 = self.p2(tau)
            b = np.array([lds[self.a1(u + L * v, k1)] for v in range(16)])
            C[tau] = np.fft.fft(b) * W ** (16 * u * np.arange(16))
        for tau in range(NTH):
            u, k1 = self.p2(tau)
            for k2 in range(16):
                lds[self.a2(u, k2, k1)] = C[tau, k2]
        # pass 3
        out = np.zeros((NTH, 16), complex)
        for s in range(NTH):
            q, k2, k1 = self.p3(s)
            if L == 16:
                c = np.array([lds[self.a2(u, k2, k1)] for u in range(16)])
                out[s] = np.fft.fft(c)
            else:
                c = np.array([lds[self.a2(q + 2 * up, k2, k1)] for up in range(16)])
                out[s] = np.fft.fft(c)
        if L == 32:
            w32 = np.exp(-2j * np.pi / 32) ** np.arange(16)
            F = out.copy()
            for s in range(NTH):
                if s & 1:
                    F[s] *= w32
            for s in range(NTH):
                own, par = F[s], F[s ^ 1]
                out[s] = own + par if not (s & 1) else par - own
        X = np.zeros(K, complex)
        for s in range(NTH):
            for m in range(16):
                X[self.out_index(s, m)] = out[s, m]
        return X

    def check_conflicts(self):
        K, NTH, L = self.K, self.NTH, self.L
        worst = {}
        for w in range(NTH // 64):
            lanes = [w * 64 + l for l in range(64)]
            for r in range(16):
                worst["x1w"] = max(worst.get("x1w", 0), wr([self.a1(t, r) for t in lanes]))
                worst["x1r"] = max(worst.get("x1r", 0), rd([self.a1(self.p2(t)[0] + L * r, self.p2(t)[1]) for t in lanes]))
                worst["x2w"] = max(worst.get("x2w", 0), wr([self.a2(*self.p2(t)[:1], r, self.p2(t)[1]) for t in lanes]))
                if L == 32:
                    ad = [self.a2(self.p3(s)[0] + 2 * r, self.p3(s)[1], self.p3(s)[2]) for s in lanes]
                else:
                    ad = [self.a2(r, self.p3(s)[1], self.p3(s)[2]) for s in lanes]
                worst["x2r"] = max(worst.get("x2r", 0), rd(ad))
                worst["x3w"] = max(worst.get("x3w", 0), wr([self.a3(self.out_index(s, r)) for s in lanes]))
                worst["x3r"] = max(worst.get("x3r", 0), rd([self.a3(t + NTH * r) for t in lanes]))
                worst["x3m"] = max(worst.get("x3m", 0), rd([self.a3((K - t - NTH * r) % K) for t in lanes]))
        return worst


class TightPlan4096(Plan):
    """The tight K = 4096 layout (RegFFT<4096, true>): exactly K slots, XOR swizzles instead of padding."""

    def __init__(self):
        super().__init__(4096)

    def a1(self, t, k1):
        return 256 * k1 + (t ^ (16 * (k1 & 1)))

    def a2(self, u, k2, k1):
        return 256 * k1 + 16 * (k2 ^ (k1 & 1)) + (u ^ k2)

    def a3(self, n):
        return n ^ ((n >> 4) & 15)


class HalfPlan4096(Plan):
    """RegFFT<4096>::run_half (the cfg3 kernel at five workgroups per CU): the padded K = 4096 slot maps
    in FLOAT units, real parts then imaginary parts through one buffer of 4352 floats; every exchange
    access is ds_read_b32 / ds_write_b32 (2 x 32 lanes, bank = float index mod 32)."""

    def __init__(self):
        super().__init__(4096)

    def check_conflicts(self):
        K, NTH, L = self.K, self.NTH, self.L
        r32 = lambda a: conflicts(a, 32, 32)  # noqa: E731  (both instructions: groups of 32, mod 32)
        worst = {}
        for w in range(NTH // 64):
            lanes = [w * 64 + l for l in range(64)]
            for r in range(16):
                worst["x1w"] = max(worst.get("x1w", 0), r32([self.a1(t, r) for t in lanes]))
                worst["x1r"] = max(worst.get("x1r", 0), r32([self.a1(self.p2(t)[0] + L * r, self.p2(t)[1]) for t in lanes]))
                worst["x2w"] = max(worst.get("x2w", 0), r32([self.a2(self.p2(t)[0], r, self.p2(t)[1]) for t in lanes]))
                worst["x2r"] = max(worst.get("x2r", 0), r32([self.a2(r, self.p3(s)[1], self.p3(s)[2]) for s in lanes]))
                worst["x3w"] = max(worst.get("x3w", 0), r32([self.a3(self.out_index(s, r)) for s in lanes]))
                worst["x3r"] = max(worst.get("x3r", 0), r32([self.a3(t + NTH * r) for t in lanes]))
                worst["x3m"] = max(worst.get("x3m", 0), r32([self.a3((K - t - NTH * r) % K) for t in lanes]))
        return worst


def check_tight():
    pl = TightPlan4096()
    rng = np.random.default_rng(1)
    x = rng.standard_normal(4096) + 1j * rng.standard_normal(4096)
    err = np.max(np.abs(pl.fft(x) - np.fft.fft(x))) / np.max(np.abs(np.fft.fft(x)))
    slots = [{pl.a1(t, k1) for t in range(256) for k1 in range(16)},
             {pl.a2(u, k2, k1) for u in range(16) for k2 in range(16) for k1 in range(16)},
             {pl.a3(n) for n in range(4096)}]
    assert all(len(s) == 4096 and max(s) == 4095 for s in slots), "each exchange a bijection onto 4096 slots"
    for t in range(256):  # the kernel's separable forms: base per thread + immediate offset per register
        for r in range(16):
            assert pl.a3(t + 256 * r) == (t ^ ((t >> 4) & 15)) + 256 * r
            if t:
                assert pl.a3(4096 - t - 256 * r) == ((256 - t) ^ (((256 - t) >> 4) & 15)) + 256 * (15 - r)
    for s_ in range(256):
        for m in range(16):
            assert pl.a3(pl.out_index(s_, m)) == ((s_ >> 4) ^ (s_ & 15)) + 16 * (s_ & 15) + 256 * m
    print(f"tight K=4096: fft err {err:.2e}, conflicts {pl.check_conflicts()}")


def truepeak_model(x):
    """The kernel's true-peak flow: rfft via the packed K-point FFT, untangle per thread set
    S_t = {t + NTH r}, then per phase p = 1..3: Y_k = X_k rho_k^p (running product), mirror exchange,
    Z'_k = conj(Y' + alpha_k (Y_k - Y')), Y' = conj(Y_{K-k}) (Nyquist share for k = 0), forward FFT
    -> max |.| / K."""
    M = len(x)
    K = M // 2
    pl = Plan(K)
    z = x[0::2] + 1j * x[1::2]
    Z = pl.fft(z)
    k = np.arange(K)
    wM = np.exp(-2j * np.pi * k / M)
    Zm = Z[(K - k) % K]
    E = (Z + np.conj(Zm)) / 2
    O = -1j * (Z - np.conj(Zm)) / 2
    X = E + wM * O
    X[0] = Z[0].real + Z[0].imag
    XN = Z[0].real - Z[0].imag
    rho = np.exp(2j * np.pi * k / (4 * M))
    alpha = (1 + 1j * np.conj(wM)) / 2
    Y = X.copy()
    mx = np.max(np.abs(x))
    for p in range(1, 4):
        Y = Y * rho
        Yp = np.conj(Y[(K - k) % K])
        Yp[0] = XN * np.cos(np.pi * p / 4)
        Zp = np.conj(Yp + alpha * (Y - Yp))
        out = pl.fft(Zp)
        mx = max(mx, np.max(np.maximum(np.abs(out.real), np.abs(out.imag))) / K)
    return 20 * np.log10(mx)


def main():
    if "--tight" in sys.argv:
        check_tight()
        return
    rng = np.random.default_rng(0)
    for K in (4096, 8192):
        pl = Plan(K)
        x = rng.standard_normal(K) + 1j * rng.standard_normal(K)
        err = np.max(np.abs(pl.fft(x) - np.fft.fft(x))) / np.max(np.abs(np.fft.fft(x)))
        print(f"K={K}: fft err {err:.2e}, conflicts {pl.check_conflicts()}")
    sys.path.insert(0, ".")
    from oracle import omega_ref as R
    for M in (8192, 16384):
        x = (0.25 * np.sin(2 * np.pi * 440 * np.arange(M) / 48000) + 0.05 * rng.standard_normal(M)).astype(np.float32)
        print(f"TP M={M}: model {truepeak_model(x.astype(np.float64)):.6f} oracle {R.true_peak(x):.6f}")


if __name__ == "__main__":
    main()


def wave_local_exchange2(K):
    """Exchange 2 is wave-local (regfft.hpp): the slots a wave's exchange-2 writes and pass-3 reads
    touch lie in rows whose exchange-1 slots only that wave's pass-2 threads read. Returns the number
    of violating slots (0)."""
    P = Plan(K)
    bad = 0
    for w in range(P.NTH // 64):
        own = set()
        for tau in range(64 * w, 64 * w + 64):
            u, k1 = P.p2(tau)
            own |= {P.a1(u + P.L * r, k1) for r in range(16)}  # exchange-1 reads of this wave
        rows = {a // P.a1(0, 1) for a in own}
        touched = set()
        for tau in range(64 * w, 64 * w + 64):
            u, k1 = P.p2(tau)
            touched |= {P.a2(u, k2, k1) for k2 in range(16)}
            q, k2, k1b = P.p3(tau)
            us = [q + 2 * i for i in range(16)] if P.L == 32 else list(range(16))
            touched |= {P.a2(uu, k2, k1b) for uu in us}
        bad += sum(1 for a in touched if a // P.a1(0, 1) not in rows)
        # and no other wave reads those rows in exchange 1
        for w2 in range(P.NTH // 64):
            if w2 == w:
                continue
            for tau in range(64 * w2, 64 * w2 + 64):
                u, k1 = P.p2(tau)
                bad += sum(1 for r in range(16) if P.a1(u + P.L * r, k1) in touched)
    return bad
