#!/usr/bin/env python3
"""Numpy model of the meter prep / query index algebra (csrc/meters.hip meter_prep_kernel,
csrc/meter_query.hpp meter_query_wave): the core (history gated keys inside every window of the
batch), the extras (evicted history keys merged with the batch's by rank, each with its core count
below), the time-order prefixes and the next sorted history -- checked against the oracle's
MeterState over random batch sequences (tests/test_layout_model.py)."""
import bisect

import numpy as np


def fkey(v):
    u = np.float32(v).view(np.uint32).item()
    return (~u) & 0xFFFFFFFF if u & 0x80000000 else u | 0x80000000


class Model:
    def __init__(self, HL=3599, HT=59, mom=24, short=180, integ=3600, peak=60, gate=-70.0):
        self.HL, self.HT, self.mom, self.short, self.integ, self.peak, self.gate = HL, HT, mom, short, integ, peak, gate
        self.hist_l, self.hist_t, self.skeys, self.T0 = [], [], [], 0

    def window_lo(self, T0, nh, f):
        n = nh + f + 1
        return T0 - nh + (n - min(self.integ, n))

    def batch(self, li, tp):
        F = len(li)
        T0, nh, A = self.T0, len(self.hist_l), self.skeys
        ns, L = len(A), nh + F
        thr = T0 + F - self.HL
        clo, chi = self.window_lo(T0, nh, F - 1), T0 - 1
        has_core = chi >= clo
        inc = [has_core and (k & 0xFFFFFFFF) >= clo for k in A]
        kep = [(k & 0xFFFFFFFF) >= thr for k in A]
        cpA = np.concatenate([[0], np.cumsum(inc)]).astype(int)
        kpA = np.concatenate([[0], np.cumsum(kep)]).astype(int)
        core = [np.float32(np.uint32(0)) for _ in range(cpA[-1])]
        for i, k in enumerate(A):
            if inc[i]:
                core[cpA[i]] = self.unkey(k >> 32)
        seq = list(self.hist_l) + [np.float32(v) for v in li]
        gp = [0] * (L + 1)
        gs = [0.0] * (L + 1)
        for u in range(L):
            g = seq[u] > self.gate
            gp[u + 1] = gp[u] + g
            gs[u + 1] = gs[u] + (float(seq[u]) if g else 0.0)
        B = sorted(((fkey(v) << 32) | (T0 + f)) for f, v in enumerate(li) if np.float32(v) > self.gate)
        Gn = len(B)
        ext = [None] * ((ns - cpA[ns]) + Gn)
        for j, kb in enumerate(B):
            ra = bisect.bisect_left(A, kb)
            ext[j + (ra - cpA[ra])] = (self.unkey(kb >> 32), kb & 0xFFFFFFFF, cpA[ra])
        for i, ka in enumerate(A):
            if not inc[i]:
                rb = bisect.bisect_left(B, ka)
                ext[(i - cpA[i]) + rb] = (self.unkey(ka >> 32), ka & 0xFFFFFFFF, cpA[i])
        assert all(e is not None for e in ext)
        out = []
        for f in range(F):
            out.append(self.query(f, F, T0, nh, seq, gp, gs, core, ext, clo, chi, has_core, tp))
        # next state
        kb_ = np.concatenate([[0], np.cumsum([(k & 0xFFFFFFFF) >= thr for k in B])]).astype(int)
        S = [None] * (kpA[ns] + kb_[Gn])
        for i, ka in enumerate(A):
            if kep[i]:
                S[kpA[i] + kb_[bisect.bisect_left(B, ka)]] = ka
        for j, kb in enumerate(B):
            if (kb & 0xFFFFFFFF) >= thr:
                S[kb_[j] + kpA[bisect.bisect_left(A, kb)]] = kb
        assert all(x is not None for x in S) and S == sorted(S)
        self.skeys = S
        klen = min(self.HL, L)
        self.hist_l = seq[L - klen:]
        tt = list(self.hist_t) + [np.float32(v) for v in tp]
        self.hist_t = tt[len(tt) - min(self.HT, len(tt)):]
        self.T0 = T0 + F
        return np.array(out)

    @staticmethod
    def unkey(k):
        k &= 0xFFFFFFFF
        u = (k & 0x7FFFFFFF) if k & 0x80000000 else (~k) & 0xFFFFFFFF
        return np.uint32(u).view(np.float32)

    def query(self, f, F, T0, nh, seq, gp, gs, core, ext, clo, chi, has_core, tp):
        n = nh + f + 1
        wm, ws = min(self.mom, n), min(self.short, n)
        mom = np.mean([float(v) for v in seq[n - wm:n]])
        sh = np.mean([float(v) for v in seq[n - ws:n]])
        wi = min(self.integ, n)
        ng = gp[n] - gp[n - wi]
        integ, rng = -100.0, 0.0
        if ng > 0:
            integ = (gs[n] - gs[n - wi]) / ng
            lo, hi = self.window_lo(T0, nh, f), T0 + f
            want, gam = [], []
            for q in (0.10, 0.95):
                vi = (ng - 1) * q
                prev = int(np.floor(vi))
                if vi >= ng - 1:
                    prev = ng - 1
                want += [prev, min(prev + 1, ng - 1)]
                gam.append(vi - np.floor(vi))
            mem = [e for e in ext if lo <= e[1] <= hi and not (has_core and clo <= e[1] <= chi)]
            val = [None] * 4
            below = [0] * 4
            for jb, e in enumerate(mem):
                rank = jb + e[2]
                for w in range(4):
                    if rank < want[w]:
                        below[w] += 1
                    if rank == want[w]:
                        val[w] = e[0]
            for w in range(4):
                if val[w] is None:
                    val[w] = core[want[w] - below[w]]

            def lerp(a, b, g):
                d = float(b) - float(a)
                return float(b) - d * (1 - g) if g >= 0.5 else float(a) + d * g
            rng = lerp(val[2], val[3], gam[1]) - lerp(val[0], val[1], gam[0])
        th = list(self.hist_t) + [np.float32(v) for v in tp[:f + 1]]
        return [mom, sh, integ, rng, float(max(th[-self.peak:]))]
