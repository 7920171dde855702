// Spectral device code shared by the spectral kernels (spectral.hip) and the fused frame kernel
// (the cfg2 role kernels): real-FFT magnitudes, the per-resolution frame body (A3-A5) and the true-peak body
// (A8). See spectral.hip for the algorithms. Include after OMEGA_STAMPS_DECL.
#pragma once
#include "fft.hpp"
#include "params.hpp"
#include "stamps.hpp"

namespace omega {

// raw v_sqrt_f32 (1 ulp): no denormal-scaling sequence around it
__device__ __forceinline__ float cabs(float2 z) { return __builtin_amdgcn_sqrtf(fmaf(z.x, z.x, z.y * z.y)); }

// untangle of one pair (k, K-k), 0 < k < K/2: returns X[k] and X[K-k]
__device__ __forceinline__ void untangle(float2 a, float2 b, float2 w, float2& xk, float2& xkk) {
  // E = (a + conj b)/2, O = -i (a - conj b)/2, X[k] = E + w O, X[K-k] = conj(E - w O)
  const float2 E = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
  const float2 O = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
  const float2 wo = cmul(w, O);
  xk = cadd(E, wo);
  xkk = cconj(csub(E, wo));
}

// |X[k]| of the rfft of N = 2K real points lands at float index magidx<K>(k) of buf.
template <int K, int NTH>
__device__ __forceinline__ int magidx(int k) {
  return k == K ? 2 * BlockFFT<K, NTH>::out(0) : 2 * BlockFFT<K, NTH>::out(k) + 1;
}

// Magnitudes from the packed complex FFT in buf (BlockFFT<K> output order). Pair (k, K-k) is owned
// by one thread, which overwrites only the imaginary slots of the two entries it read: no barrier
// between reads and writes, nothing held in registers. Pairs k0 <= k < k1 (pair 0 carries bins 0, K
// and K/2).
template <int K, int NTH>
__device__ __forceinline__ void rfft_magnitudes(float2* buf, const float2* __restrict__ twN, int tid, int k0 = 0,
                                                int k1 = K / 2) {
  using FFT = BlockFFT<K, NTH>;
  float* mag = reinterpret_cast<float*>(buf);
  for (int k = k0 + tid; k < k1; k += NTH) {
    if (k == 0) {
      const float2 z = buf[FFT::out(0)];
      const float2 zm = buf[FFT::out(K / 2)];
      mag[magidx<K, NTH>(0)] = fabsf(z.x + z.y);
      mag[magidx<K, NTH>(K)] = fabsf(z.x - z.y);
      mag[magidx<K, NTH>(K / 2)] = cabs(zm);  // X[K/2] = conj(Z[K/2])
    } else {
      float2 xk, xkk;
      untangle(buf[FFT::out(k)], buf[FFT::out(K - k)], twN[k], xk, xkk);
      mag[magidx<K, NTH>(k)] = cabs(xk);
      mag[magidx<K, NTH>(K - k)] = cabs(xkk);
    }
  }
  __syncthreads();
}

// Multi-resolution kernel for one resolution of K = N_r/2 complex points (A3-A5). Launched once per
// resolution, in resolution order: a target with several owners (multi_resolution_fft.py:387-395)
// is stored by its first owner's kernel and accumulated by the later ones (CombEnt).
// One resolution of one channel-frame with a group of NTH threads (tid relative to the group; the
// barriers inside are workgroup-wide, so every group of a workgroup runs the same K). valid = false:
// a padding group of a partly filled workgroup -- it takes part in the barriers only.
template <int K, int NTH>
__device__ __forceinline__ void mrfft_frame(const SpectralParams& p, int r, int64_t cf, bool valid, int tid, float2* buf) {
  const int64_t f = cf / p.C, c = cf % p.C;
  const ResParam& rp = p.res[r];
  const float* __restrict__ x = p.x + f * p.frame_stride + c * p.chan_stride + rp.offset;
  const float2* x2 = reinterpret_cast<const float2*>(x);
  const float2* w2 = reinterpret_cast<const float2*>(rp.win);
  // twiddles and this thread's first combine entries are fetched together with the frame: one
  // global-memory latency before the transform instead of one per pass and per epilogue load
  using FFT = BlockFFT<K, NTH>;
  OMEGA_STAMP(10 + 4 * (ilog2(K) - 9));
  const typename FFT::Tw tw = FFT::load_tw(p.tw[ilog2(K)], tid);
  constexpr int EP = NTH >= 256 ? 1 : (NTH >= 128 ? 256 / NTH : 512 / NTH);
  CombEnt ent[EP];
  static_for<0, EP>([&](auto i) {
    const int e = rp.ent_begin + tid + i * NTH;
    if (p.comb_out && e < rp.ent_end) ent[i] = p.ent[e];
  });
  // the first FFT pass reads the windowed frame straight from global memory (coalesced float2)
  FFT::run_from(buf, tw, tid, [&](int i) {
    const float2 a = valid ? x2[i] : make_float2(0.f, 0.f), w = w2[i];
    return make_float2(a.x * w.x, a.y * w.y);
  });
  OMEGA_STAMP(11 + 4 * (ilog2(K) - 9));
  const bool pair_range = !rp.mag_out && rp.pair_hi > 0;
  if (!rp.mag_out && !pair_range) {
    // combine only (no magnitude output; uniform over the workgroup's groups): each entry untangles
    // the two bins it reads straight from the packed spectrum -- the combine reads a few hundred of
    // the K + 1 bins, so the all-bin magnitude pass and its barrier are skipped
    if (!valid || !p.comb_out) return;
    const float2* __restrict__ twN = p.tw[ilog2(2 * K)];
    auto mag_at = [&](int j) -> float {  // |X_j|, 0 <= j <= K
      const float2 a = buf[FFT::out(j == K ? 0 : j)];
      if (j == 0) return fabsf(a.x + a.y);
      if (j == K) return fabsf(a.x - a.y);
      if (j == K / 2) return cabs(a);  // X[K/2] = conj(Z[K/2])
      float2 xk, xkk;
      untangle(a, buf[FFT::out(K - j)], twN[j], xk, xkk);
      return cabs(xk);
    };
    float* o = p.comb_out + cf * p.T;
    auto apply = [&](const CombEnt& en) {
      const int t = en.tm & 0xFFFFFF, op = en.tm >> 24;
      if (op == 2) {
        o[t] = 0.f;
        return;
      }
      const float v = fmaf(en.c1, mag_at(en.j + 1), en.c0 * mag_at(en.j));
      if (op == 0)
        o[t] = v;
      else
        o[t] += v;
    };
    static_for<0, EP>([&](auto i) {
      if (rp.ent_begin + tid + i * NTH < rp.ent_end) apply(ent[i]);
    });
    for (int e = rp.ent_begin + tid + EP * NTH; e < rp.ent_end; e += NTH) apply(p.ent[e]);
    return;
  }
  // (combine only over many bins: just the pairs the entries read, ResParam::pair_lo / pair_hi)
  rfft_magnitudes<K, NTH>(buf, p.tw[ilog2(2 * K)], tid, pair_range ? rp.pair_lo : 0, pair_range ? rp.pair_hi : K / 2);
  OMEGA_STAMP(12 + 4 * (ilog2(K) - 9));
  if (!valid) return;
  const float* mag = reinterpret_cast<const float*>(buf);
  const float* __restrict__ wgt = rp.wgt;
  if (rp.mag_out) {
    float* o = rp.mag_out + cf * (K + 1);
    for (int k = tid; k <= K; k += NTH) o[k] = mag[magidx<K, NTH>(k)] * wgt[k];
  }
  if (p.comb_out) {
    float* o = p.comb_out + cf * p.T;
    auto apply = [&](const CombEnt& en) {
      const int t = en.tm & 0xFFFFFF, op = en.tm >> 24;
      const float v = fmaf(en.c1, mag[magidx<K, NTH>(en.j + 1)], en.c0 * mag[magidx<K, NTH>(en.j)]);
      if (op == 0)
        o[t] = v;
      else if (op == 1)
        o[t] += v;
      else
        o[t] = 0.f;
    };
    static_for<0, EP>([&](auto i) {
      if (rp.ent_begin + tid + i * NTH < rp.ent_end) apply(ent[i]);
    });
    for (int e = rp.ent_begin + tid + EP * NTH; e < rp.ent_end; e += NTH) apply(p.ent[e]);
  }
  OMEGA_STAMP(13 + 4 * (ilog2(K) - 9));
}

// True-peak workgroup size: 1024 threads (16 waves, 4 per SIMD) for the 8192-point transforms.
template <int K>
constexpr int tp_threads() { return K == 8192 ? 1024 : threads_for<K>(); }

// True peak of one frame of M = 2K samples (dBTP; float32 like scipy on float32 input). The four
// transforms ping-pong between two K-point LDS buffers (one barrier per pass).
template <int K, int NTH>
__device__ __forceinline__ void truepeak_body(const SpectralParams& p, int64_t cf, int tid, float2* bufA, float2* bufB,
                                              float* red) {
  constexpr int M = 2 * K;
  using FFT = BlockFFT<K, NTH>;
  const int64_t f = cf / p.C, c = cf % p.C;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride);
  float mx = 0.f;  // p = 0 phase: the samples themselves (every one is loaded exactly once below)
  OMEGA_STAMP(0);
  const typename FFT::Tw tw = FFT::load_tw(p.tw[ilog2(K)], tid);  // shared by all four transforms
  const float2* buf = FFT::run_from_pp(bufA, bufB, tw, tid, [&](int i) {
    const float2 a = x2[i];
    mx = fmaxf(mx, fmaxf(fabsf(a.x), fabsf(a.y)));
    return a;
  });
  OMEGA_STAMP(1);
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  constexpr int NP = K / 2;  // pairs (k, K-k), k < K/2; k = 0 carries X[0], X[K] and X[K/2]
  constexpr int PB = (NP + NTH - 1) / NTH;
  float2 Xlo[PB], Xhi[PB];
  float2 Xmid = make_float2(0.f, 0.f);
  static_for<0, PB>([&](auto b) {
    const int k = tid + b * NTH;
    if (NP % NTH == 0 || k < NP) {
      // branch-free selects keep Xlo/Xhi in registers (a conditional write through a reference
      // to an array element sent the arrays to scratch)
      const int kk = k == 0 ? K / 2 : K - k;
      const float2 a = buf[FFT::out(k)], bz = buf[FFT::out(kk)];
      float2 lo, hi;
      untangle(a, bz, twM[k], lo, hi);
      if (k == 0) Xmid = cconj(bz);
      Xlo[b] = k == 0 ? make_float2(a.x + a.y, 0.f) : lo;
      Xhi[b] = k == 0 ? make_float2(a.x - a.y, 0.f) : hi;
    }
  });
  // Phase P multiplies X_k by r_k^P (r_k = e^{2 pi i k / 4M}) and X_{K-k} by q_k^P
  // (q_k = e^{2 pi i (K-k) / 4M} = e^{i pi/4} conj r_k): carried as running products, one complex
  // multiply per value and phase; e_k = r_k^4 = e^{2 pi i k / M} is phase-independent.
  const float2* __restrict__ rot = p.rot;  // e^{2 pi i k / 4M}, k <= K
  constexpr float kS2 = 7.071067812e-01f;
  float2 rk[PB], ek[PB];
  static_for<0, PB>([&](auto b) {
    const int k = tid + b * NTH;
    rk[b] = (NP % NTH == 0 || k < NP) ? rot[k] : make_float2(1.f, 0.f);
    const float2 r2 = cmul(rk[b], rk[b]);
    ek[b] = cmul(r2, r2);
  });
  const float2 rh = rot[K / 2];
  float fmx = 0.f;
  // transform P writes its input into `zin` and runs zin -> zalt -> zin ...; the next transform's
  // input goes to the buffer the previous one's last pass did not read
  constexpr bool kOddPasses = FFT::kPasses % 2 == 1;
  OMEGA_STAMP(2);
  int zsel = buf == bufA ? 1 : 0;  // input buffer of the next transform: not the one the untangle reads
#pragma unroll 1
  for (int P = 1; P <= 3; ++P) {
    // opaque per-iteration values: stop LICM from hoisting (and keeping live across the loop) the
    // twiddle powers of the three inverse transforms (tid is laundered too: otherwise every LDS
    // address of the inlined FFT, a function of tid alone, is hoisted out of the loop and pinned
    // in VGPRs)
    int tl = tid;
    typename FFT::Tw twl = tw;
    twl.launder();
    asm volatile("" : "+v"(tl));
    float2* zin = zsel ? bufB : bufA;
    float2* zalt = zsel ? bufA : bufB;
    if (!((p.tp_phases >> P) & 1)) {  // phase not requested (oversampling 2 or 1): advance the rotations only
      static_for<0, PB>([&](auto b) {
        const int k = tl + b * NTH;
        if (NP % NTH == 0 || k < NP) {
          const float2 r1 = rk[b];
          Xlo[b] = cmul(Xlo[b], r1);
          Xhi[b] = cmul(Xhi[b], make_float2(kS2 * (r1.x + r1.y), kS2 * (r1.x - r1.y)));
          if (k == 0) Xmid = cmul(Xmid, rh);
        }
      });
      continue;
    }
    static_for<0, PB>([&](auto b) {
      const int k = tl + b * NTH;
      if (NP % NTH == 0 || k < NP) {
        const float2 r1 = rk[b];
        const float2 q1 = make_float2(kS2 * (r1.x + r1.y), kS2 * (r1.x - r1.y));
        Xlo[b] = cmul(Xlo[b], r1);
        Xhi[b] = cmul(Xhi[b], q1);
        const float2 yk = Xlo[b];
        // k = 0 carries the Nyquist bin X_K (real): its share is Re(X_K e^{i pi P/4}) = X_K cos(pi P/4)
        const float2 ykk = (k == 0) ? make_float2(Xhi[b].x, 0.f) : Xhi[b];
        // Z'[k] = E + iO, Z'[K-k] = conj(E) + i conj(O); E = (Y_k + conj Y_{K-k})/2,
        // O = (Y_k - conj Y_{K-k})/2 e. Stored conjugated: a forward FFT then gives conj(ifft).
        const float2 E = make_float2(0.5f * (yk.x + ykk.x), 0.5f * (yk.y - ykk.y));
        const float2 O = cmul(make_float2(0.5f * (yk.x - ykk.x), 0.5f * (yk.y + ykk.y)), ek[b]);
        zin[k] = make_float2(E.x - O.y, -(E.y + O.x));
        if (k != 0) {
          zin[K - k] = make_float2(E.x + O.y, E.y - O.x);
        } else {
          // k = K/2: Z'[K/2] = conj(Y[K/2]), Y[K/2] = X[K/2] rot^P(K/2); stored conjugated = Y
          Xmid = cmul(Xmid, rh);
          zin[K / 2] = Xmid;
        }
      }
    });
    OMEGA_STAMP(1 + 2 * P);
    __syncthreads();
    // the last pass reduces straight from registers: no LDS write of the inverse transform
    FFT::run_to_pp(zin, zalt, twl, tl, [&](int, float2 z) { fmx = fmaxf(fmx, fmaxf(fabsf(z.x), fabsf(z.y))); });
    // the last pass read zin (odd pass count: passes read zin, zalt, zin, ...) -> next input in zalt
    if (kOddPasses) zsel ^= 1;
    OMEGA_STAMP(2 + 2 * P);
  }
  const float peak = block_max<NTH>(fmaxf(mx, fmx * (1.0f / K)), red, tid);
  if (tid == 0) {
    const float db = peak < 1e-10f ? -100.0f : 20.0f * log10f(peak);
    if (p.tp_done) {  // write-through, drained, then counted in (see SpectralParams::tp_done)
      __hip_atomic_store(reinterpret_cast<unsigned*>(p.tp_out + cf), __float_as_uint(db), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(p.tp_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      p.tp_out[cf] = db;
    }
  }
  OMEGA_STAMP(9);
}

}  // namespace omega
