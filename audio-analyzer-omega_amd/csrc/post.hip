// App spectrum post-processing after the path: what
// omega4_main.ProfessionalLiveAudioAnalyzer does to the combined spectrum of every frame
//   process_multi_resolution_fft  omega4_main.py:748-752  equal-loudness curve by position, bass boost
//   update_content_type           :805-840   bass / vocal / high energy ratios -> content type
//   process_audio_spectrum        :991-997   98th-percentile normalisation (x 0.8)
//   apply_frequency_compensation  :855-926   content-dependent per-bin factors, vocal suppression
//                                 :1004-1005 optional max normalisation
//                                 :1011-1036 band means, sqrt, clamp to [0, 1]
//                                 :1041-1056 frequency-dependent band EMA across frames
// in float32 as numpy runs them (in-place multiplies by weak Python scalars; the percentile's virtual
// index and gamma in float32; np.mean as numpy's float32 pairwise sum, divided in float64 by the
// np.intp count and rounded to float32).
//
// Bit-exactness needs every float32 operation rounded on its own: floating-point contraction is off
// for this file, and the arithmetic is written with plain operators -- HIP's __fmul_rn / __fsub_rn
// come from the device library with contraction allowed, and the backend still fused the
// percentile's lerp into an FMA (1 ulp off the reference value on the last golden frame, then every
// bin of that frame).
//   post_frame_kernel: one 256-thread workgroup per frame (independent frames).
//   post_ema_kernel + post_ema_fix_kernel: the band EMA in numpy's dtypes, warmed-up chunks checked
//   and, where needed, re-run against the sequential recurrence.
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "fft.hpp"
#include "numpy_emul.hpp"
#include "params.hpp"

#pragma clang fp contract(off)

namespace omega {

namespace {

constexpr int kPostThreads = 256;

template <class T, class Op>
__device__ __forceinline__ T block_reduce(T v, T* red, int t, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  T r = red[0];
#pragma unroll
  for (int w = 1; w < kPostThreads / 64; ++w) r = op(r, red[w]);
  return r;
}

}  // namespace

// order-preserving unsigned key of a float (-0 and +0 one key: numpy's sort holds them equal)
__device__ __forceinline__ unsigned order_key(float v) {
  const unsigned u = __float_as_uint(v == 0.f ? 0.f : v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// The value of sorted rank r of s[0..T) (no NaN): radix select over the order keys, 8 bits a round --
// a histogram of the candidates' next digit (LDS atomics), the digit whose cumulative count passes r,
// then the candidates narrowed to that digit. T / 256 elements per thread per round instead of the
// T^2 / 256 comparisons of rank counting.
__device__ float select_rank(const float* s, int T, int r, int t, unsigned (*hist)[256], unsigned (*sel)[8]) {
  // histograms and selection words double-buffered by round parity: each round clears the next
  // round's histogram while it scans its own, so a round needs three barriers
  unsigned prefix = 0, mask = 0;
  hist[0][t] = 0;
  __syncthreads();
  for (int round = 0, shift = 24; shift >= 0; ++round, shift -= 8) {
    unsigned* h = hist[round & 1];
    unsigned* sl = sel[round & 1];
    // the top byte (sign and exponent) clusters in a few digits: there lanes with the same digit add
    // once, by their first lane, instead of serialising on one LDS address; the later digits spread
    // out and take plain atomics
    for (int i0 = 0; i0 < T; i0 += kPostThreads) {
      const int i = i0 + t;
      unsigned d = 0;
      bool want = false;
      if (i < T) {
        const unsigned k = order_key(s[i]);
        want = (k & mask) == prefix;
        d = (k >> shift) & 255u;
      }
      if (shift != 24) {
        if (want) atomicAdd(&h[d], 1u);
        continue;
      }
      unsigned long long act = __ballot(want);
      while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const unsigned ld = __shfl(d, leader, 64);
        const unsigned long long peers = __ballot(want && d == ld);
        if ((t & 63) == leader) atomicAdd(&h[ld], (unsigned)__popcll(peers));
        if (d == ld) want = false;
        act &= ~peers;
      }
    }
    __syncthreads();
    // inclusive scan of the 256 counts: thread t owns digit t
    const unsigned c = h[t];
    unsigned inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = __shfl_up(inc, o, 64);
      if ((t & 63) >= o) inc += u;
    }
    if ((t & 63) == 63) sl[2 + (t >> 6)] = inc;
    hist[(round + 1) & 1][t] = 0;
    __syncthreads();
    for (int w = 0; w < (t >> 6); ++w) inc += sl[2 + w];
    const unsigned exc = inc - c;
    if (c > 0 && exc <= (unsigned)r && (unsigned)r < inc) {
      sl[0] = (unsigned)t;
      sl[1] = (unsigned)r - exc;
    }
    __syncthreads();
    prefix |= sl[0] << shift;
    mask |= 255u << shift;
    r = (int)sl[1];
  }
  const unsigned u = (prefix & 0x80000000u) ? (prefix & 0x7FFFFFFFu) : ~prefix;
  return __uint_as_float(u);
}

// The percentile of a frame of at most 512 bins whose ranks lie in its top 16 (the 98th percentile
// up to 512 bins), by bitonic folds over the order keys: each wave sorts its 128 keys as 8 runs of 16
// lanes (two keys per lane: s[128 w + l] ascending, s[128 w + 64 + l] descending), keeps the larger key
// of each pair (a bitonic run holding the top 16 of the two), and folds the runs by lane xor 16 and 32
// the same way; every wave then folds the four waves' top-16 runs into the frame's top 16 in order --
// any key of the frame's top 16 is in its own wave's top 16. No LDS atomics and one barrier instead
// of the radix select's twelve and the p_hi pass's four.
template <int M>
__device__ __forceinline__ unsigned lane_xor(unsigned v) {  // lane l reads lane l ^ M
  if constexpr (M == 1)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm 1032
  else if constexpr (M == 2)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm 2301
  else if constexpr (M == 8)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror 8
  else if constexpr (M == 32)
    return (unsigned)__shfl_xor((int)v, 32, 64);
  else
    return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (M << 10));  // bitmask mode, xor M
}
// compare-exchange with lane l ^ M: the lower lane keeps the smaller key when ascending
template <int M>
__device__ __forceinline__ unsigned cas_lane(unsigned x, bool asc) {
  const unsigned y = lane_xor<M>(x);
  return (((threadIdx.x & M) == 0) == asc) ? min(x, y) : max(x, y);
}
// a bitonic run of 16 lanes sorted (ascending where up)
__device__ __forceinline__ unsigned bitonic16_merge(unsigned x, bool up) {
  x = cas_lane<8>(x, up);
  x = cas_lane<4>(x, up);
  x = cas_lane<2>(x, up);
  return cas_lane<1>(x, up);
}
// any run of 16 lanes sorted: the 2-, 4- and 8-lane stages alternate by lane bit 2, 4, 8 (flipped for
// a descending run), then the run's merge
__device__ __forceinline__ unsigned bitonic16_sort(unsigned x, bool up) {
  const int l = threadIdx.x & 63;
  bool a = ((l & 2) == 0) == up;
  x = cas_lane<1>(x, a);
  a = ((l & 4) == 0) == up;
  x = cas_lane<2>(x, a);
  x = cas_lane<1>(x, a);
  a = ((l & 8) == 0) == up;
  x = cas_lane<4>(x, a);
  x = cas_lane<2>(x, a);
  x = cas_lane<1>(x, a);
  return bitonic16_merge(x, up);
}
// the wave's top 16 of s[128 w .. 128 w + 128) (keys past T are 0, below every non-NaN key) ascending
// into top[0 .. 16)
__device__ __forceinline__ void wave_top16(const float* s, int T, int w, unsigned* top) {
  const int l = threadIdx.x & 63, i = 128 * w + l;
  unsigned x0 = i < T ? order_key(s[i]) : 0u, x1 = i + 64 < T ? order_key(s[i + 64]) : 0u;
  x0 = bitonic16_sort(x0, true);
  x1 = bitonic16_sort(x1, false);
  unsigned y = max(x0, x1);  // 4 bitonic runs, each the top 16 of its two
  y = bitonic16_merge(y, (l & 16) == 0);
  y = max(y, lane_xor<16>(y));
  y = bitonic16_merge(y, (l & 32) == 0);
  y = max(y, lane_xor<32>(y));
  y = bitonic16_merge(y, true);
  if (l < 16) top[l] = y;
}
// the four waves' top-16 runs (top[0 .. 64)) folded: lane l returns the frame's key of rank
// T - 16 + l % 16 (runs 1 and 3 read reversed, so each pair folds into a bitonic run)
__device__ __forceinline__ unsigned merge_top16(const unsigned* top) {
  const int l = threadIdx.x & 63;
  unsigned y = top[(l & 16) ? (l | 15) - (l & 15) : l];
  y = max(y, lane_xor<16>(y));
  y = bitonic16_merge(y, (l & 32) == 0);
  y = max(y, lane_xor<32>(y));
  return bitonic16_merge(y, true);
}
__device__ __forceinline__ float unkey(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__global__ __launch_bounds__(kPostThreads) void post_frame_kernel(PostParams p) {
  __shared__ float s[kPostMaxBins];
  __shared__ unsigned hist[2][256];
  __shared__ unsigned sel[2][8];
  __shared__ float redf[kPostThreads / 64];
  const int t = threadIdx.x, T = p.T;
  const int64_t f = blockIdx.x;
  const float* in = p.in + f * p.stride;
  OMEGA_STAMP(0);
  // 1) equal-loudness curve (float64 product rounded into the float32 array) and bass boost
  for (int i = t; i < T; i += kPostThreads) {
    float v = in[i];
    if (p.flags & 1) {
      v = (float)((double)v * p.curve[i]);
      if (p.bass[i]) v = v * p.bass_boost;
    }
    s[i] = v;
  }
  __syncthreads();
  OMEGA_STAMP(1);
  // 2) content type from the range means (omega4_main.py:805-840; voice detection is not on the path):
  // four np.mean calls, one wave each (wave w: range w), numpy's pairwise sum restated lane-parallel
  // (numpy_emul.hpp: the leaf accumulators on 8 lanes each, the leaf sums combined in numpy's order)
  __shared__ float means[4];
  __shared__ float leaves[4][64];
  __shared__ int anynan;
  if (t == 0) anynan = 0;
  const int w = t >> 6;
  int m_lo = 0, m_n = 0;
  bool m_on = false;  // (an empty range gives numpy's NaN mean: 0 / 0)
  if (w == 0 && p.be < T) m_on = true, m_n = p.be;
  if (w == 1 && p.ve < T) m_on = true, m_lo = p.vs, m_n = p.ve - p.vs;
  if (w == 2 && p.hs < T) m_on = true, m_lo = p.hs, m_n = T - p.hs;
  if (w == 3) m_on = true, m_n = T;
  if (m_on) np_leaf_sums_tab(s + m_lo, p.leaf_tab + 32 * __builtin_amdgcn_readfirstlane(w), leaves[w]);
  OMEGA_STAMP(6);
  __shared__ unsigned top[4 * 16];
  const bool top_sel = T <= 512 && T - 1 - p.p_lo <= 15;
  if (top_sel) wave_top16(s, T, w, top + 16 * w);  // (published by the barriers below)
  OMEGA_STAMP(7);
  auto fmx = [](float a, float b) { return fmaxf(a, b); };
  float mx = -INFINITY;
  bool nan_here = false;
  for (int i = t; i < T; i += kPostThreads) {
    mx = fmaxf(mx, s[i]);
    nan_here |= isnan(s[i]);
  }
  __syncthreads();  // anynan initialised
  if (nan_here) anynan = 1;
  mx = block_reduce(mx, redf, t, fmx);  // (its barriers publish the leaf sums and anynan)
  if ((t & 63) == 0) {
    float m = 0.f;
    if (m_on) {
      int idx = 0;
      m = (float)((double)np_leaf_combine<6>(m_n, leaves[w], idx) / (double)m_n);
    }
    means[w] = m;
  }
  __syncthreads();
  const bool has_nan = anynan != 0;
  OMEGA_STAMP(2);
  const float eb = means[0], ev = means[1], eh = means[2], et = means[3];
  int content = 0;  // 0 instrumental, 1 vocal, 2 bass-heavy
  if (et > 0.f) {  // (NaN means fail every comparison, as in numpy)
    const float br = eb / et, vr = ev / et;
    if (br > 0.6f)
      content = 2;
    else if ((vr > 0.4f && br < 0.4f) || (vr > 0.3f && eh < ev * 0.5f))
      content = 1;
  }
  // 3) 98th percentile (numpy 'linear', float32): the values of sorted ranks p_lo and p_hi
  // np.max and np.percentile propagate NaN: `nan > 0` is false, no normalisation
  if (mx > 0.f && !has_nan) {
    float a, b;
    if (top_sel) {
      const unsigned x = merge_top16(top);
      a = unkey(__shfl(x, 16 - T + p.p_lo, 64));
      b = unkey(__shfl(x, 16 - T + p.p_hi, 64));
    } else {
      a = select_rank(s, T, p.p_lo, t, hist, sel);
      // rank p_hi (= p_lo or p_lo + 1): v_lo again while rank p_hi still holds a copy of it, else the
      // smallest value above it
      const unsigned klo = order_key(a);
      int le = 0;
      float above = INFINITY;
      for (int i = t; i < T; i += kPostThreads) {
        const float v = s[i];
        if (order_key(v) <= klo)
          ++le;
        else
          above = fminf(above, v);
      }
      le = block_reduce(le, reinterpret_cast<int*>(hist), t, [](int x, int y) { return x + y; });
      above = block_reduce(above, redf, t, [](float x, float y) { return fminf(x, y); });
      b = p.p_hi < le ? a : above;
    }
    const float d = b - a;
    // numpy _lerp, no contraction
    const float ref = p.p_g >= 0.5f ? b - d * (1.0f - p.p_g) : a + d * p.p_g;
    if (ref > 0.f)
      for (int i = t; i < T; i += kPostThreads) s[i] = s[i] / ref * 0.8f;
  }
  OMEGA_STAMP(3);
  // 4) frequency compensation (factors by position) and 5) optional max normalisation
  const float* comp = p.comp[content == 1 ? 1 : 0];
  if (p.flags & 2)
    for (int i = t; i < T; i += kPostThreads) s[i] = s[i] * comp[i] * p.vsup[i];
  __syncthreads();
  if (p.flags & 4) {
    float m = -INFINITY;
    for (int i = t; i < T; i += kPostThreads) m = fmaxf(m, s[i]);
    m = block_reduce(m, redf, t, fmx);
    if (m > 0.f && !has_nan)
      for (int i = t; i < T; i += kPostThreads) s[i] = s[i] / m;
    __syncthreads();
  }
  OMEGA_STAMP(4);
  for (int i = t; i < T; i += kPostThreads) p.spec_out[f * T + i] = s[i];
  // 6) band means -> sqrt -> clamp (before the EMA). max(0, min(1, v)) returns the Python int 1 when
  // sqrt(v) >= 1: the frame's band list then holds an int and np.array makes it float64 (:1034, :1037)
  __shared__ int clamp_any;
  if (t == 0) clamp_any = 0;
  __syncthreads();
  for (int b = t; b < p.nb; b += kPostThreads) {
    const int lo = p.bs[b], hi = p.bend[b];
    float v;
    if (hi > lo) {
      v = np_mean_f32(s + lo, hi - lo);
    } else {
      v = s[lo];
    }
    if (v > 0.f) {
      v = np_sqrt_f32(v);
      if (!(v < 1.0f)) {
        v = 1.0f;
        clamp_any = 1;
      }
    }
    p.band_raw[f * p.nb + b] = v;
  }
  __syncthreads();
  if (t == 0 && p.nb > 0) p.frame64[f] = clamp_any;
  if (t == 0 && p.content_out) p.content_out[f] = content;
  OMEGA_STAMP(5);
}

// The band EMA (omega4_main.py:1041-1056) over band_raw in frame order into band_out, with numpy's
// types: the frame's band array is float32, or float64 when a band clamped to the int 1 (frame64);
// prev_band_values keeps the previous array's dtype. Per band and frame, with P the previous value and
// x this frame's raw value:
//   a = P * f          in the previous array's dtype (f a weak Python float: float32(f) on float32)
//   b = x * (1 - f)    in this array's dtype
//   v = a + b          float64 if either is, stored into this frame's array (rounded to float32 there)
// Every operation is rounded on its own (contraction off), so the device repeats numpy's results bit
// for bit, denormals included (a decaying band sticks at the smallest denormal as it does on the CPU).
// Branch-free: both products of each term, selected; the all-float32 case float32(a32 + b32) equals
// float32(float64(a32) + float64(b32)) (float64 carries more than 2 x 24 + 2 bits, so rounding the
// float64 sum again to float32 is innocuous), so one float64 add serves all four dtype combinations.
struct EmaState {
  double v;
  bool f64;
};
__device__ __forceinline__ double ema_step(const EmaState& s, float x, bool x64, const EmaCoef& k) {
  const double a64 = s.v * k.f;
  const double a32 = (double)((float)s.v * k.f32);
  const double b64 = (double)x * k.g;
  const double b32 = (double)(x * k.g32);
  const double v = (s.f64 ? a64 : a32) + (x64 ? b64 : b32);
  return x64 ? v : (double)(float)v;
}

// One thread per (band, chunk of kEmaChunk frames). The first chunks (up to frame kEmaWarm) start at
// the stream's state; a later chunk starts kEmaWarm frames early as at a stream start (no previous
// value) and runs the same recurrence up to its own frames, recording its value at the frame before its
// own (ema_pre). Where the warm-up's start has faded out of every rounding (the usual case) that value
// equals the chunk before's stored one, and then (same operations on the same values from there on)
// the chunk holds the sequential values; post_ema_fix_kernel re-runs the chunks where it differs. Loads
// go in blocks of kEmaBlock frames, the next block's in flight during this block's recurrence; a block
// whose frames all share the state's dtype runs the plain float64 or float32 recurrence (the frames'
// dtype flags are the same on every lane: a uniform branch).
constexpr int kEmaBlock = 32;
static_assert(kEmaBlock <= kEmaSpareRows, "the spare rows cover a block");
constexpr int kEmaChunk = 64;
constexpr int kEmaWarm = 256;
// Grid: 8 x nch x ceil(band groups / 8) workgroups, workgroup w on XCD w % 8 (the hardware's
// placement): band group g = w % 8 + 8 (w / 8 / nch), chunk w / 8 % nch -- every chunk of a band
// group runs on one XCD, so the rows the chunks' warm-ups re-read (each raw band row is read by
// 1 + kEmaWarm / kEmaChunk chunks) come from that XCD's L2 instead of memory.
__device__ __forceinline__ bool ema_block(const PostParams& p, int& g, int64_t& ch) {
  const int64_t nch = (p.n + kEmaChunk - 1) / kEmaChunk;
  const int w = blockIdx.x, slot = w >> 3;
  g = (w & 7) + 8 * (int)(slot / nch);
  ch = slot % nch;
  return g < (p.nb + 63) / 64;
}

__global__ __launch_bounds__(64) void post_ema_kernel(PostParams p) {
  int g;
  int64_t ch;
  if (!ema_block(p, g, ch)) return;
  const int64_t c0 = ch * kEmaChunk;
  if (c0 >= p.n) return;
  // every lane stays (its flag load serves the block's dtype bits); lanes past the last band compute
  // the last band's values and store nothing
  const int bl = g * 64 + threadIdx.x;
  const bool live = bl < p.nb;
  const int b = live ? bl : p.nb - 1;
  const EmaCoef k = p.sf[b];
  const bool smooth = (p.flags & 8) != 0;
  const int64_t c1 = c0 + kEmaChunk < p.n ? c0 + kEmaChunk : p.n;
  const int64_t s0 = c0 == 0 ? 0 : (c0 > kEmaWarm ? c0 - kEmaWarm : 0);
  const bool exact_start = c0 == 0 || s0 == 0;
  const bool had = exact_start && p.has_prev[0] != 0;
  EmaState st{had ? p.prev[b] : 0.0, had && p.has_prev[1] != 0};
  bool use = smooth && had;  // this frame takes the EMA (no previous value: the raw value)
  // the row stride in a VGPR (opaque): the per-frame offsets are then vector arithmetic, instead of
  // 32 + 32 uniform 64-bit offsets the compiler would hold in (spilled) SGPRs
  int nb = p.nb;
  asm volatile("" : "+v"(nb));
  // blocks of kEmaBlock frames from s0: c0 - s0 is a multiple of the block (kEmaWarm and kEmaChunk
  // are), so a block is all warm-up or all output. Loads are never guarded: band_raw and frame64 have
  // kEmaBlock spare rows past the last frame (values never used); only the stream's last partial
  // block guards its stores. A block's dtype flags come as one load per lane (lane l: frame f0 + l %
  // kEmaBlock) and a ballot: bit i of `dm` = frame f0 + i holds a float64 array (uniform).
  float nx[kEmaBlock];
  int nd;
  auto load = [&](int64_t g0) {
    const float* c = p.band_raw + g0 * nb + b;
#pragma unroll
    for (int i = 0; i < kEmaBlock; ++i) {
      nx[i] = *c;
      c += nb;
    }
    nd = p.frame64[g0 + (threadIdx.x & (kEmaBlock - 1))];
  };
  load(s0);
  for (int64_t f0 = s0; f0 < c1; f0 += kEmaBlock) {
    float x[kEmaBlock];
#pragma unroll
    for (int i = 0; i < kEmaBlock; ++i) x[i] = nx[i];
    const unsigned dm = (unsigned)__ballot(nd != 0);
    if (f0 + kEmaBlock < c1) load(f0 + kEmaBlock);
    const int sf64 = __builtin_amdgcn_readfirstlane((int)st.f64);
    const int nf = c1 - f0 < kEmaBlock ? (int)(c1 - f0) : kEmaBlock;
    double v[kEmaBlock];
    if (use && dm == 0xFFFFFFFFu && sf64) {  // float64 arrays throughout: a = P f, b = x (1 - f) in float64
      double w = st.v;
#pragma unroll
      for (int i = 0; i < kEmaBlock; ++i) {
        w = w * k.f + (double)x[i] * k.g;
        v[i] = w;
      }
      st = EmaState{w, true};
    } else if (use && dm == 0u && !sf64) {  // float32 arrays throughout
      float w = (float)st.v;
#pragma unroll
      for (int i = 0; i < kEmaBlock; ++i) {
        w = w * k.f32 + x[i] * k.g32;
        v[i] = (double)w;
      }
      st = EmaState{(double)w, false};
    } else {
#pragma unroll
      for (int i = 0; i < kEmaBlock; ++i) {
        const bool d = (dm >> i) & 1u;
        const double e = ema_step(st, x[i], d, k);
        v[i] = use ? e : (double)x[i];  // (a select: the step always runs)
        st = EmaState{v[i], d};         // (past the stream's last frame: never stored)
        use = smooth;
      }
    }
    if (!live) continue;
    if (f0 >= c0) {  // this chunk's frames (the warm-up frames belong to the chunks before)
      double* o = p.band_out + f0 * nb + b;
      if (nf == kEmaBlock) {
#pragma unroll
        for (int i = 0; i < kEmaBlock; ++i) o[i * (int64_t)nb] = v[i];
      } else {  // (unrolled with a guard: a dynamic index would put v in scratch memory)
#pragma unroll
        for (int i = 0; i < kEmaBlock; ++i)
          if (i < nf) o[i * (int64_t)nb] = v[i];
      }
      if (f0 + kEmaBlock >= c1) {  // the chunk's last value (a select chain: v stays in registers)
        double last = v[0];
#pragma unroll
        for (int i = 1; i < kEmaBlock; ++i) last = i < nf ? v[i] : last;
        p.ema_end[ch * (int64_t)p.nb + b] = last;
      }
    } else if (f0 + kEmaBlock == c0) {  // the warm-up's value at the frame before this chunk
      p.ema_pre[ch * (int64_t)p.nb + b] = v[kEmaBlock - 1];
    }
  }
}

// One thread per band, after post_ema_kernel. By induction over the chunks: when chunk c's warm-up
// value at frame c0 - 1 (ema_pre) equals the (already true) value there (ema_end of chunk c - 1),
// chunk c holds the sequential values; otherwise it is re-run from that true value until a recomputed
// value equals the stored one (from there on the stored values are the recurrence's again: usually a
// few frames, as the two runs differ by an ulp that the decay drops). A re-run that does not meet the
// stored values by the chunk's end rewrote that end, so the next chunk is checked against the new
// value. Four threads per band compare the boundaries of 64 chunks at a time (16 each, their ema_pre /
// ema_end loads issued together), then the first re-runs the flagged chunks in order (rare; kFixRun frames loaded at a
// time) and writes the stream state for the next call.
constexpr int kFixRun = 8;

// re-run chunk frames [f0, f1] from the true value tv (dtype d64) at f0 - 1 until a recomputed value
// equals the stored one; returns whether it met them (else *last = the rewritten value at f1)
__device__ __forceinline__ bool ema_rerun(const PostParams& p, int b, int64_t f0, int64_t f1, double tv, bool d64,
                                       const EmaCoef& k, double* last) {
  const int64_t nb = p.nb;
  EmaState st{tv, d64};
  for (int64_t f = f0; f <= f1; f += kFixRun) {
    float xr[kFixRun];
    int dr[kFixRun];
    double vr[kFixRun];
#pragma unroll
    for (int i = 0; i < kFixRun; ++i) {
      const int64_t g = f + i <= f1 ? f + i : f1;
      xr[i] = p.band_raw[g * nb + b];
      dr[i] = p.frame64[g];
      vr[i] = p.band_out[g * nb + b];
    }
#pragma unroll
    for (int i = 0; i < kFixRun; ++i) {
      if (f + i > f1) break;
      const bool x64 = dr[i] != 0;
      const double w = ema_step(st, xr[i], x64, k);
      if (__double_as_longlong(w) == __double_as_longlong(vr[i])) return true;  // the stored run continues
      p.band_out[(f + i) * nb + b] = w;
      st = EmaState{w, x64};
    }
  }
  *last = st.v;
  return false;
}

__global__ __launch_bounds__(256) void post_ema_fix_kernel(PostParams p) {
  // four waves per 64 bands: each loads and compares 16 of a group's 64 chunk boundaries; wave 0 then
  // re-runs the flagged chunks and writes the state
  __shared__ unsigned long long part_mm[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int bl = blockIdx.x * 64 + lane;
  const bool live = bl < p.nb;
  const int b = live ? bl : p.nb - 1;
  const EmaCoef k = p.sf[b];
  const bool smooth = (p.flags & 8) != 0;
  const int64_t n = p.n, nb = p.nb;
  const int64_t nch = (n + kEmaChunk - 1) / kEmaChunk;
  OMEGA_STAMP(10);
  int reruns = 0;
  if (smooth) {
    bool dirty = false;  // the chunk before was re-run without meeting its stored values; its true
    double carry = 0.0;  // last value is `carry`
    // chunks whose warm-up starts at frame 0 continue the stream exactly: the checks start after them
    for (int64_t g0 = kEmaWarm / kEmaChunk + 1; g0 < nch; g0 += 64) {
      const int gn = nch - g0 < 64 ? (int)(nch - g0) : 64;
      // bit j: chunk g0 + j's warm-up value at its boundary differs from the value there (each wave's
      // 32 loads issued together)
      {
        unsigned long long part = 0;
        long long pre[16], end[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int j = 16 * q + i;
          const int64_t chj = g0 + j < nch ? g0 + j : nch - 1;
          pre[i] = __double_as_longlong(p.ema_pre[chj * nb + b]);
          end[i] = __double_as_longlong(p.ema_end[(chj - 1) * nb + b]);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (16 * q + i < gn && pre[i] != end[i]) part |= 1ull << (16 * q + i);
        part_mm[q][lane] = live ? part : 0ull;  // (lanes past the last band re-run nothing)
      }
      __syncthreads();
      unsigned long long mm = part_mm[0][lane] | part_mm[1][lane] | part_mm[2][lane] | part_mm[3][lane];
      __syncthreads();  // (the next group's masks overwrite these)
      if (q != 0) continue;
      OMEGA_STAMP(11 + g0 / 64);
      int c = -1;  // chunk g0 + c was the last one handled
      while (true) {
        double tv;
        if (!dirty) {
          if (!mm) break;
          c = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          tv = p.ema_end[(g0 + c - 1) * nb + b];
        } else {
          if (++c >= gn) break;  // (the carry reaches the next group's first chunk)
          mm &= ~(1ull << c);
          if (__double_as_longlong(p.ema_pre[(g0 + c) * nb + b]) == __double_as_longlong(carry)) {
            dirty = false;
            continue;
          }
          tv = carry;
        }
        ++reruns;
        const int64_t f0 = (g0 + c) * kEmaChunk;
        const int64_t f1 = f0 + kEmaChunk - 1 < n - 1 ? f0 + kEmaChunk - 1 : n - 1;
        dirty = !ema_rerun(p, b, f0, f1, tv, p.frame64[f0 - 1] != 0, k, &carry);
      }
    }
  }
  OMEGA_STAMP(20);
  OMEGA_STAMP_AT(21, (unsigned long long)__popcll(__ballot(reruns >= 1)));
  OMEGA_STAMP_AT(22, (unsigned long long)__popcll(__ballot(reruns >= 2)));
  OMEGA_STAMP_AT(23, (unsigned long long)__popcll(__ballot(reruns >= 4)));
  (void)reruns;
  if (q != 0 || !live) return;
  p.prev_out[b] = p.band_out[(n - 1) * nb + b];
  if (b == 0) {
    p.has_prev_out[0] = 1;
    p.has_prev_out[1] = p.frame64[n - 1] != 0 ? 1 : 0;
  }
}

OMEGA_STAMPS_GETTER(omega_debug_post_stamps)

hipError_t launch_post(const PostParams& p, hipStream_t s) {
  if (p.T < 1 || p.T > kPostMaxBins || p.nb < 0 || p.nb > kPostMaxBands) return hipErrorInvalidValue;
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(post_frame_kernel, dim3((unsigned)p.n), dim3(kPostThreads), 0, s, p);
  if (p.nb > 0) {
    const int64_t nch = (p.n + kEmaChunk - 1) / kEmaChunk, ngrp = ((p.nb + 63) / 64 + 7) / 8;
    hipLaunchKernelGGL(post_ema_kernel, dim3((unsigned)(8 * nch * ngrp)), dim3(64), 0, s, p);
    hipLaunchKernelGGL(post_ema_fix_kernel, dim3((p.nb + 63) / 64), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace omega
