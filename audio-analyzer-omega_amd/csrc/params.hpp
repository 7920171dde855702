// Kernel parameter blocks shared by the host launcher (capi.cpp) and the device code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace omega {

constexpr int kMaxRes = 4;
constexpr int kMaxLog2 = 15;  // twiddle tables for sizes 2^1 .. 2^14 (+1 spare)

// One resolution of the multi-resolution FFT (FFTConfig, multi_resolution_fft.py:26-44).
// One combine entry. tm = t | op << 24 with op 0: store, 1: add (a later owner of t), 2: store 0
// (no owner). Entries of a resolution are contiguous; owners of one target run in resolution order.
struct alignas(16) CombEnt {
  int tm, j;
  float c0, c1;
};

struct ResParam {
  int n;                 // real FFT size N_r
  int offset;            // W - N_r: the resolution reads the last N_r samples of the frame
  const float* win;      // [N_r] window (np.blackman(N).astype(f32))
  const float* wgt;      // [N_r/2+1] psychoacoustic weights (ones if apply_weighting is off)
  float* mag_out;        // [n_cf, N_r/2+1] or nullptr
  int ent_begin, ent_end;  // this resolution's combine entries
  float cw;              // combine weight (config.weight)
  int low_band;          // the entries read only bins < 256 (the 16384-point register FFT then forms
                         // just the lowest and highest 256 frequencies: RegFFT::run_low)
  // combine without a magnitude output, when the entries read more bins than half their count: the
  // magnitudes of the pairs (k, K - k), pair_lo <= k < pair_hi, into the spectrum's slots first (one
  // untangle per pair), then the entries from them (two LDS reads each). pair_hi == 0: every entry
  // untangles the two bins it reads itself.
  int pair_lo, pair_hi;
};

struct SpectralParams {
  const float* x;
  int64_t frame_stride, chan_stride;
  int C;
  int64_t n_cf;
  int n_res;
  ResParam res[kMaxRes];
  // combine plan (multi_resolution_fft.py:353-395): entry e writes or adds
  // c0 * mag[j] + c1 * mag[j+1] to target t (c0, c1 fold the interpolation fraction, the
  // psychoacoustic weights of bins j, j+1, the resolution weight and 1 / the target's weight sum)
  const CombEnt* ent;
  int T;
  float* comb_out;    // [n_cf, T] or nullptr
  // true peak (professional_meters.py:283-299)
  float* tp_out;      // [n_cf] or nullptr
  const float2* rot;  // [W/2 + 1] exp(+2 pi i k / (4W))
  // true-peak phases y(n + P/4) computed besides the samples (P = 0): bit P set. 0xE = 4x
  // oversampling (the reference's default), 0x4 = 2x (n + 1/2 only), 0 = 1x (the samples)
  int tp_phases;
  const float2* tw[kMaxLog2];  // tw[l][m] = exp(-2 pi i m / 2^l)
  int rf_sizes;  // host-side launch choice: bit log2(N) set = resolution size N runs on the register-FFT kernel
  // batch_kernel's true-peak role: when set, the value is stored write-through and the workgroup adds 1
  // after it (the true-peak meter query on the side stream waits for the batch's count)
  unsigned* tp_done;
  // batch_kernel's true-peak role with meter pipelining: tp_out is the context's staging slot the
  // deferred meter segment reads, and the caller's buffer (when given) gets this copy
  float* tp_copy;
};

// One zero-phase biquad (filtfilt with scipy's defaults) in state-space form:
// s' = A s + B u, y = s0 + b0 u, A = [[-a1, 1], [-a2, 0]], B = [b1 - a1 b0, b2 - a2 b0].
struct BiquadTab {
  float b0, a1, a2, B0, B1;
  float zi0, zi1;      // scipy.signal.lfilter_zi
  float h0[64], h1[64];  // first row of A^n, n < L (zero-input response of a chunk)
  float pw[64][4];     // P^(l+1), P = A^L, row-major 2x2
  float g0[64], g1[64];  // A^j B, j < L: a sample's share of its (sub-)chunk's zero-state end state
};

// K-weighting LDS table per filter (float4 entries): [0, 64) the scan powers P^(l+1), [64, 96) the
// first row of A^i and A^i B, i < 32, as (h0, h1, g0, g1) -- read where used, not held in registers
constexpr int kPwl = 96;
// K-weighting workgroup: up to 32 samples per thread (M/32 threads, 64..512), the chunk length L of
// the scan tables (make_biquad_tab) follows from it.
constexpr int kw_threads(int M) { return M / 32 < 64 ? 64 : (M / 32 > 512 ? 512 : M / 32); }
constexpr int kw_chunk(int M) { return M / kw_threads(M); }

struct KWeightParams {
  const float* x;
  int64_t frame_stride, chan_stride;
  int C;
  int64_t n_cf;
  const BiquadTab* hp;     // 38 Hz Butterworth high-pass (professional_meters.py:52-54)
  const BiquadTab* shelf;  // 1500 Hz Butterworth high-pass "shelf" (:56-64)
  float* lufs_out;         // [n_cf] or nullptr
  float* weighted_out;     // [n_cf, M] or nullptr
  int mode;                // 0: K-weighting, 3: Z (no filter, no gate: professional_meters.py:228-229)
  // when set: LUFS_inst is stored write-through and each workgroup adds 1 after it (the meter prep
  // kernel on the side stream waits for the batch's count instead of a stream event)
  unsigned* kw_done;
  // batch_kernel with meter pipelining: lufs_out is the context's staging slot the meter prep and the
  // deferred segment read, and the caller's buffer (when given) gets this copy
  float* lufs_copy;
  // (meter pipelining) instead of the count: thread 0 also stores {mirror_gen, LUFS bits} as one 64-bit
  // word into lufs_mirror[cf] -- no drain, no count; the meter prep polls the words for the generation
  unsigned long long* lufs_mirror;
  unsigned mirror_gen;
};

// Meter aggregates (meters.hip): per-channel double-buffered state (in -> out) plus per-batch scratch.
// Meter aggregate capacities: frames per launch (the host splits longer batches), history length
// (>= integrated_len - 1) and the time-ordered sequence history ++ batch.
constexpr int kMeterChunk = 2048;
constexpr int kMeterHistCap = 4096;
constexpr int kMeterSeqCap = kMeterChunk + kMeterHistCap;

// A gated value outside the batch's common window core: value, absolute frame index, and the number
// of core values below it.
struct alignas(16) MeterExt {
  float v;
  uint32_t t;
  int rc;
  int pad;
};

// omega_meter_load_history: the meter state (parity cur) of a stream whose last n_l frames had the
// LUFS_inst values lufs[f * C + c] and whose last n_t of them the true peaks tp[f * C + c] (time order),
// the next frame at absolute index n_l -- what omega_meter_reset + omega_meter_update over those frames
// leave (true peaks of the older frames -100), without computing their aggregates.
struct MeterLoadParams {
  const float* lufs;  // [n_l, C]
  const float* tp;    // [n_t, C]
  int n_l, n_t, C, HL, HT;
  float gate;
  float* hist_l;      // [C, HL]
  float* hist_t;      // [C, HT]
  int* n_l_out;
  int* n_t_out;
  unsigned long long* skeys;  // [C, HL]
  int* n_s_out;
  uint32_t* t0_out;
};

struct MeterPrepParams {
  const float* lufs;    // [n_frames * C] batch instantaneous LUFS
  // when set (meter pipelining): the batch's values come from these {generation, value} words instead of
  // `lufs` after wait_ctr (KWeightParams::lufs_mirror): each is polled until it carries mirror_gen
  const unsigned long long* lufs_mirror;
  unsigned mirror_gen;
  const float* tp;      // [n_frames * C]
  int64_t n_frames;     // <= kMeterChunk per launch
  int C;
  const float* hist_l_in;  // [C, HL] last LUFS_inst values, time order
  const float* hist_t_in;  // [C, HT] last TP values
  const int* n_l_in;
  const int* n_t_in;
  const unsigned long long* skeys_in;  // [C, HL] gated keys of hist_l, sorted
  const int* n_s_in;
  const uint32_t* t0_in;  // absolute index of the batch's first frame
  float* hist_l_out;
  float* hist_t_out;
  int* n_l_out;
  int* n_t_out;
  unsigned long long* skeys_out;
  int* n_s_out;
  uint32_t* t0_out;
  int HL, HT;  // integrated_len - 1, peak_len - 1
  int mom_len, short_len, int_len, peak_len;
  float gate;
  // per-batch scratch written by meter_prep_kernel for meter_query_kernel
  float* core;      // [C, kMeterSeqCap] gated values in every window of the batch, ascending
  MeterExt* ext;    // [C, kMeterSeqCap] the other gated values of the batch's windows, ascending
  int* n_core;      // [C]
  int* n_ext;       // [C]
  int* gcount;      // [C, kMeterSeqCap + 1] gated-count prefix in time order
  double* gsum;     // [C, kMeterSeqCap + 1] gated-sum prefix in time order
  double* out;                     // [n_frames * C, 5]
  int parts;  // meter_query_kernel: bit 0 the LUFS meters (columns 0-3), bit 1 the true-peak meter (4)
  // meter_prep_kernel: when set, wait until (int)(*wait_ctr - wait_target) >= 0 before reading `lufs`
  // (the batch kernel's K-weighting workgroups count themselves in after storing their value)
  unsigned* wait_ctr;
  unsigned wait_target;
  // meter_query_kernel: q_done set -> every workgroup adds 1 after its outputs are out (release);
  // join_ctr set -> workgroup (0, 0) does not finish before (int)(*join_ctr - join_target) >= 0, so the
  // stream it runs on completes only after the side stream's query workgroups (no stream event)
  unsigned* q_done;
  unsigned* join_ctr;
  unsigned join_target;
  // tail layout (omega_ctx::meter_tail): meter_prep_kernel counts itself into q_done when set;
  // meter_query_kernel waits (every workgroup, bounded) until (int)(*start_ctr - start_target) >= 0
  unsigned* start_ctr;
  unsigned start_target;
  // the batch's meter segment (batch_meter_role): when seg_ctr is set every workgroup adds 1 to it
  // once its reads are done. meter_prep_kernel: before writing the per-batch scratch of its parity it
  // waits until (int)(*seg_ctr - seg_pre_target) >= 0 (the last segment that reads that scratch is
  // done), before writing the next state until (int)(*seg_ctr - seg_post_target) >= 0 (the last
  // segment that reads that state) -- with meter pipelining that segment may run in a later launch
  unsigned* seg_ctr;
  unsigned seg_pre_target, seg_post_target;
  // bounded polls: at most poll_limit iterations; on expiry the kernel stores 1 into err_word[0] (prep)
  // or err_word[1] (join) -- host-mapped memory the host checks in omega_synchronize and the next call
  // (OMEGA_EHIP instead of silently stale meters)
  int poll_limit;
  unsigned* err_word;
};

struct BandParams {
  const float* spec;
  int64_t n, spec_stride;
  int n_bins;
  int n_out;
  const int* starts;
  const int* ends;
  const float* scale;      // [n_out] per-band multiplier (MAX) or nullptr
  const float* bin_scale;  // [n_bins] per-bin multiplier (MEAN) or nullptr
  int op;                  // 0 max, 1 mean
  int n_valid;             // bands computed; the rest are 0
  float* out;              // [n, n_out]
};

struct ChromaParams {
  const float* spec;
  int64_t n;
  int n_bins;
  double df;
  const float* mat;     // [12, n_bins] projection (chromagram.py:122-146), zero outside 20..8000 Hz
  double* out;          // [n, 12] normalised smoothed chroma (before the temporal blend)
};

// combine_results_optimized over externally supplied (already weighted) magnitudes; a missing
// resolution (mag[r] == nullptr) is skipped like a key absent from the results dict.
struct CombineParams {
  const float* mag[kMaxRes];
  int nbins[kMaxRes];
  float cw[kMaxRes];
  int64_t n_cf;
  int T;
  const int* own_off;   // [T+1]
  const int* own_rj;    // (r << 24) | j
  const float* own_frac;
  float* out;           // [n_cf, T]
};

// Segments of one mrfft_multi_kernel launch: resolution res[s] owns workgroups
// [wg_begin[s], wg_begin[s+1]) (the last one up to the grid end).
struct MultiPlan {
  int n_seg;
  int res[4];
  int wg_begin[4];
};

// One launch for the per-channel-frame work of a batch of 16384-sample frames (rfkern.hip
// batch_kernel), 512-thread workgroups. Roles: 0 K-weighting + LUFS_inst, 1 true peak, 2 the
// 16384-point resolution (mr_res). Two segments of role groups, then the small resolutions:
//   [seg_begin[s], seg_begin[s + 1])  groups of 8 * n_roles[s] workgroups; workgroup b of the segment
//       runs role roles[s][(b / 8) % n_roles[s]] of channel-frame 8 (b / (8 n_roles[s])) + b % 8, so
//       the roles of a frame land on one XCD (blockIdx % 8). (The hardware places an XCD's workgroups
//       in blockIdx order round-robin over its 4 shader engines and holds the next one until its
//       engine has room, so with two roles each engine runs one role and the engines of the short
//       16384-point-resolution workgroups idle ~5 us behind the K-weighting ones: 80 % of the slot-time
//       used, tools/wgtrace.py. Role chunks of one workgroup per CU fill 90 % of it, but the shader
//       clock drops from ~2120 to ~1890 MHz and the launch takes longer: the batch runs at the chip's
//       power limit, so idle slots are not free time. DESIGN.md §8.)
//   pat: the group order of a two-role segment: 0 alternating groups (each shader engine runs one
//       role), 1 the period-8 order A B A B B A B A (seen by one XCD through blockIdx % 8, its engines
//       get the roles in turn, so an engine's short workgroups do not wait behind another's long
//       ones; the product's order, round 4: batch kernel 71.3 -> 65.9 us).
//   seg_start / multi_start / multi_n: where segment s and the small resolutions begin in the grid.
struct BatchPlan {
  int seg_begin[3];
  int n_roles[2];
  int roles[2][3];
  int mr_res;
  MultiPlan multi;
  int q_begin, q_n;
  unsigned* tail_ctr;  // (meter pipelining) the last workgroup adds 1 at its start: see capi.cpp d_tail
  int pat;
  int seg_start[2];
  int multi_start, multi_n;
};

// Fused spectrum analysis (cfg3): windowed rfft magnitude (A13) -> log-band max (A10) and raw
// chromagram (A12) of each frame, one pass over the frame.
struct SpectraParams {
  const float* x;
  int64_t n, stride;       // frames of 2K samples at x + f * stride
  const float* win;        // [2K]
  const float4* wgen;      // the window as a per-thread generator (WinGen, regfft.hpp)
  float* mag_out;          // [n, K+1] or nullptr
  // A10 (MAX op): bands [0, n_valid) of n_out, band i = max(mag[starts[i]:ends[i]]) * scale[i]
  int n_out, n_valid;
  const int* starts;
  const int* ends;
  const float* scale;
  float* bands_out;        // [n, n_out] or nullptr
  // A12: bins [c_lo, c_hi): weights of the 5 pitch classes base-2..base+2 (w4 = 5th); the bins
  // grouped by base class: cperm[cgoff[b] .. cgoff[b+1]) = bin - c_lo of the bins with base class b
  int c_lo, c_hi;
  const float4* cw4;
  const float* cw1;
  const unsigned short* cperm;
  const int* cgoff;        // [13]
  // the same bins in group order as 12-byte records {a, g, bin} for the register-FFT kernel (record j
  // read directly: no dependent permutation load): with u = c - b the fraction of the bin's pitch class
  // and s its octave-band scale, a = s exp(-2 u^2) and g = exp(4 u), so the five weights
  // s exp(-2 (u - o)^2), o = -2..2, are a g^o e^{-2 o^2} (rtol 1e-5 of the chromagram: ~3e-7 here)
  const float* crec;       // [3 * cgoff[12]]
  double* chroma_out;      // [n, 12] or nullptr (smoothed, normalised; before the temporal blend)
  const float2* tw[kMaxLog2];
};

// Drum-detection spectral features (drum.hip): 7 flux bands (kick sub / body /
// click, snare fundamental / body / snap / rattle), the snare centroid range, and one stream's state
// (previous magnitude frame, 21-deep flux histories, frames seen), double-buffered (in -> out).
constexpr int kDrumBands = 7;
constexpr int kDrumHist = 21;
constexpr int kDrumCols = 14;

// App spectrum post-processing (post.hip): per-bin tables from the host.
constexpr int kPostMaxBins = 2048;
constexpr int kEmaSpareRows = 32;  // band_raw rows past the last frame (post_ema_kernel's unguarded block loads)
constexpr int kPostMaxBands = 1024;
// band EMA factor f (omega4_main.py:1044-1054: prev * f + v * (1 - f) with a Python float f): the
// float64 forms (f, 1 - f) and the float32 forms numpy's weak-scalar promotion uses on float32 scalars
struct EmaCoef {
  double f, g;    // f, 1 - f
  float f32, g32; // float32(f), float32(1 - f)
};
struct PostParams {
  const float* in;  // [n, stride] combined spectra
  int64_t n, stride;
  int T;
  const double* curve;         // [T] equal-loudness curve by position
  const unsigned char* bass;   // [T] combine frequency < 250 Hz
  const float* comp[2];        // [T] frequency compensation: [0] instrumental / bass-heavy, [1] vocal
  const float* vsup;           // [T] vocal-suppression factor (1 outside 800-4000 Hz)
  int be, vs, ve, hs;          // content ranges [0, be), [vs, ve), [hs, T)
  const unsigned* leaf_tab;    // [4][32] numpy pairwise-sum leaves of the four ranges (capi post configure)
  int p_lo, p_hi;              // 98th percentile: sorted ranks and float32 gamma
  float p_g;
  const int* bs;               // [nb] band starts / ends
  const int* bend;
  const EmaCoef* sf;           // [nb] EMA factor f in the forms the reference's numpy arithmetic uses
  int nb;
  int flags;                   // OMEGA_POST_* bits
  float bass_boost;
  float* spec_out;             // [n, T]
  double* band_out;            // [n, nb] (float32 values, or float64 on frames whose list held the int 1)
  float* band_raw;             // [n, nb] scratch: the clamped band values before the EMA
  int* frame64;                // [n] scratch: 1 where a band clamped to the Python int 1 (float64 array)
  double* ema_pre;             // [n / 64 chunks, nb] scratch: each EMA chunk's warm-up value at the frame
                               // before it (post.hip post_ema_kernel)
  double* ema_end;             // [n / 64 chunks, nb] scratch: each chunk's value at its last frame
  int* content_out;            // [n]
  // EMA state {value, float64 dtype, present} in (double-buffered: the kernels read one, write the
  // other)
  double* prev;                // [nb]
  int* has_prev;               // [2]: present, float64 dtype
  double* prev_out;            // [nb] EMA state out
  int* has_prev_out;
};

struct DrumParams {
  const float* mag;
  int64_t n, stride;
  int n_bins;
  int bs[kDrumBands], be[kDrumBands];  // band bins [bs, be)
  int cs, ce;                          // centroid bins
  double fstep;                        // rfftfreq(2 n_bins - 1) spacing: fs / (2 n_bins - 1)
  float mult[kDrumBands];              // float32(sensitivity * multiplier); 0: no threshold
  const float* prev_in;
  float* prev_out;                     // [n_bins]
  const float* hist_in;
  float* hist_out;                     // [kDrumBands][kDrumHist], oldest first
  const int* len_in;
  int* len_out;                        // [kDrumBands]
  const long long* pos_in;
  long long* pos_out;                  // frames of the stream seen before / after this call
  float* flux;                         // [n, kDrumBands] scratch
  double* out;                         // [n, kDrumCols] (oracle DRUM_COLUMNS order)
};

struct RfftParams {
  const float* x;
  int64_t n;
  const float* win;
  float* mag;    // [n, m/2+1] or nullptr
  float* cplx;   // [n, m/2+1, 2] or nullptr
  const float2* tw[kMaxLog2];
};

// VU meter ballistics (vu.hip; vu_meters.py:55-99) over n consecutive update calls of chunk samples
// per channel: update u of channel c at x + u * frame_stride + c * channel_stride (float32 or float64)
struct VuParams {
  const void* x;
  int f64;
  int64_t n;
  int chunk;
  int64_t frame_stride, channel_stride;
  int C;
  const double* dt;        // [n] seconds since the previous update
  const double* hist_in;   // [C, Wv] the last hist_n samples before this batch, oldest first
  double* hist_out;        // [C, Wv]
  int64_t hist_n;
  int64_t Wv;              // int(0.3 fs): the deque length
  double* ms;              // [n, C] scratch: window mean squares
  const double* st_in;     // [C, 3] display, peak, peak_time
  double* st_out;
  double* out;             // [n, C, 3] vu_db (+18 offset applied), display, peak_db
};

// TransientAnalyzer.analyze_transients (transient.hip; transient.py:19-108), one frame per workgroup
constexpr int kTransientCols = 6;  // detected, attack_time_ms, punch, envelope_peak, envelope_rms, envelope_mean
constexpr int kTrMaxStages = 32;
struct TransientParams {
  const void* x;
  int f64;
  int64_t n_frames;
  int n;                    // frame length (>= 64; powers of two up to 8192 on the packed transform)
  int64_t frame_stride;
  const double2* tw;        // [n/4] e^{-2 pi i m / (n/2)}
  const double2* tw2;       // [n/2 + 1] e^{-2 pi i q / n}
  const double* sg;         // [21, 21] Savitzky-Golay (21, 3) weights by output position in the window
  double fs;
  double* out;              // [n_frames, kTransientCols]
  // other lengths: a complex n-point mixed-radix transform (radices as anyfft.hip) with the float64
  // table e^{-2 pi i m / n}, buffers in LDS (2 n double2) or, when scratch is set, global memory
  int n_stages;
  int radix[kTrMaxStages];
  const double2* twn;       // [n] or nullptr (power-of-two path)
  double2* scratch;         // [n_frames, 2 n] or nullptr
};

// omega_weighting (weight64.hip): scipy's float64 filtfilt cascades of professional_meters.py:129-218
// for frames of any length > 9. One section: DF2T biquad (first-order sections have b2 = a2 = 0), its
// lfilter_zi and filtfilt's padlen E.
struct W64Stage {
  double b0, b1, b2, a1, a2, zi0, zi1;
  int E;
  int pad_;
};
// weighting modes (omega.h omega_weighting_mode)
enum WeightMode : int { kWeightK = 0, kWeightA = 1, kWeightC = 2, kWeightZ = 3 };
struct Weight64Params {
  const float* x;           // [n, M]
  int M;
  int mode;                 // OMEGA_WEIGHT_K / A / C / Z
  int64_t n;
  W64Stage* st;             // the mode's sections in order
  int n_st;
  double* scratch;          // [n, scratch_stride]: signal (M) + odd extension (M + 2E)
  int64_t scratch_stride;
  float* weighted_out;      // [n, M] or nullptr
  float* lufs_out;          // [n] or nullptr
};

// Frames of any length (anyfft.hip): mixed-radix Stockham transform, true peak and windowed rfft
constexpr int kAnyMaxStages = 32;
constexpr int kAnyLdsMax = 6826;  // 3 N float2 in 160 KiB of LDS; above: global scratch
struct AnyFftParams {
  const float* x;           // frame f at x + f * frame_stride
  int64_t frame_stride;
  int64_t n;
  int N;
  int n_stages;
  int radix[kAnyMaxStages];
  const float2* tw;         // [N] e^{-2 pi i m / N}
  const float2* rot;        // [3 (N / 2) + 1] e^{2 pi i m / (4N)} (true peak)
  float nyq_cos[4];         // cos(pi p / 4)
  int phases;               // true peak: bit p set for each phase p in 1..3
  float* tp_out;            // [n] dBTP
  const float* win;         // rfft: window [N] or nullptr
  float* mag;               // rfft: [n, N/2 + 1] or nullptr
  float* cplx;              // rfft: [n, N/2 + 1, 2] or nullptr
  float2* scratch;          // [n, 3N] when N > kAnyLdsMax, else nullptr (LDS)
};

}  // namespace omega
