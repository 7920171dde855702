// libomega.so host side: the C ABI declared in include/omega.h.
//
// The context precomputes (in float64, cast like the reference casts) every table the kernels read:
// windows (np.blackman/np.hanning/np.hamming), psychoacoustic weights (multi_resolution_fft.py:304-329,
// float32 compounding), the combine plan (multi_resolution_fft.py:353-395), FFT twiddles, the
// true-peak rotation table, the two K-weighting biquads in state-space form with their chunk-scan
// tables (professional_meters.py:48-72, scipy.signal.butter/lfilter_zi closed forms), and owns the
// per-channel meter state (professional_meters.py:19-25) on the device, double-buffered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/omega.h"
#include "params.hpp"

namespace omega {
hipError_t launch_spectral(int W, const SpectralParams& p, hipStream_t s);
hipError_t launch_mrfft(const SpectralParams& p, hipStream_t s);
hipError_t launch_mrfft_range(const SpectralParams& p, int r0, int r1, hipStream_t s);
hipError_t launch_mrfft_independent(const SpectralParams& p, hipStream_t s);
hipError_t launch_truepeak(int W, const SpectralParams& p, hipStream_t s);
hipError_t launch_truepeak_rf(int W, const SpectralParams& p, hipStream_t s, int extra_lds = 0);
hipError_t launch_mrfft_rf(int n, const SpectralParams& p, int r, hipStream_t s);
hipError_t launch_rfft(int m, const RfftParams& p, hipStream_t s);
hipError_t launch_kweight(int m, const KWeightParams& p, hipStream_t s);
hipError_t launch_weight64(const Weight64Params& p, hipStream_t s);
hipError_t launch_any(const AnyFftParams& p, int truepeak, hipStream_t s);
hipError_t launch_spectra(int m, const SpectraParams& p, int grid, hipStream_t s);
hipError_t launch_spectra_rf(int m, const SpectraParams& p, hipStream_t s);
hipError_t launch_meters(const MeterPrepParams& p, hipStream_t s);
hipError_t launch_meter_prep(const MeterPrepParams& p, hipStream_t s);
hipError_t launch_meter_query(const MeterPrepParams& p, hipStream_t s);
hipError_t launch_meter_load(const MeterLoadParams& p, hipStream_t s);
hipError_t launch_queue_probe(unsigned* w, unsigned target, int limit, hipStream_t side, hipStream_t main);
hipError_t launch_bands(const BandParams& p, hipStream_t s);
hipError_t launch_chroma(const float* spec, int64_t n, int n_bins, int lo, int hi, const double* mat, double* out,
                         hipStream_t s);
hipError_t launch_combine(const CombineParams& p, hipStream_t s);
hipError_t launch_drum(const DrumParams& p, hipStream_t s);
hipError_t launch_vu(const VuParams& p, hipStream_t s);
hipError_t launch_transients(const TransientParams& p, hipStream_t s);
hipError_t launch_transients_any(const TransientParams& p, hipStream_t s);
hipError_t launch_post(const PostParams& p, hipStream_t s);
hipError_t launch_batch(const SpectralParams& sp, const KWeightParams& kp, const BatchPlan& bp, const MeterPrepParams& mp,
                        int grid, hipStream_t s);
}  // namespace omega

using namespace omega;

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr int kChunkFrames = kMeterChunk;
constexpr int kBatchWaves = 8;  // waves of a batch_kernel workgroup (rfkern.hip kBatchThreads / 64)
// meter workgroups of the batch grid at most: they wait (spinning) for the meter prep kernel, which
// may be dispatched after them and needs a CU with at most one batch workgroup resident (1024 threads
// and 72.6 KiB of LDS beside one 512-thread, 71.9 KiB batch workgroup). 64 waiting workgroups hold at
// most 64 of the 512 batch slots, so at least 192 CUs keep a slot that other roles free as they
// finish. (Round 1: one meter workgroup per 8 outputs of a 4096-frame batch took every slot and waited
// until the poll bound expired.)
#ifndef OMEGA_METER_WGS
#define OMEGA_METER_WGS 64  // (measured: 16 and 32 slower, profiles/r04_ab_meter_wgs.txt)
#endif
constexpr int kMeterWgs = OMEGA_METER_WGS;


struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
};

bool is_pow2_in(int v, int lo, int hi) { return v >= lo && v <= hi && (v & (v - 1)) == 0; }

// numpy window formulas (numpy 2.x): n = arange(1-M, M, 2)
std::vector<float> make_window(int M, int kind) {
  std::vector<float> w(M);
  for (int i = 0; i < M; ++i) {
    const double n = (double)(1 - M + 2 * i);
    double v;
    switch (kind) {
      case OMEGA_WIN_BLACKMAN: v = 0.42 + 0.5 * std::cos(kPi * n / (M - 1)) + 0.08 * std::cos(2.0 * kPi * n / (M - 1)); break;
      case OMEGA_WIN_HANN: v = 0.5 + 0.5 * std::cos(kPi * n / (M - 1)); break;
      case OMEGA_WIN_HAMMING: v = 0.54 + 0.46 * std::cos(kPi * n / (M - 1)); break;
      default: v = 1.0;
    }
    if (M == 1) v = 1.0;
    w[i] = (float)v;
  }
  return w;
}

// np.fft.rfftfreq(N, 1/fs)
double rfreq(int k, int N, double fs) {
  const double d = 1.0 / fs;
  const double val = 1.0 / (N * d);
  return k * val;
}

struct BiquadCoef {
  double b[3], a[3];
};

// scipy.signal.butter(2, fc/(fs/2), 'low') and butter(1, ..., 'high' / 'low') (bilinear, prewarped);
// first-order sections as biquads with b2 = a2 = 0
BiquadCoef butter2_lowpass(double fc, double fs) {
  const double K = std::tan(kPi * fc / fs);
  const double n = 1.0 + std::sqrt(2.0) * K + K * K;
  BiquadCoef c;
  c.b[0] = K * K / n;
  c.b[1] = 2.0 * K * K / n;
  c.b[2] = K * K / n;
  c.a[0] = 1.0;
  c.a[1] = 2.0 * (K * K - 1.0) / n;
  c.a[2] = (1.0 - std::sqrt(2.0) * K + K * K) / n;
  return c;
}
BiquadCoef butter1(double fc, double fs, bool high) {
  const double K = std::tan(kPi * fc / fs);
  BiquadCoef c;
  c.b[0] = high ? 1.0 / (1.0 + K) : K / (1.0 + K);
  c.b[1] = high ? -1.0 / (1.0 + K) : K / (1.0 + K);
  c.b[2] = 0.0;
  c.a[0] = 1.0;
  c.a[1] = (K - 1.0) / (K + 1.0);
  c.a[2] = 0.0;
  return c;
}

// scipy.signal.butter(2, fc/(fs/2), 'high') (bilinear transform, prewarped)
BiquadCoef butter2_highpass(double fc, double fs) {
  const double K = std::tan(kPi * fc / fs);
  const double n = 1.0 + std::sqrt(2.0) * K + K * K;
  BiquadCoef c;
  c.b[0] = 1.0 / n;
  c.b[1] = -2.0 / n;
  c.b[2] = 1.0 / n;
  c.a[0] = 1.0;
  c.a[1] = 2.0 * (K * K - 1.0) / n;
  c.a[2] = (1.0 - std::sqrt(2.0) * K + K * K) / n;
  return c;
}

void mat2_mul(const double* A, const double* B, double* C) {
  double t[4] = {A[0] * B[0] + A[1] * B[2], A[0] * B[1] + A[1] * B[3], A[2] * B[0] + A[3] * B[2],
                 A[2] * B[1] + A[3] * B[3]};
  std::memcpy(C, t, sizeof t);
}

BiquadTab make_biquad_tab(const BiquadCoef& c, int L) {
  BiquadTab t{};
  const double b0 = c.b[0], a1 = c.a[1], a2 = c.a[2];
  const double B0 = c.b[1] - a1 * b0, B1 = c.b[2] - a2 * b0;
  t.b0 = (float)b0;
  t.a1 = (float)a1;
  t.a2 = (float)a2;
  t.B0 = (float)B0;
  t.B1 = (float)B1;
  // scipy.signal.lfilter_zi: solve (I - companion(a).T) zi = B
  const double z0 = (B0 + B1) / (1.0 + a1 + a2);
  t.zi0 = (float)z0;
  t.zi1 = (float)(B1 - a2 * z0);
  const double A[4] = {-a1, 1.0, -a2, 0.0};
  double An[4] = {1, 0, 0, 1};
  for (int n = 0; n < 64; ++n) {
    if (n < L) {
      t.h0[n] = (float)An[0];
      t.h1[n] = (float)An[1];
    }
    if (n + 1 <= L) mat2_mul(A, An, An);
  }
  // A^j B, j < L
  {
    double g[2] = {B0, B1};
    for (int j = 0; j < L && j < 64; ++j) {
      t.g0[j] = (float)g[0];
      t.g1[j] = (float)g[1];
      const double n0 = A[0] * g[0] + A[1] * g[1], n1 = A[2] * g[0] + A[3] * g[1];
      g[0] = n0;
      g[1] = n1;
    }
  }
  // An = A^L now (L <= 64)
  double P[4];
  std::memcpy(P, An, sizeof P);
  double Pk[4] = {P[0], P[1], P[2], P[3]};
  for (int l = 0; l < 64; ++l) {
    for (int q = 0; q < 4; ++q) t.pw[l][q] = (float)Pk[q];
    mat2_mul(P, Pk, Pk);
  }
  return t;
}

}  // namespace

struct omega_bands {
  omega_ctx* ctx;
  int op, n_bands, n_out, n_bins, n_valid;
  int32_t* d_starts;
  int32_t* d_ends;
  float* d_scale;
  float* d_bin_scale;
};

struct omega_ctx {
  omega_config cfg{};
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  // fork/join streams + events for the concurrent branches, and the graph cache
  hipStream_t cap = nullptr, fork[1] = {nullptr};
  std::vector<hipStream_t> spare;  // side streams found on the context stream's hardware queue (kept
                                   // alive so the next one created lands on another queue; at most
                                   // kMaxSpare, the oldest destroyed beyond that)
  unsigned* d_probe = nullptr;     // side_stream_check's two words
  unsigned probe_seq = 0;
  std::vector<hipStream_t> checked;  // streams probed against the current fork[0] (cleared when it changes)
  bool queue_shared = false;         // the last probe found no independent queue for fork[0]
  hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
  // HIP graph replay of device-memory calls: off by default -- on MI355X (ROCm 7) a replayed graph
  // put the stream layout's nodes on other queues, with ~12 us cross-queue waits and ~20 us between
  // consecutive launches (cfg2 step 149.5 us vs 128.8 us for direct launches of the same layout)
  bool use_graph = false;
  // stream layout of the per-batch work (enqueue_frames): 3 (default; 16384-sample frames, direct
  // launches) one batch_kernel launch for all per-channel-frame work, the meter prep on the side stream
  // waiting on the batch's K-weighting count (kw_done) instead of a stream event; 2 (other frame sizes,
  // graph capture, or omega_set_graphs layout bits) the full-chip kernels back to back with the meter
  // aggregates on a side stream joined by events.
  int layout = 3;
  unsigned* d_kw_done = nullptr;  // batch_kernel's K-weighting workgroups count themselves in here
  unsigned kw_issued = 0;         // K-weighting workgroups launched with the count on (wraps)
  unsigned q_issued = 0;          // LUFS-meter query workgroups launched with the count on (d_kw_done[1])
  unsigned tp_issued = 0;         // batch true-peak workgroups launched with the count on (d_kw_done[2])
  unsigned prep_issued = 0;       // meter prep workgroups launched with the count on (d_kw_done[3])
  unsigned seg_issued = 0;        // meter-segment workgroups launched (they count in at d_kw_done[4])
  unsigned lt_issued = 0;         // omega_calculate_lufs true-peak workgroups (they count in at d_kw_done[5])
  unsigned* tp_count_to = nullptr;  // set inside omega_calculate_lufs: its true peaks count in here
  bool side_meters = false;  // meter kernels enqueued on fork[0] since omega_calculate_lufs last joined it
  // seg_issued once the last meter segment that reads parity p's scratch / state has counted in: the
  // preps' targets before they overwrite them (MeterPrepParams::seg_ctr)
  unsigned seg_par[2] = {0, 0};
  // meter pipelining (omega_set_meter_pipelining): the meter segment of the last default-layout batch
  // with meters, not yet launched -- the next such batch launch runs it first in its grid, any other
  // use of the meter state (and omega_synchronize / omega_flush_meters) launches it on its own
  bool pipe = false;
  bool pend = false;
  MeterPrepParams pend_mq{};
  int pend_nq = 0, pend_par = 0;
  int stage_par = 0;  // pipelined calls alternate the staging of LUFS_inst / TP (the segment reads them later)
  // pipelined launches: the grid's last-dispatched workgroup counts in here (signal memory, so the side
  // stream's command processor can wait on it: hipStreamWaitValue32) -- the prep is dispatched only
  // once the batch has no workgroup left to place, into the slots its tail leaves idle, instead of
  // holding a CU through the batch (step 66.5-67.1 vs 67.2-67.9 us); -1: not supported, no wait
  unsigned* d_tail = nullptr;
  unsigned tail_issued = 0;
  // (meter pipelining) the K-weighting workgroups' {generation, LUFS} words, two parities of
  // kChunkFrames x C (KWeightParams::lufs_mirror)
  unsigned long long* d_mirror = nullptr;
  unsigned mirror_gen = 0;
  int tail_ok = 0;
  // device-side poll expiry flags (host-mapped: [0] meter prep, [1] join), checked by
  // check_device_err; the poll bound (OMEGA_POLL_LIMIT, a test knob)
  unsigned* h_err = nullptr;
  unsigned* d_err = nullptr;
  int poll_limit = 1 << 22;
  float* d_lufs_scr = nullptr;  // omega_calculate_lufs: instantaneous values kept on the device
  int64_t lufs_scr_cap = 0;
  bool res_independent = false;  // no combine target has several owners: resolution kernels commute
  hipEvent_t ev_kw = nullptr;
  struct GraphEntry {
    std::vector<uint64_t> key;
    hipGraph_t graph;
    hipGraphExec_t exec;
  };
  std::vector<GraphEntry> graphs;
  char err[512] = {};  // omega_last_error (a fixed buffer: reporting an error allocates nothing)
  // tables
  float2* d_tw[kMaxLog2] = {};

  float2* d_rot = nullptr;
  float* d_win[kMaxRes] = {};
  float* d_wgt[kMaxRes] = {};
  CombEnt* d_ent = nullptr;
  int ent_begin[kMaxRes] = {}, ent_end[kMaxRes] = {};
  int pair_lo[kMaxRes] = {}, pair_hi[kMaxRes] = {};  // ResParam::pair_lo / pair_hi
  int ent_jmax[kMaxRes] = {};  // the highest bin a resolution's combine entries read (j + 1)
  std::map<std::pair<int, int>, BiquadTab*> kw_tabs;  // (M, chunk) -> device {hp, shelf}
  int rf_sizes = 1 << 14;   // resolution sizes on the register-FFT kernel (bit log2 N): the 16384-point one
  std::map<std::pair<int, int>, float*> windows;  // (m, kind) -> device window
  std::map<int, float2*> rots;                     // m -> true-peak rotation table
  std::map<std::pair<int, int>, float4*> wgens;     // (m, kind) -> WinGen table
  // combine plan as per-target owner lists (CSR) for omega_combine over a subset of resolutions
  int* d_own_off = nullptr;
  int* d_own_rj = nullptr;  // (r << 24) | j
  float* d_own_frac = nullptr;
  std::map<int, std::pair<double*, std::pair<int, int>>> chroma_mats;  // n_bins -> (mat, [lo, hi))
  double chroma_df = 0.0;
  // compact chromagram tables of omega_spectra, per (n_bins, df): 5 float32 weights per bin, bins
  // grouped by base pitch class
  struct ChromaTab {
    int n_bins = 0, lo = 0, hi = 0;
    double df = 0.0;
    float4* w4 = nullptr;
    float* w1 = nullptr;
    unsigned short* perm = nullptr;
    int* goff = nullptr;
    float* rec = nullptr;
  } ctab;
  int n_cu = 0;
  // drum-feature stream state (omega_drum_features), double-buffered, for drum_bins bins per frame
  int drum_bins = 0, drum_cur = 0;
  float* d_dprev[2] = {};
  float* d_dhist[2] = {};
  int* d_dlen[2] = {};
  long long* d_dpos[2] = {};
  float* d_dflux = nullptr;
  PostParams post{};  // omega_post_configure's tables (post.n_bins = 0: not configured)
  float* d_post_raw = nullptr;  // post-processing band scratch (pre-EMA values)
  int64_t post_raw_cap = 0;
  // VU meter state (omega_vu_update), double-buffered: sample history, display / peak / hold time
  double* d_vu_hist[2] = {};
  double* d_vu_st[2] = {};
  double* d_vu_ms = nullptr;
  int64_t vu_ms_cap = 0, vu_total = 0;
  int vu_cur = 0;
  // transient-analysis tables per frame length: twiddles (float64) and the Savitzky-Golay weights
  std::map<int, std::pair<double2*, double2*>> tr_tw;
  std::map<int, std::pair<std::vector<int>, double2*>> tr_any;  // other lengths: radices, e^{-2 pi i m / n}
  double2* d_tr_scratch = nullptr;
  int64_t tr_scratch_cap = 0;
  double* d_sg = nullptr;
  int64_t dflux_cap = 0;  // (elements)
  // omega_weighting: float64 filter cascades per mode and the per-launch working buffers
  W64Stage* w64[4] = {};
  // frames of any length (anyfft.hip): per N the radices and the twiddle / rotation tables
  struct AnyPlan {
    std::vector<int> radix;
    float2* tw = nullptr;
    float2* rot = nullptr;
  };
  std::map<int, AnyPlan> any_plans;
  float2* d_any = nullptr;
  int64_t any_cap = 0;
  double* d_w64 = nullptr;
  int64_t w64_cap = 0;
  // meter state (double-buffered)
  float* d_hist_l[2] = {};
  float* d_hist_t[2] = {};
  int* d_nl[2] = {};
  int* d_nt[2] = {};
  int cur = 0;
  unsigned long long* d_skeys[2] = {};  // sorted gated history keys (double-buffered state)
  int* d_ns[2] = {};
  uint32_t* d_t0[2] = {};
  // per-batch meter scratch, two sets by the state's parity (cur): the next batch's prep writes the
  // other set from before its K-weighting values are in, while this batch's queries read this one
  float* d_core[2] = {nullptr, nullptr};
  MeterExt* d_ext[2] = {nullptr, nullptr};
  int* d_ncore[2] = {nullptr, nullptr};
  int* d_next[2] = {nullptr, nullptr};
  int* d_gcount[2] = {nullptr, nullptr};
  double* d_gsum[2] = {nullptr, nullptr};
  int HL = 0, HT = 0;
  // staging for OMEGA_MEM_HOST: device slots, page-locked host slots for the inputs, and one device +
  // page-locked output arena per call (every output of a call comes back in one D2H copy)
  std::vector<DevBuf> stage;
  std::vector<DevBuf> pin;
  DevBuf oarena, oarena_pin;
  size_t oarena_used = 0, oarena_want = 0;  // the device output arena's use in this call, its wanted size
  size_t zc_used = 0;                       // the zero-copy output buffer's use in this call
  // the call's outputs may be written by the kernels straight into the page-locked arena (set by calls
  // whose kernels only store their outputs: no output is read back by another workgroup)
  bool zc_ok = false;
  DevBuf zc_pin;
  void* zc_dev = nullptr;
  std::vector<void*> allocs;
};

namespace {

int fail(omega_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) {
    std::memcpy(c->err, buf, sizeof buf);
    c->zc_ok = false;  // (a host call that fails before finish_host)
  }
  return code;
}

#define HIPC(ctx, x)                                                                           \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(ctx, OMEGA_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// The ABI contract (omega.h: no C++ exception and no abort crosses it): every extern "C" entry point
// is a function-try-block whose handler maps what escaped -- std::bad_alloc from a host container, or
// anything else -- to a status code and omega_last_error. Called only from inside a catch clause.
int guard_fail(omega_ctx* c) noexcept {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    return fail(c, OMEGA_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(c, OMEGA_EHIP, "internal error: %s", e.what());
  } catch (...) {
    return fail(c, OMEGA_EHIP, "internal error: unknown exception");
  }
}

template <class T>
int dalloc(omega_ctx* c, T** p, size_t count) {
  void* q = nullptr;
  const hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) return fail(c, OMEGA_ENOMEM, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
  c->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return 0;
}

// A per-call scratch buffer of at least `need` elements: grown by replacement (the old buffer freed
// once this context's streams are idle -- work already enqueued may still read it; other contexts and
// streams on the device are not waited for), so repeated calls with growing sizes keep one buffer
// instead of accumulating them until omega_destroy.
template <class T>
int grow(omega_ctx* c, T** p, int64_t* cap, int64_t need) {
  if (need <= *cap) return 0;
  if (*p) {
    HIPC(c, hipStreamSynchronize(c->stream));
    for (hipStream_t f : c->fork)
      if (f) HIPC(c, hipStreamSynchronize(f));
    auto it = std::find(c->allocs.begin(), c->allocs.end(), static_cast<void*>(*p));
    if (it != c->allocs.end()) c->allocs.erase(it);
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
  }
  if (int e = dalloc(c, p, (size_t)need)) return e;
  *cap = need;
  return 0;
}

template <class T>
int upload(omega_ctx* c, T** p, const std::vector<T>& v) {
  int r = dalloc(c, p, v.size());
  if (r) return r;
  HIPC(c, hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// staging buffer slot i of at least bytes
int stage_buf(omega_ctx* c, int i, size_t bytes, void** out) {
  if ((int)c->stage.size() <= i) c->stage.resize(i + 1);
  DevBuf& b = c->stage[i];
  if (b.n < bytes) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    const hipError_t e = hipMalloc(&b.p, std::max<size_t>(bytes, 256));
    if (e != hipSuccess) return fail(c, OMEGA_ENOMEM, "staging hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    b.n = std::max<size_t>(bytes, 256);
  }
  *out = b.p;
  return 0;
}

int build_twiddles(omega_ctx* c) {
  for (int l = 1; l < kMaxLog2; ++l) {
    const int N = 1 << l;
    std::vector<float2> t(N);
    for (int m = 0; m < N; ++m) {
      const double a = 2.0 * kPi * (double)m / (double)N;
      t[m] = make_float2((float)std::cos(a), (float)-std::sin(a));
    }
    int r = upload(c, &c->d_tw[l], t);
    if (r) return r;
  }
  return 0;
}

int get_kw_tab(omega_ctx* c, int M, int L, BiquadTab** out) {
  const auto key = std::make_pair(M, L);
  auto it = c->kw_tabs.find(key);
  if (it != c->kw_tabs.end()) {
    *out = it->second;
    return 0;
  }
  const double fs = c->cfg.sample_rate;
  std::vector<BiquadTab> t = {make_biquad_tab(butter2_highpass(38.0, fs), L),
                              make_biquad_tab(butter2_highpass(1500.0, fs), L)};
  BiquadTab* d = nullptr;
  int r = upload(c, &d, t);
  if (r) return r;
  c->kw_tabs[key] = d;
  *out = d;
  return 0;
}
int get_kw_tab(omega_ctx* c, int M, BiquadTab** out) { return get_kw_tab(c, M, kw_chunk(M), out); }

int get_window(omega_ctx* c, int m, int kind, float** out) {
  auto key = std::make_pair(m, kind);
  auto it = c->windows.find(key);
  if (it != c->windows.end()) {
    *out = it->second;
    return 0;
  }
  float* d = nullptr;
  int r = upload(c, &d, make_window(m, kind));
  if (r) return r;
  c->windows[key] = d;
  *out = d;
  return 0;
}

// The window of make_window as the register-FFT bodies' generator (regfft.hpp WinGen): with
// phi = pi n / (M - 1), n = 1 - M + 2i, cos(phi) = -C_i and cos(2 phi) = 2 C_i^2 - 1, C_i = cos(2 pi i / (M - 1)),
// so a0 + a1 cos(phi) + a2 cos(2 phi) = (a0 - a2) + C_i (-a1 + 2 a2 C_i); thread t of NTH = M / 32 takes the
// points 2 (t + NTH q) + e
int get_wingen(omega_ctx* c, int m, int kind, float4** out) {
  auto key = std::make_pair(m, kind);
  auto it = c->wgens.find(key);
  if (it != c->wgens.end()) {
    *out = it->second;
    return 0;
  }
  if (m < 1024 || m % 32) return fail(c, OMEGA_EINVAL, "window generator: %d points", m);
  double a0 = 1.0, a1 = 0.0, a2 = 0.0;
  switch (kind) {
    case OMEGA_WIN_BLACKMAN: a0 = 0.42; a1 = 0.5; a2 = 0.08; break;
    case OMEGA_WIN_HANN: a0 = 0.5; a1 = 0.5; break;
    case OMEGA_WIN_HAMMING: a0 = 0.54; a1 = 0.46; break;
    default: break;
  }
  const int nth = m / 32;
  const double th = 2.0 * kPi / (m - 1);
  std::vector<float4> g(9 + nth);
  g[0] = make_float4((float)(a0 - a2), (float)(-a1), (float)(2.0 * a2), 0.f);
  for (int q = 0; q < 16; ++q) {
    const double b = th * (2.0 * nth * q);
    float4& e = g[1 + q / 2];
    if (q & 1) {
      e.z = (float)std::cos(b);
      e.w = (float)std::sin(b);
    } else {
      e.x = (float)std::cos(b);
      e.y = (float)std::sin(b);
    }
  }
  for (int t = 0; t < nth; ++t)
    g[9 + t] = make_float4((float)std::cos(th * 2 * t), (float)std::sin(th * 2 * t), (float)std::cos(th * (2 * t + 1)),
                           (float)std::sin(th * (2 * t + 1)));
  float4* d = nullptr;
  int r = upload(c, &d, g);
  if (r) return r;
  c->wgens[key] = d;
  *out = d;
  return 0;
}

// true-peak rotation e^{2 pi i k / (4M)}, k <= M/2
int get_rot(omega_ctx* c, int M, float2** out) {
  auto it = c->rots.find(M);
  if (it != c->rots.end()) {
    *out = it->second;
    return 0;
  }
  std::vector<float2> rot(M / 2 + 1);
  for (int k = 0; k <= M / 2; ++k) {
    const double a = 2.0 * kPi * (double)k / (4.0 * M);
    rot[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  float2* d = nullptr;
  int r = upload(c, &d, rot);
  if (r) return r;
  c->rots[M] = d;
  *out = d;
  return 0;
}

int validate(omega_ctx* c, const omega_config* cfg) {
  // MultiResolutionFFT.__init__ (multi_resolution_fft.py:139-142) and FFTConfig.__post_init__ (:35-44)
  if (cfg->sample_rate <= 0) return fail(c, OMEGA_EINVAL, "Sample rate must be positive");
  if (cfg->max_freq <= 0 || cfg->max_freq > cfg->sample_rate / 2.0)
    return fail(c, OMEGA_EINVAL, "Max frequency must be positive and <= Nyquist");
  if (cfg->n_res < 1 || cfg->n_res > OMEGA_MAX_RES) return fail(c, OMEGA_EINVAL, "n_res must be 1..%d", OMEGA_MAX_RES);
  for (int r = 0; r < cfg->n_res; ++r) {
    const omega_resolution& q = cfg->res[r];
    if (q.freq_lo >= q.freq_hi) return fail(c, OMEGA_EINVAL, "Invalid frequency range: (%g, %g)", q.freq_lo, q.freq_hi);
    if (q.fft_size <= 0 || (q.fft_size & (q.fft_size - 1)) != 0)
      return fail(c, OMEGA_EINVAL, "FFT size must be power of 2: %d", q.fft_size);
    if (q.hop_size <= 0) return fail(c, OMEGA_EINVAL, "Hop size must be positive: %d", q.hop_size);
    if (!(q.weight > 0)) return fail(c, OMEGA_EINVAL, "Weight must be positive: %g", q.weight);
  }
  if (!is_pow2_in(cfg->frame_size, 512, 16384))
    return fail(c, OMEGA_EUNSUP, "frame_size %d: power of two 512..16384 required", cfg->frame_size);
  for (int r = 0; r < cfg->n_res; ++r) {
    const omega_resolution& q = cfg->res[r];
    if (q.fft_size < 2 || q.fft_size > cfg->frame_size)
      return fail(c, OMEGA_EUNSUP, "fft_size %d: 2..frame_size(%d) supported", q.fft_size, cfg->frame_size);
  }
  if (cfg->target_bins < 1 || cfg->target_bins > (1 << 24)) return fail(c, OMEGA_EINVAL, "target_bins out of range");
  if (cfg->n_channels < 1) return fail(c, OMEGA_EINVAL, "n_channels must be >= 1");
  if (cfg->integrated_len < 1 || cfg->integrated_len > 4096)
    return fail(c, OMEGA_EUNSUP, "integrated_len %d: 1..4096 supported", cfg->integrated_len);
  if (cfg->momentary_len < 1 || cfg->short_len < 1 || cfg->peak_len < 1)
    return fail(c, OMEGA_EINVAL, "deque lengths must be >= 1");
  return 0;
}

void drop_graphs(omega_ctx* c) {
  for (auto& g : c->graphs) {
    (void)hipGraphExecDestroy(g.exec);
    (void)hipGraphDestroy(g.graph);
  }
  c->graphs.clear();
}

// True-peak kernel choice: the register-FFT kernel for 8192- and 16384-sample frames, the LDS-pass
// kernel for the other powers of two.
hipError_t tp_launch(omega_ctx* c, int W, const SpectralParams& sp, hipStream_t s) {
  (void)c;
  if (W == 16384 || W == 8192) return launch_truepeak_rf(W, sp, s);
  return launch_truepeak(W, sp, s);
}

int build_spectral_tables(omega_ctx* c) {
  const omega_config& cfg = c->cfg;
  const double fs = cfg.sample_rate;
  std::vector<std::vector<float>> wg(cfg.n_res);  // host copies of the weight tables
  for (int r = 0; r < cfg.n_res; ++r) {
    const omega_resolution& q = cfg.res[r];
    const int N = q.fft_size;
    int e = get_window(c, N, q.window, &c->d_win[r]);
    if (e) return e;
    // multi_resolution_fft.py:310-326 -- float32 weights, float32 compounding
    std::vector<float> w(N / 2 + 1);
    for (int k = 0; k <= N / 2; ++k) {
      const double f = rfreq(k, N, fs);
      float v = (float)q.weight;
      if (cfg.apply_weighting) {
        const bool in = f >= q.freq_lo && f <= q.freq_hi;
        if (in && f >= 60 && f <= 120) v = v * 1.8f;
        if (in && f >= 200 && f <= 400) v = v * 1.4f;
        if (in && f >= 2000 && f <= 5000) v = v * 1.2f;
        if (in && f >= 20 && f <= 80) v = v * 1.6f;
      } else {
        v = 1.0f;
      }
      w[k] = v;
    }
    e = upload(c, &c->d_wgt[r], w);
    if (e) return e;
    wg[r] = std::move(w);
  }
  // combine plan (multi_resolution_fft.py:353-395)
  const int T = cfg.target_bins;
  const double mf = std::min(cfg.max_freq, fs / 2);
  std::vector<double> tgt(T);
  const double step = T > 1 ? mf / (T - 1) : 0.0;  // np.linspace(0, mf, T)
  for (int t = 0; t < T; ++t) tgt[t] = t * step;
  if (T > 1) tgt[T - 1] = mf;
  struct Ent {
    int r, j;
    float fr;
  };
  std::vector<std::vector<Ent>> own(T);
  for (int r = 0; r < cfg.n_res; ++r) {
    const omega_resolution& q = cfg.res[r];
    const int N = q.fft_size;
    std::vector<int> vidx;
    for (int k = 0; k <= N / 2; ++k) {
      const double f = rfreq(k, N, fs);
      if (f >= q.freq_lo && f <= q.freq_hi) vidx.push_back(k);
    }
    if (vidx.size() < 2) continue;  // :367-374
    for (int t = 0; t < T; ++t) {
      const double x = tgt[t];
      if (!(x >= q.freq_lo && x <= q.freq_hi)) continue;
      const double f0 = rfreq(vidx.front(), N, fs), f1 = rfreq(vidx.back(), N, fs);
      Ent en{r, 0, 0.f};
      if (x <= f0) {
        en.j = vidx.front();
      } else if (x >= f1) {
        en.j = vidx.back();
      } else {
        // vidx is contiguous: x in [f_j, f_{j+1})
        const double val = rfreq(1, N, fs);
        int j = (int)std::floor(x / val);
        j = std::max(vidx.front(), std::min(j, vidx.back() - 1));
        while (j > vidx.front() && rfreq(j, N, fs) > x) --j;
        while (j + 1 < vidx.back() && rfreq(j + 1, N, fs) <= x) ++j;
        const double fa = rfreq(j, N, fs), fb = rfreq(j + 1, N, fs);
        en.j = j;
        en.fr = (float)((x - fa) / (fb - fa));
      }
      own[t].push_back(en);
    }
  }
  c->res_independent = true;
  for (int t = 0; t < T; ++t)
    if (own[t].size() > 1) c->res_independent = false;
  // per-resolution combine entries (see CombEnt): the interpolation of weighted magnitudes
  // m_j + fr (m_{j+1} - m_j), m = |X| * wgt, times cw / sum of the target's owner weights
  std::vector<std::vector<CombEnt>> er(cfg.n_res);
  for (int t = 0; t < T; ++t) {
    const auto& o = own[t];
    if (o.empty()) {
      er[0].push_back(CombEnt{t | (2 << 24), 0, 0.f, 0.f});
      continue;
    }
    double ws = 0.0;
    for (const Ent& en : o) ws += (double)(float)cfg.res[en.r].weight;
    for (size_t q = 0; q < o.size(); ++q) {
      const Ent& en = o[q];
      const double s = (double)(float)cfg.res[en.r].weight / ws;
      const double fr = en.fr;
      const int op = (q == 0 ? 0 : 1) << 24;
      if (en.fr == 0.f && en.j == cfg.res[en.r].fft_size / 2)  // last bin: keep j + 1 in range
        er[en.r].push_back(CombEnt{t | op, en.j - 1, 0.f, (float)(wg[en.r][en.j] * s)});
      else
        er[en.r].push_back(CombEnt{t | op, en.j, (float)((1.0 - fr) * wg[en.r][en.j] * s),
                                   (float)(en.fr != 0.f ? fr * wg[en.r][en.j + 1] * s : 0.0)});
    }
  }
  std::vector<CombEnt> all;
  for (int r = 0; r < cfg.n_res; ++r) {
    c->ent_begin[r] = (int)all.size();
    all.insert(all.end(), er[r].begin(), er[r].end());
    c->ent_end[r] = (int)all.size();
    c->ent_jmax[r] = 0;
    for (const CombEnt& en : er[r]) c->ent_jmax[r] = std::max(c->ent_jmax[r], en.j + 1);
    // the magnitude pairs (k, K - k) holding every bin an entry reads (j and j + 1): one untangle per
    // pair instead of two per entry, where that is fewer (ResParam::pair_lo / pair_hi)
    const int K = cfg.res[r].fft_size / 2;
    int plo = K, phi = -1;
    for (const CombEnt& en : er[r]) {
      if ((en.tm >> 24) == 2) continue;
      for (int b = en.j; b <= en.j + 1; ++b) {
        const int k = (b == K || b == K / 2) ? 0 : std::min(b, K - b);
        plo = std::min(plo, k);
        phi = std::max(phi, k);
      }
    }
    c->pair_lo[r] = c->pair_hi[r] = 0;
    if (phi >= 0 && K >= 2 && (phi + 1 - plo) < 2 * (int)er[r].size()) {
      c->pair_lo[r] = plo;
      c->pair_hi[r] = phi + 1;
    }
  }
  std::vector<int> ooff(1, 0), orj;
  std::vector<float> ofr;
  for (int t = 0; t < T; ++t) {
    for (const Ent& en : own[t]) {
      orj.push_back((en.r << 24) | en.j);
      ofr.push_back(en.fr);
    }
    ooff.push_back((int)orj.size());
  }
  int e = upload(c, &c->d_own_off, ooff);
  if (!e) e = upload(c, &c->d_own_rj, orj);
  if (!e) e = upload(c, &c->d_own_frac, ofr);
  if (!e) e = upload(c, &c->d_ent, all);
  if (e) return e;
  return get_rot(c, cfg.frame_size, &c->d_rot);
}

int build_meter_state(omega_ctx* c) {
  const int C = c->cfg.n_channels;
  c->HL = std::max(1, c->cfg.integrated_len - 1);
  c->HT = std::max(1, c->cfg.peak_len - 1);
  for (int b = 0; b < 2; ++b) {
    int e = dalloc(c, &c->d_hist_l[b], (size_t)C * c->HL);
    if (!e) e = dalloc(c, &c->d_hist_t[b], (size_t)C * c->HT);
    if (!e) e = dalloc(c, &c->d_nl[b], C);
    if (!e) e = dalloc(c, &c->d_nt[b], C);
    if (e) return e;
  }
  int e = 0;
  for (int b = 0; b < 2 && !e; ++b) {
    e = dalloc(c, &c->d_skeys[b], (size_t)C * c->HL);
    if (!e) e = dalloc(c, &c->d_ns[b], C);
    if (!e) e = dalloc(c, &c->d_t0[b], C);
  }
  for (int b = 0; b < 2; ++b) {
    if (!e) e = dalloc(c, &c->d_core[b], (size_t)C * kMeterSeqCap);
    if (!e) e = dalloc(c, &c->d_ext[b], (size_t)C * kMeterSeqCap);
    if (!e) e = dalloc(c, &c->d_ncore[b], C);
    if (!e) e = dalloc(c, &c->d_next[b], C);
    if (!e) e = dalloc(c, &c->d_gcount[b], (size_t)C * (kMeterSeqCap + 1));
    if (!e) e = dalloc(c, &c->d_gsum[b], (size_t)C * (kMeterSeqCap + 1));
  }
  if (!e) e = dalloc(c, &c->d_kw_done, 8);
  if (e) return e;
  if (!c->h_err) {
    HIPC(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_err), 2 * sizeof(unsigned),
                          hipHostMallocMapped | hipHostMallocCoherent));
    c->h_err[0] = c->h_err[1] = 0;
    HIPC(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_err), c->h_err, 0));
  }
  HIPC(c, hipMemset(c->d_kw_done, 0, 8 * sizeof(unsigned)));
  c->kw_issued = c->q_issued = c->tp_issued = c->prep_issued = c->seg_issued = c->lt_issued = 0;
  c->seg_par[0] = c->seg_par[1] = 0;
  c->pend = false;
  return omega_meter_reset(c);
}

SpectralParams spectral_params(omega_ctx* c) {
  SpectralParams p{};
  p.tp_phases = 0xE;
  p.C = c->cfg.n_channels;
  p.n_res = c->cfg.n_res;
  p.rf_sizes = c->rf_sizes;
  for (int r = 0; r < p.n_res; ++r) {
    ResParam& q = p.res[r];
    q.n = c->cfg.res[r].fft_size;
    q.offset = c->cfg.frame_size - q.n;
    q.win = c->d_win[r];
    q.wgt = c->d_wgt[r];
    q.ent_begin = c->ent_begin[r];
    q.ent_end = c->ent_end[r];
    q.cw = (float)c->cfg.res[r].weight;
    q.low_band = c->ent_jmax[r] < 256;
    q.pair_lo = c->pair_lo[r];
    q.pair_hi = c->pair_hi[r];
  }
  p.ent = c->d_ent;
  p.T = c->cfg.target_bins;
  p.rot = c->d_rot;
  for (int l = 0; l < kMaxLog2; ++l) p.tw[l] = c->d_tw[l];
  return p;
}

bool aligned8(const void* p) { return ((uintptr_t)p & 7) == 0; }

// ---- host-memory staging helpers ----
struct HostOut {
  void* host;
  void* dev;
  size_t bytes;
  size_t arena_off;  // offset in the output arena, or ~0 (a slot of its own)
};

// Page-locked host buffer of at least `bytes` (grown on demand; hipHostMalloc).
int pinned_buf(omega_ctx* c, DevBuf& b, size_t bytes) {
  if (b.n >= bytes) return 0;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.n = 0;
  const size_t n = std::max<size_t>(bytes, 4096);
  const hipError_t e = hipHostMalloc(&b.p, n, hipHostMallocDefault);
  if (e != hipSuccess) return fail(c, OMEGA_ENOMEM, "staging hipHostMalloc(%zu): %s", n, hipGetErrorString(e));
  b.n = n;
  return 0;
}

// Host input -> device-visible buffer: copied into the slot's page-locked buffer on the CPU. Up to
// kZeroCopyIn bytes the kernels read it there (one fabric read per element, no copy command before the
// launch); larger inputs follow with an async H2D copy into the slot's device buffer (a pageable source
// would make the runtime stage and wait on every copy).
constexpr size_t kZeroCopyIn = 256 * 1024;
constexpr size_t kZeroCopyOut = 256 * 1024;
constexpr size_t kZeroCopyTag = (size_t)1 << 62;  // HostOut::arena_off of an output in zc_pin
int stage_in(omega_ctx* c, int slot, const void* host, size_t bytes, const void** dev) {
  if ((int)c->pin.size() <= slot) c->pin.resize(slot + 1);
  int e = pinned_buf(c, c->pin[slot], bytes);
  if (e) return e;
  if (bytes) std::memcpy(c->pin[slot].p, host, bytes);
  if (bytes <= kZeroCopyIn) {
    void* dp = nullptr;
    HIPC(c, hipHostGetDevicePointer(&dp, c->pin[slot].p, 0));
    *dev = dp;
    return 0;
  }
  void* d = nullptr;
  e = stage_buf(c, slot, bytes, &d);
  if (e) return e;
  HIPC(c, hipMemcpyAsync(d, c->pin[slot].p, bytes, hipMemcpyHostToDevice, c->stream));
  *dev = d;
  return 0;
}

// Host output: a device range of the call's output arena, or (zc_ok) of the zero-copy buffer, each with
// its own use counter, both reset by the call's first output. The device arena is grown, when an earlier
// call wanted more, at this call's first output placed in it (nothing of this call is in it yet); this
// call's outputs past its end use their own slots. finish_host copies the arena back in one D2H copy.
template <class T>
int stage_out(omega_ctx* c, int slot, T* host, size_t count, std::vector<HostOut>& outs, T** dev) {
  if (!host) {
    *dev = nullptr;
    return 0;
  }
  if (outs.empty()) {
    c->oarena_used = 0;
    c->zc_used = 0;
  }
  const size_t bytes = count * sizeof(T);
  if (c->zc_ok) {
    // small outputs of a store-only call: straight into page-locked memory (no copy command after the
    // kernels; finish_host only copies them to the caller's buffers on the CPU)
    const size_t off = (c->zc_used + 255) & ~(size_t)255;
    if (off + bytes <= kZeroCopyOut) {
      if (!c->zc_pin.p) {
        if (int e = pinned_buf(c, c->zc_pin, kZeroCopyOut)) return e;
        HIPC(c, hipHostGetDevicePointer(&c->zc_dev, c->zc_pin.p, 0));
      }
      c->zc_used = off + bytes;
      outs.push_back({host, static_cast<char*>(c->zc_pin.p) + off, bytes, kZeroCopyTag + off});
      *dev = reinterpret_cast<T*>(static_cast<char*>(c->zc_dev) + off);
      return 0;
    }
  }
  if (c->oarena_used == 0) {
    if (c->oarena_want > c->oarena.n) {
      const size_t n = c->oarena_want + c->oarena_want / 4;
      if (c->oarena.p) (void)hipFree(c->oarena.p);
      c->oarena.p = nullptr;
      c->oarena.n = 0;
      if (hipMalloc(&c->oarena.p, n) == hipSuccess) {
        c->oarena.n = n;
        if (int e = pinned_buf(c, c->oarena_pin, n)) return e;
      }
    }
  }
  const size_t off = (c->oarena_used + 255) & ~(size_t)255;
  if (off + bytes <= c->oarena.n && c->oarena_pin.n >= c->oarena.n) {
    c->oarena_used = off + bytes;
    outs.push_back({host, static_cast<char*>(c->oarena.p) + off, bytes, off});
    *dev = reinterpret_cast<T*>(static_cast<char*>(c->oarena.p) + off);
    return 0;
  }
  c->oarena_want = std::max(c->oarena_want, off + bytes);
  void* d = nullptr;
  int e = stage_buf(c, slot, bytes, &d);
  if (e) return e;
  outs.push_back({host, d, bytes, ~(size_t)0});
  *dev = static_cast<T*>(d);
  return 0;
}

// A device-side ordering wait that expired (meters.hip: the prep kernel's wait for the batch's
// K-weighting count, the join of the LUFS meters into the caller's stream) means some meter aggregates
// were computed from, or returned before, incomplete inputs: report it once as OMEGA_EHIP.
int check_device_err(omega_ctx* c) {
  if (!c->h_err) return 0;
  volatile unsigned* e = c->h_err;
  const unsigned prep = e[0], join = e[1];
  if (!prep && !join) return 0;
  e[0] = 0;
  e[1] = 0;
  return fail(c, OMEGA_EHIP, "device-side meter ordering wait expired (%s%s%s): meter aggregates of an earlier call "
              "may be stale", prep ? "meter prep waiting for the K-weighting count" : "", prep && join ? ", " : "",
              join ? "caller's stream joining the LUFS meters" : "");
}

// Host-memory calls: copy the outputs back and wait; an ordering wait of THIS call that expired is
// reported by this call (device-memory calls report it at the next call or omega_synchronize).
int finish_host(omega_ctx* c, const std::vector<HostOut>& outs) {
  c->zc_ok = false;
  size_t span = 0;
  for (const HostOut& o : outs) {
    if (o.arena_off == ~(size_t)0)
      HIPC(c, hipMemcpyAsync(o.host, o.dev, o.bytes, hipMemcpyDeviceToHost, c->stream));
    else if (o.arena_off < kZeroCopyTag)
      span = std::max(span, o.arena_off + o.bytes);
  }
  if (span) HIPC(c, hipMemcpyAsync(c->oarena_pin.p, c->oarena.p, span, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  if (c->fork[0] && hipStreamQuery(c->fork[0]) != hipSuccess) HIPC(c, hipStreamSynchronize(c->fork[0]));
  for (const HostOut& o : outs) {
    if (o.arena_off == ~(size_t)0) continue;
    const char* src = o.arena_off >= kZeroCopyTag ? static_cast<const char*>(o.dev)
                                                   : static_cast<char*>(c->oarena_pin.p) + o.arena_off;
    std::memcpy(o.host, src, o.bytes);
  }
  return check_device_err(c);
}

// Meter aggregates over n_frames x C values, in chunks of at most kChunkFrames frames; each chunk
// reads the state buffers `cur` and writes `cur ^ 1`.
std::vector<MeterPrepParams> meter_chunks(omega_ctx* c, const float* lufs, const float* tp, int64_t n_frames,
                                          double* out) {
  const int C = c->cfg.n_channels;
  std::vector<MeterPrepParams> v;
  for (int64_t f0 = 0; f0 < n_frames; f0 += kChunkFrames) {
    const int64_t nf = std::min<int64_t>(kChunkFrames, n_frames - f0);
    const int a = c->cur, b = c->cur ^ 1;
    MeterPrepParams p{};
    p.lufs = lufs + f0 * C;
    p.tp = tp + f0 * C;
    p.n_frames = nf;
    p.C = C;
    p.hist_l_in = c->d_hist_l[a];
    p.hist_t_in = c->d_hist_t[a];
    p.n_l_in = c->d_nl[a];
    p.n_t_in = c->d_nt[a];
    p.skeys_in = c->d_skeys[a];
    p.n_s_in = c->d_ns[a];
    p.t0_in = c->d_t0[a];
    p.hist_l_out = c->d_hist_l[b];
    p.hist_t_out = c->d_hist_t[b];
    p.n_l_out = c->d_nl[b];
    p.n_t_out = c->d_nt[b];
    p.skeys_out = c->d_skeys[b];
    p.n_s_out = c->d_ns[b];
    p.t0_out = c->d_t0[b];
    p.HL = c->HL;
    p.HT = c->HT;
    p.mom_len = c->cfg.momentary_len;
    p.short_len = c->cfg.short_len;
    p.int_len = c->cfg.integrated_len;
    p.peak_len = c->cfg.peak_len;
    p.poll_limit = c->poll_limit;
    p.err_word = c->d_err;
    p.gate = (float)c->cfg.gate_lufs;
    p.core = c->d_core[a];
    p.ext = c->d_ext[a];
    p.n_core = c->d_ncore[a];
    p.n_ext = c->d_next[a];
    p.gcount = c->d_gcount[a];
    p.gsum = c->d_gsum[a];
    p.out = out + f0 * C * OMEGA_N_METERS;
    p.parts = 3;
    p.seg_ctr = c->d_kw_done + 4;
    p.seg_pre_target = c->seg_par[a];
    p.seg_post_target = c->seg_par[b];
    v.push_back(p);
    c->cur = b;
  }
  return v;
}

// All meter chunks on one stream. tp_ready: when set, an event the true peaks of the batch wait on
// (the prep kernels only read the LUFS_inst values, so they may start before it).
int meters_enqueue(omega_ctx* c, const float* lufs, const float* tp, int64_t n_frames, double* out,
                   hipStream_t stream, hipEvent_t tp_ready, unsigned* wait_ctr = nullptr, unsigned wait_target = 0) {
  bool first = true;
  for (MeterPrepParams p : meter_chunks(c, lufs, tp, n_frames, out)) {
    // (wait_ctr: the first chunk's prep polls it before reading the batch's values -- the true peaks
    // of omega_calculate_lufs on the side stream counting in, instead of an event join)
    if (first && wait_ctr) {
      p.wait_ctr = wait_ctr;
      p.wait_target = wait_target;
    }
    HIPC(c, launch_meter_prep(p, stream));
    if (tp_ready && first) HIPC(c, hipStreamWaitEvent(stream, tp_ready, 0));
    HIPC(c, launch_meter_query(p, stream));
    first = false;
  }
  return 0;
}

// Meter pipelining: the pending meter segment as a launch of its own on the context's stream (the
// stream of the batch it belongs to: omega_set_stream flushes before switching).
// Meter pipelining: the pending meter segment as a launch of its own on the context's stream (the
// stream of the batch it belongs to: omega_set_stream flushes before switching).
int flush_meters(omega_ctx* c) {
  if (!c->pend) return 0;
  HIPC(c, hipSetDevice(c->device));
  BatchPlan bp{};
  bp.q_begin = 0;
  bp.q_n = c->pend_nq;
  bp.seg_start[0] = bp.seg_start[1] = bp.multi_start = c->pend_nq;  // (no other workgroups)
  SpectralParams sp{};
  KWeightParams kp{};
  const hipError_t le = launch_batch(sp, kp, bp, c->pend_mq, c->pend_nq, c->stream);
  if (le != hipSuccess) return fail(c, OMEGA_EHIP, "meter segment launch: %s", hipGetErrorString(le));
  c->pend = false;
  c->seg_par[c->pend_par] = c->seg_issued + (unsigned)c->pend_nq;
  c->seg_issued += (unsigned)c->pend_nq;
  return 0;
}

// Layout 3 applies to 16384-sample frames on direct launches (a captured graph would freeze the
// kw_done target) when every requested stage has a 512-thread batch role: the register-FFT true peak,
// at most one 16384-point resolution (on the register FFT), the others at most 8192 points, and
// resolutions that commute (no combine target with several owners). *mr: the 16384-point resolution.
bool batch_eligible(omega_ctx* c, const SpectralParams& sp, const KWeightParams& kp, int W, bool do_res, hipStream_t s,
                    int* mr) {
  *mr = -1;
  if (W != 16384 || (c->cap && s == c->cap)) return false;  // (graph capture: the other layout)
  if ((kp.lufs_out || kp.weighted_out) && kp.mode != 0) return false;
  if (!do_res) return true;
  if (!c->res_independent) return false;
  for (int r = 0; r < sp.n_res; ++r) {
    if (!sp.comb_out && !sp.res[r].mag_out) continue;
    const int n = sp.res[r].n;
    if (n == 16384) {
      if (*mr >= 0 || !((sp.rf_sizes >> 14) & 1)) return false;
      *mr = r;
    } else if (n < 512 || n > 8192) {
      return false;
    }
  }
  return true;
}

// The default layout for 16384-sample frames. On `s`: one batch_kernel launch (BatchPlan: K-weighting
// and 16384-point-resolution workgroups mixed, then the true peaks, then the small resolutions, then --
// for a batch of at most kChunkFrames frames per channel -- the meter aggregates as the grid's last
// segment; pipelined, the previous call's, between the true peaks and the small resolutions). On
// fork[0]: the meter prep (it waits on the K-weighting count, kw_done, and counts itself
// in). The meter workgroups wait for the prep's count and for the true peaks' count, so `s` completes
// only after fork[0]'s work: no stream events and no kernel after the batch (each event record / wait
// cost ~7-13 us of idle GPU between kernels). Longer batches (chunks chained through the per-context
// scratch) keep the meter query kernels: the LUFS query on fork[0] counting itself in, the true-peak
// query after the batch on `s` joining that count. Mixing the latency-bound K-weighting scans with
// transform work is what pays (K-weighting alone 25.7 us, the true peak 37, the resolutions 26.5; one
// batch launch of all three 73.9). Measured and rejected on MI355X (rounds 1-3): other role
// orders (K-weighting as its own kernel 110.4 us per step; mixed with the true peaks 85.2; the true
// peaks first ~equal; role chunks of one workgroup per CU), the meter queries after the batch (88 vs
// 81-82), the true-peak query on the side stream joined in the batch's last workgroup (85-87), the
// true-peak meter as a batch role (86-88), the true-peak meter by the batch's last true-peak workgroup,
// joined there (86.2 vs 81.1, round 3). The in-grid meter segment measured even with the query kernels
// (step 79.4-80.6 vs 79.0-79.4 us) at two fewer launches per call (host enqueue 13-17 vs 22-27 us).
int enqueue_batch(omega_ctx* c, SpectralParams sp, KWeightParams kp, int W, int64_t n_frames, const float* lufs,
                  const float* tp, double* meters, hipStream_t s, int mr, bool do_tp, bool do_kw, bool fold) {
  (void)W;
  const int64_t n = sp.n_cf;
  BatchPlan bp{};
  int seg[2][3], ns[2] = {0, 0};
  auto add = [&](int sg, int role, bool on) {
    if (on) seg[sg][ns[sg]++] = role;
  };
  // (measured: the true peaks in segment 0 beside the K-weighting, the 16384-point resolution in
  // segment 1, with or without the small resolutions before it: step 73.5-75.1 vs 68.8-70.5 us)
  // (measured, round 5, pipelined step on one box: the K-weighting beside the true peaks with the
  // 16384-point resolution after them, or the true peaks beside the 16384-point resolution with the
  // K-weighting after them, 65.3-67.3 us against 65.3-67.1 for this order: the same)
  add(0, 0, do_kw);        // segment 0: K-weighting and the 16384-point resolution, groups of 8 frames
  add(0, 2, mr >= 0);
  add(1, 1, do_tp);        // segment 1: the true peaks
  const int64_t groups = (n + 7) / 8;
  int64_t end = 0;
  for (int sg = 0; sg < 2; ++sg) {
    bp.n_roles[sg] = ns[sg] ? ns[sg] : 1;
    for (int i = 0; i < 3; ++i) bp.roles[sg][i] = i < ns[sg] ? seg[sg][i] : 0;
    end += ns[sg] ? 8 * ns[sg] * groups : 0;
    if (end > 0x7FFFFFFF) return fail(c, OMEGA_EINVAL, "batch of %lld channel-frames too large", (long long)n);
    bp.seg_begin[sg + 1] = (int)end;
  }
  bp.mr_res = mr < 0 ? 0 : mr;
  int64_t nwg = 0;
  for (int r = 0; r < sp.n_res; ++r) {
    if (r == mr || (!sp.comb_out && !sp.res[r].mag_out)) continue;
    const int K = sp.res[r].n / 2;
    const int G = K / 16 < 64 ? 64 : K / 16;  // threads_for<K>() for K <= 4096
    const int fpw = 512 / G;
    bp.multi.res[bp.multi.n_seg] = r;
    bp.multi.wg_begin[bp.multi.n_seg] = (int)nwg;
    ++bp.multi.n_seg;
    nwg += (n + fpw - 1) / fpw;
  }
  // the meter aggregates of a one-chunk batch as the grid's last segment (batch_meter_role): the prep
  // kernel on fork[0] (it waits for the K-weighting count) counts itself in, the true-peak workgroups
  // count themselves in, the meter workgroups wait for both; longer batches chain their chunks through
  // the per-context scratch and keep the query kernels
  const bool in_grid = meters && do_tp && do_kw && n_frames > 0 && n_frames <= kChunkFrames;
  const int64_t n_mq = in_grid ? std::min<int64_t>((n + kBatchWaves - 1) / kBatchWaves, kMeterWgs) : 0;
  // meter pipelining (fold): this launch runs the PREVIOUS call's meter segment as its last workgroups
  // (its inputs are complete: that batch ended before this one starts; the prep that reads this batch's
  // values still runs beside it on the side stream) and leaves its own pending
  fold = fold && in_grid;
  const int64_t q_n = fold ? (c->pend ? c->pend_nq : 0) : n_mq;
  // grid order: segment 0 | segment 1 | small resolutions (measured: the small resolutions between the
  // segments, step 80.4-81.3 vs 76.6-77.5 us, round 4); segment 0 in the period-8 role order
  // (BatchPlan::pat: batch kernel 65.7-66.1 vs 70.9-71.5 us)
  bp.pat = 1;
  bp.multi_n = (int)nwg;
  bp.seg_start[0] = 0;
  bp.seg_start[1] = bp.seg_begin[1];
  bp.multi_start = bp.seg_begin[2];
  const int64_t body_end = end + nwg;
  // the grid's last segment unpipelined (measured: placed before the small resolutions it holds 64
  // slots from ~50 us on while it waits and the step is no shorter, 77.4-79.2 vs 77.0-78.0 us);
  // pipelined, it waits for nothing (first in the grid it delayed the true peaks: step 68-69 vs 64-65
  // us without meters)
  bp.q_begin = (int)body_end;
  bp.q_n = (int)q_n;
  // pipelined (the previous call's segment: it waits for nothing), the segment goes after the true peaks
  // and before the small resolutions instead: longest-first in the tail, its ~9-10 us workgroups ahead
  // of the 7-12 us resolution ones (pipelined step 63.5-64.4 vs 64.9-65.2 us last, four alternations on
  // one box, tools/ab.sh, outputs bitwise equal direct and pipelined; on a second box 62.8-64.7 vs
  // 64.6-65.1 last and 62.8-64.4 after the 8192-point resolution).
  // Unpipelined it stays last: before the small resolutions its waiting workgroups cost the in-call
  // step 70.4-73.1 vs 66.9-67.6 us
  if (fold) bp.q_begin = bp.multi_start;
  // (measured, round 5: the pipelined segment between segment 0 and the true peaks instead, step
  // 65.3-67.1 vs 66.5-66.6 us on one box: no difference)
  const int64_t grid = body_end + q_n;
  if (grid > 0x7FFFFFFF) return fail(c, OMEGA_EINVAL, "batch of %lld channel-frames too large", (long long)n);
  MeterPrepParams mq{};
  std::vector<MeterPrepParams> mc;
  if (in_grid) {
    const int a = c->cur;
    const unsigned seg_par_was = c->seg_par[a ^ 1];
    // the pending segment (parity a ^ 1) is enqueued by this launch: the prep's target for the state it
    // reads (meter_chunks) counts it
    if (fold && c->pend) c->seg_par[c->pend_par] = c->seg_issued + (unsigned)c->pend_nq;
    const int cur_was = c->cur;  // (meter_chunks flips the state parity)
    mc = meter_chunks(c, lufs, tp, n_frames, meters);
    // the prep on the side stream, waiting for this batch's K-weighting count
    MeterPrepParams p = mc[0];
    p.q_done = c->d_kw_done + 3;
    // pipelined: the prep polls generation-tagged words the K-weighting workgroups store without a
    // drain or a count; unpipelined: the count
    const size_t mir_n = (size_t)kChunkFrames * c->cfg.n_channels;
    if (fold && !c->d_mirror) {
      HIPC(c, hipMalloc(&c->d_mirror, 2 * mir_n * sizeof(unsigned long long)));
      HIPC(c, hipMemset(c->d_mirror, 0, 2 * mir_n * sizeof(unsigned long long)));
    }
    const bool mirror = fold;
    const unsigned gen_was = c->mirror_gen;
    if (mirror) {
      // consecutive launches alternate parity: a prep still reading one parity while the next launch's
      // K-weighting writes the other (it waits for nothing), and done before the launch after that
      // (whose predecessor's segment waits for it)
      c->mirror_gen = c->mirror_gen == 0xFFFFFFFFu ? 2u : c->mirror_gen + 1;
      kp.lufs_mirror = c->d_mirror + (c->mirror_gen & 1) * mir_n;
      kp.mirror_gen = c->mirror_gen;
      p.lufs_mirror = kp.lufs_mirror;
      p.mirror_gen = c->mirror_gen;
    } else {
      kp.kw_done = c->d_kw_done;
      c->kw_issued += (unsigned)n;
      p.wait_ctr = c->d_kw_done;
      p.wait_target = c->kw_issued;
    }
    if (fold && c->tail_ok == 0) {
      int ok = 0;
      HIPC(c, hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, c->device));
      c->tail_ok = -1;
      if (ok && hipExtMallocWithFlags(reinterpret_cast<void**>(&c->d_tail), 8, hipMallocSignalMemory) == hipSuccess) {
        HIPC(c, hipMemset(c->d_tail, 0, 8));
        c->tail_issued = 0;
        c->tail_ok = 1;
      }
    }
    const bool tail = fold && c->tail_ok > 0;
    if (tail) bp.tail_ctr = c->d_tail;
    // unpipelined: the prep before the batch (it must be resident while the batch runs: its segment
    // waits for it); pipelined: after it, behind the stream wait -- enqueued before the batch, a wait
    // whose stream shared a hardware queue with the batch's would block the batch behind it for ever
    if (!fold) HIPC(c, launch_meter_prep(p, c->fork[0]));
    c->side_meters = true;
    mq = mc[0];
    mq.start_ctr = c->d_kw_done + 3;
    mq.start_target = c->prep_issued + (unsigned)p.C;
    // the meter segment's wait for the true peaks (each true-peak workgroup stores its value
    // write-through and counts in); a pipelined segment runs in a later launch, after this batch ended
    if (!fold) {
      sp.tp_done = c->d_kw_done + 2;
      mq.join_ctr = c->d_kw_done + 2;
      mq.join_target = c->tp_issued + (unsigned)n;
    }
    const hipError_t le = launch_batch(sp, kp, bp, fold ? c->pend_mq : mq, (int)grid, s);
    if (le != hipSuccess) {
      // the prep kernel already waits for this batch's count: publish it (see below)
      if (!fold) {
        (void)hipMemcpy(c->d_kw_done, &c->kw_issued, sizeof(unsigned), hipMemcpyHostToDevice);
        c->prep_issued += (unsigned)p.C;
      } else {
        // (no prep waits for this launch: nothing was enqueued; the generation goes back so the next
        // launch takes the other parity)
        c->mirror_gen = gen_was;
        c->seg_par[a ^ 1] = seg_par_was;  // (the pending segment stays pending)
        c->cur = cur_was;                 // (no prep writes the other parity's state)
      }
      return fail(c, OMEGA_EHIP, "batch launch: %s", hipGetErrorString(le));
    }
    if (!fold) c->tp_issued += (unsigned)n;
    if (tail) {
      HIPC(c, hipStreamWaitValue32(c->fork[0], c->d_tail, c->tail_issued + 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
      ++c->tail_issued;
    }
    if (fold) HIPC(c, launch_meter_prep(p, c->fork[0]));
    c->side_meters = true;
    c->prep_issued += (unsigned)p.C;
    if (fold) {
      if (c->pend) c->seg_issued += (unsigned)c->pend_nq;
      c->pend = true;
      c->pend_mq = mq;
      c->pend_nq = (int)n_mq;
      c->pend_par = a;
    } else {
      c->seg_par[a] = c->seg_issued + (unsigned)n_mq;
      c->seg_issued += (unsigned)n_mq;
    }
    return 0;
  }
  if (meters) {
    mc = meter_chunks(c, lufs, tp, n_frames, meters);
    kp.kw_done = c->d_kw_done;
    c->kw_issued += (unsigned)n;
    for (size_t i = 0; i < mc.size(); ++i) {
      MeterPrepParams p = mc[i];
      if (i == 0) {
        p.wait_ctr = c->d_kw_done;
        p.wait_target = c->kw_issued;
      }
      HIPC(c, launch_meter_prep(p, c->fork[0]));
      c->side_meters = true;
      p.parts = 1;
      p.q_done = c->d_kw_done + 1;
      HIPC(c, launch_meter_query(p, c->fork[0]));
      c->side_meters = true;
      c->q_issued += (unsigned)(((p.n_frames + 3) / 4) * p.C);  // (counted once it is enqueued)
    }
  }
  if (grid > 0) {
    const hipError_t le = launch_batch(sp, kp, bp, mq, (int)grid, s);
    if (le != hipSuccess) {
      // the prep kernel already waits for this batch's count: publish it, so that it (and every later
      // call's target) stays in step with the device counter instead of timing out
      if (meters) (void)hipMemcpy(c->d_kw_done, &c->kw_issued, sizeof(unsigned), hipMemcpyHostToDevice);
      return fail(c, OMEGA_EHIP, "batch launch: %s", hipGetErrorString(le));
    }
  }
  for (size_t i = 0; i < mc.size(); ++i) {
    MeterPrepParams p = mc[i];
    p.parts = 2;
    if (i + 1 == mc.size()) {
      p.join_ctr = c->d_kw_done + 1;
      p.join_target = c->q_issued;
    }
    HIPC(c, launch_meter_query(p, s));
  }
  return 0;
}

// fork[0] carries the latency-bound meter kernels beside full-chip work, at the default priority: a
// high-priority side stream measured the same on the cfg2 step (pipelined 65.7-68.7 vs 65.5-67.8 us,
// profiles/r05_ab_side_priority.txt) and made the event-joined paths 2-4x slower per call with one
// other context alive in the process (profiles/r05_side_order.txt)
hipError_t create_side_stream(hipStream_t* st) { return hipStreamCreateWithFlags(st, hipStreamNonBlocking); }

// The meter ordering needs the context's stream and fork[0] on different hardware queues (omega.h,
// omega_set_stream), and HIP deals streams out over GPU_MAX_HW_QUEUES (4) queues per process, so with
// other contexts or streams alive the two can share one: the batch path's device waits then run into
// their bound (OMEGA_EHIP), and the event-joined paths serialise (bench.py's cfg1 line measured 0.28 ms
// per call instead of 0.07 with one other context alive, tools/side_order_probe.py). Probe the pair
// (a waiter on fork[0], then a setter on the stream: the waiter sees the value only if they run at
// once); on a shared queue keep that side stream as a spare and take a new one -- the next queue -- and
// probe again (three times at most). Run at creation and on a stream switch.
// A stream already probed against the current side stream is not probed again (a caller alternating
// streams keeps its host/GPU overlap); force re-probes the pair (omega_check_queues: streams created
// since, e.g. an RCCL communicator's, may have been dealt onto the side stream's queue).
constexpr int kProbePolls = 2048;  // x ~0.3 us: the waiter's bound (paid only on a shared queue)
constexpr size_t kMaxSpare = 6;
int side_stream_check(omega_ctx* c, bool force = false) {
  if (!force && std::find(c->checked.begin(), c->checked.end(), c->stream) != c->checked.end()) return 0;
  if (!c->d_probe) {
    HIPC(c, hipMalloc(&c->d_probe, 2 * sizeof(unsigned)));
    HIPC(c, hipMemset(c->d_probe, 0, 2 * sizeof(unsigned)));
  }
  // both streams idle first: a setter queued behind earlier work on the caller's stream would read as
  // a shared queue (a rocprofv3 trace of bench.py showed probe waiters running to their bound)
  HIPC(c, hipStreamSynchronize(c->stream));
  HIPC(c, hipStreamSynchronize(c->fork[0]));
  for (int attempt = 0; attempt < 3; ++attempt) {
    const unsigned target = ++c->probe_seq;  // (w[0] holds the previous one: never equal)
    HIPC(c, launch_queue_probe(c->d_probe, target, kProbePolls, c->fork[0], c->stream));
    HIPC(c, hipStreamSynchronize(c->fork[0]));
    HIPC(c, hipStreamSynchronize(c->stream));
    unsigned r[2] = {0u, 0u};
    HIPC(c, hipMemcpy(r, c->d_probe, sizeof r, hipMemcpyDeviceToHost));
    if (r[1] == target) {
      c->queue_shared = false;
      c->checked.push_back(c->stream);
      return 0;
    }
    // a new side stream: what was checked against the old one no longer holds
    c->checked.clear();
    if (c->spare.size() >= kMaxSpare) {
      HIPC(c, hipStreamDestroy(c->spare.front()));
      c->spare.erase(c->spare.begin());
    }
    c->spare.push_back(c->fork[0]);
    c->fork[0] = nullptr;
    HIPC(c, create_side_stream(&c->fork[0]));
  }
  // No independent queue found: not an error (the device waits stay bounded, omega.h), but reported --
  // omega_check_queues returns it, and omega_last_error says why the batch path may return OMEGA_EHIP.
  // The stream is not marked checked: the next switch to it probes again.
  c->queue_shared = true;
  std::snprintf(c->err, sizeof c->err,
                "side stream: no hardware queue independent of the context's stream found after 3 attempts "
                "(more streams than GPU_MAX_HW_QUEUES?): batch-path device waits may run to their bound "
                "(OMEGA_POLL_LIMIT) and return OMEGA_EHIP");
  return 0;
}

// The per-batch work: layout 3 (enqueue_batch) where eligible, otherwise the full-chip kernels back to
// back on `s` (K-weighting first); the meter aggregates' prep and LUFS query kernels (one or two
// workgroups per channel: latency-bound) run on fork[0] beside the resolution and true-peak kernels,
// the true-peak meter after the true peaks on `s`. (Concurrent full-chip kernels lose to this: 512
// channel-frames are exactly two rounds of 256 CUs, and a CU held by another kernel pushes a third.)
// lufs_st / tp_st: the context's staging slots of a pipelined call with meters (omega_process_frames).
int enqueue_frames(omega_ctx* c, SpectralParams sp, KWeightParams kp, int W, int64_t n_frames, const float* lufs,
                   const float* tp, double* meters, hipStream_t s, bool pipe = false, float* lufs_st = nullptr,
                   float* tp_st = nullptr) {
  const bool do_tp = sp.tp_out != nullptr, do_kw = kp.lufs_out || kp.weighted_out;
  const bool do_res = sp.comb_out != nullptr || sp.res[0].mag_out || sp.res[1].mag_out || sp.res[2].mag_out ||
                      sp.res[3].mag_out;
  int mr = -1;
  const bool batch = c->layout == 3 && batch_eligible(c, sp, kp, W, do_res, s, &mr);
  // a pending meter segment goes first: folded into this batch's launch when it has an in-grid meter
  // segment of its own, else on its own
  const bool fold = pipe && batch && meters && do_tp && do_kw && n_frames > 0 && n_frames <= kChunkFrames;
  if (c->pend && !fold)
    if (int e = flush_meters(c)) return e;
  if (fold && lufs_st && tp_st) {
    // the segment and the prep read the staging slots; the caller's buffers get copies
    if (kp.lufs_out != lufs_st) kp.lufs_copy = kp.lufs_out;
    if (sp.tp_out != tp_st) sp.tp_copy = sp.tp_out;
    kp.lufs_out = lufs_st;
    sp.tp_out = tp_st;
    lufs = lufs_st;
    tp = tp_st;
  }
  if (batch) return enqueue_batch(c, sp, kp, W, n_frames, lufs, tp, meters, s, mr, do_tp, do_kw, fold);
  if (do_kw) HIPC(c, launch_kweight(W, kp, s));
  std::vector<MeterPrepParams> mc;
  if (meters) {
    mc = meter_chunks(c, lufs, tp, n_frames, meters);
    HIPC(c, hipEventRecord(c->ev_kw, s));
    HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_kw, 0));
    for (MeterPrepParams p : mc) {
      HIPC(c, launch_meter_prep(p, c->fork[0]));
      c->side_meters = true;
      p.parts = 1;
      HIPC(c, launch_meter_query(p, c->fork[0]));
      c->side_meters = true;
    }
    HIPC(c, hipEventRecord(c->ev_join[0], c->fork[0]));
  }
  if (do_res) HIPC(c, c->res_independent ? launch_mrfft_independent(sp, s) : launch_mrfft(sp, s));
  if (do_tp) HIPC(c, tp_launch(c, W, sp, s));
  for (MeterPrepParams p : mc) {
    p.parts = 2;
    HIPC(c, launch_meter_query(p, s));
  }
  if (meters) HIPC(c, hipStreamWaitEvent(s, c->ev_join[0], 0));
  return 0;
}

}  // namespace

extern "C" {

const char* omega_version(void) { return "omega-mi355x 0.3 (gfx950, ABI 3)"; }

#ifdef OMEGA_STAMPS
// Development build only (make dev): one kernel variant over n_cf channel-frames of the context's
// frames x (device memory, frame stride W, channel stride W * ... as omega_process_frames with
// frame_stride = C * W, channel_stride = W), outputs to device buffers. which: 0 the 16384-point
// resolution kernel, 2 the true-peak kernel (aux: [n_cf] true peaks), 3 the same at one workgroup per
// CU (dynamic LDS padded past half the CU's 160 KiB). (Two frames per workgroup
// through one exchange buffer -- the 16384-point resolution interleaved, and a true peak with its
// spectrum parked in L2 between phases -- measured no faster at 8192 channel-frames (true peak 614 vs
// 621 us at a shader clock of 1773 vs 1897 MHz): the extra frames in flight bought activity and the
// clock gave it back; both were deleted.)
int omega_dev_probe(omega_ctx* c, int which, const float* x, int64_t n_frames, float* comb, float* aux) {
  SpectralParams sp = spectral_params(c);
  const int W = c->cfg.frame_size;
  sp.x = x;
  sp.frame_stride = (int64_t)c->cfg.n_channels * W;
  sp.chan_stride = W;
  sp.n_cf = n_frames * c->cfg.n_channels;
  sp.comb_out = comb;
  (void)aux;
  for (int r = 0; r < kMaxRes; ++r) sp.res[r].mag_out = nullptr;
  hipError_t e = hipErrorInvalidValue;
  sp.tp_out = aux;
  float2* rot = nullptr;
  if (int r = get_rot(c, W, &rot)) return r;
  sp.rot = rot;
  if (which == 0) e = launch_mrfft_rf(16384, sp, 0, c->stream);
  if (which == 2) e = launch_truepeak_rf(16384, sp, c->stream);
  // 3: the true-peak kernel at one workgroup per CU (extra dynamic LDS), the occupancy probe
  if (which == 3) e = launch_truepeak_rf(16384, sp, c->stream, 16 * 1024);
  return e == hipSuccess ? 0 : fail(c, OMEGA_EHIP, "probe %d: %s", which, hipGetErrorString(e));
}
#endif

void omega_config_default(omega_config* cfg) try {
  std::memset(cfg, 0, sizeof *cfg);
  cfg->sample_rate = 48000;
  cfg->max_freq = 20000;
  cfg->n_res = 4;
  const omega_resolution def[4] = {{20, 200, 4096, 1024, 1.5, OMEGA_WIN_BLACKMAN},
                                   {200, 1000, 2048, 512, 1.2, OMEGA_WIN_BLACKMAN},
                                   {1000, 5000, 1024, 256, 1.0, OMEGA_WIN_BLACKMAN},
                                   {5000, 20000, 1024, 256, 1.5, OMEGA_WIN_BLACKMAN}};
  std::memcpy(cfg->res, def, sizeof def);
  cfg->apply_weighting = 1;
  cfg->target_bins = 1024;
  cfg->frame_size = 4096;
  cfg->n_channels = 1;
  cfg->gate_lufs = -70.0;
  cfg->momentary_len = 24;
  cfg->short_len = 180;
  cfg->integrated_len = 3600;
  cfg->peak_len = 60;
} catch (...) {
}

int omega_create(const omega_config* cfg, int device, omega_ctx** out) try {
  if (!cfg || !out) return OMEGA_EINVAL;
  *out = nullptr;
  omega_ctx* c = new (std::nothrow) omega_ctx();
  if (!c) return OMEGA_ENOMEM;
  int e = validate(c, cfg);
  if (e) {
    // surface the message through a throwaway context: callers read it via omega_last_error(*out)
    *out = c;
    return e;
  }
  c->cfg = *cfg;
  c->device = device;
  hipError_t he = hipSetDevice(device);
  if (he == hipSuccess) he = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (he != hipSuccess) {
    *out = c;
    return fail(c, OMEGA_EHIP, "device %d: %s", device, hipGetErrorString(he));
  }
  c->stream = c->own;
  // the one environment variable the library reads: the device-wait bound of the meter ordering
  // (a test knob: tests/test_gpu_parity.py test_meter_ordering_expiry_is_reported)
  if (const char* pl = std::getenv("OMEGA_POLL_LIMIT")) c->poll_limit = std::atoi(pl) > 0 ? std::atoi(pl) : 1;
  // (the graph-capture stream is created on the first capture: a context holds two streams --
  // the hardware has GPU_MAX_HW_QUEUES = 4 queues per process, see omega.h on the meter ordering)
  if (he == hipSuccess) he = create_side_stream(&c->fork[0]);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->ev_join[0], hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->ev_join[1], hipEventDisableTiming);
  if (he == hipSuccess) he = hipEventCreateWithFlags(&c->ev_kw, hipEventDisableTiming);
  if (he != hipSuccess) {
    *out = c;
    return fail(c, OMEGA_EHIP, "streams/events: %s", hipGetErrorString(he));
  }
  e = build_twiddles(c);
  if (!e) e = build_spectral_tables(c);
  if (!e) e = build_meter_state(c);
  if (!e) e = side_stream_check(c);
  *out = c;
  return e;
} catch (...) {
  return guard_fail(out ? *out : nullptr);
}

int omega_vu_reset(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  c->vu_total = 0;
  if (!c->d_vu_st[0]) return 0;
  HIPC(c, hipSetDevice(c->device));
  const int C = c->cfg.n_channels;
  std::vector<double> st((size_t)C * 3);
  for (int i = 0; i < C; ++i) {  // vu_meters.py:33-42: display and peak at -60, hold time 0
    st[i * 3] = -60.0;
    st[i * 3 + 1] = -60.0;
    st[i * 3 + 2] = 0.0;
  }
  for (int b = 0; b < 2; ++b)
    HIPC(c, hipMemcpyAsync(c->d_vu_st[b], st.data(), st.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_vu_update(omega_ctx* c, const void* x, int32_t f64, int64_t n_updates, int32_t chunk, int64_t update_stride,
                    int64_t channel_stride, const double* dt, double* out, int mem) try {
  if (!c || !out || !dt) return OMEGA_EINVAL;
  if (!x || n_updates < 0 || chunk < 1) return fail(c, OMEGA_EINVAL, "vu update: bad input layout");
  if (n_updates == 0) return 0;
  HIPC(c, hipSetDevice(c->device));
  const int C = c->cfg.n_channels;
  const int64_t Wv = (int64_t)(0.3 * c->cfg.sample_rate);  // vu_meters.py:28-30
  if (!c->d_vu_st[0]) {
    for (int b = 0; b < 2; ++b) {
      int e = dalloc(c, &c->d_vu_hist[b], (size_t)C * Wv);
      if (!e) e = dalloc(c, &c->d_vu_st[b], (size_t)C * 3);
      if (e) return e;
    }
    if (int e = omega_vu_reset(c)) return e;
  }
  if (int e = grow(c, &c->d_vu_ms, &c->vu_ms_cap, n_updates * C)) return e;
  std::vector<HostOut> outs;
  const void* dx = x;
  const double* ddt = dt;
  double* dout = out;
  if (mem == OMEGA_MEM_HOST) {
    const size_t el = f64 ? 8 : 4;
    const size_t span = (size_t)((n_updates - 1) * update_stride + (C - 1) * channel_stride + chunk);
    int e = stage_in(c, 0, x, span * el, &dx);
    if (!e) e = stage_in(c, 1, dt, (size_t)n_updates * sizeof(double), reinterpret_cast<const void**>(&ddt));
    if (!e) e = stage_out(c, 2, out, (size_t)n_updates * C * 3, outs, &dout);
    if (e) return e;
  }
  VuParams p{};
  p.x = dx;
  p.f64 = f64 ? 1 : 0;
  p.n = n_updates;
  p.chunk = chunk;
  p.frame_stride = update_stride;
  p.channel_stride = channel_stride;
  p.C = C;
  p.dt = ddt;
  const int a = c->vu_cur, b = a ^ 1;
  p.hist_in = c->d_vu_hist[a];
  p.hist_out = c->d_vu_hist[b];
  p.hist_n = std::min(c->vu_total, Wv);
  p.Wv = Wv;
  p.ms = c->d_vu_ms;
  p.st_in = c->d_vu_st[a];
  p.st_out = c->d_vu_st[b];
  p.out = dout;
  HIPC(c, launch_vu(p, c->stream));
  c->vu_cur = b;
  c->vu_total += n_updates * chunk;
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

// Savitzky-Golay (21, 3) weights of scipy.signal.savgol_filter's 'interp' mode: the least-squares
// cubic through the 21 samples of a window evaluated at window position p (p = 10: the interior
// convolution; p < 10 / p > 10: the first / last 10 outputs of a frame), in centred, scaled
// coordinates u = (t - 10) / 10 so that the 4 x 4 normal equations stay well conditioned.
static void savgol_21_3(double W[21][21]) {
  double A[21][4], G[4][4] = {};
  for (int t = 0; t < 21; ++t)
    for (int j = 0; j < 4; ++j) A[t][j] = std::pow((t - 10) / 10.0, j);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int t = 0; t < 21; ++t) G[i][j] += A[t][i] * A[t][j];
  double Gi[4][4];  // Gauss-Jordan inverse
  double M[4][8];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) M[i][j] = j < 4 ? G[i][j] : (j - 4 == i ? 1.0 : 0.0);
  for (int c = 0; c < 4; ++c) {
    int pv = c;
    for (int r = c + 1; r < 4; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[pv][c])) pv = r;
    for (int j = 0; j < 8; ++j) std::swap(M[c][j], M[pv][j]);
    const double d = M[c][c];
    for (int j = 0; j < 8; ++j) M[c][j] /= d;
    for (int r = 0; r < 4; ++r)
      if (r != c) {
        const double f = M[r][c];
        for (int j = 0; j < 8; ++j) M[r][j] -= f * M[c][j];
      }
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) Gi[i][j] = M[i][j + 4];
  for (int p = 0; p < 21; ++p) {
    double v[4], q[4] = {};
    for (int j = 0; j < 4; ++j) v[j] = std::pow((p - 10) / 10.0, j);
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 4; ++i) q[j] += v[i] * Gi[i][j];
    for (int t = 0; t < 21; ++t) {
      double w = 0.0;
      for (int j = 0; j < 4; ++j) w += q[j] * A[t][j];
      W[p][t] = w;
    }
  }
}

int omega_transients(omega_ctx* c, const void* x, int32_t f64, int64_t n_frames, int32_t n, int64_t frame_stride,
                     double* out, int mem) try {
  if (!c || !out) return OMEGA_EINVAL;
  if (!x || n_frames < 0 || frame_stride < n) return fail(c, OMEGA_EINVAL, "transients: bad frame layout");
  if (n < 64) return fail(c, OMEGA_EINVAL, "transients: frame length %d below 64 (transient.py:21)", n);
  const bool pow2 = n <= 8192 && !(n & (n - 1));
  if (n_frames == 0) return 0;
  HIPC(c, hipSetDevice(c->device));
  if (!c->d_sg) {
    double W[21][21];
    savgol_21_3(W);
    std::vector<double> v(&W[0][0], &W[0][0] + 21 * 21);
    if (int e = upload(c, &c->d_sg, v)) return e;
  }
  TransientParams p{};
  if (!pow2) {  // other lengths: the complex mixed-radix transform (transient_any_kernel)
    auto ia = c->tr_any.find(n);
    if (ia == c->tr_any.end()) {
      std::vector<int> rad;
      int r = n;
      while (r % 4 == 0) rad.push_back(4), r /= 4;
      for (int fct : {2, 3, 5, 7})
        while (r % fct == 0) rad.push_back(fct), r /= fct;
      for (int fct = 11; (int64_t)fct * fct <= r; fct += 2)
        while (r % fct == 0) rad.push_back(fct), r /= fct;
      if (r > 1) rad.push_back(r);
      if ((int)rad.size() > kTrMaxStages) return fail(c, OMEGA_EUNSUP, "transients: length %d: too many factors", n);
      std::vector<double2> tw(n);
      for (int m = 0; m < n; ++m) tw[m] = make_double2(std::cos(2 * M_PI * m / n), -std::sin(2 * M_PI * m / n));
      double2* d = nullptr;
      if (int e = upload(c, &d, tw)) return e;
      ia = c->tr_any.emplace(n, std::make_pair(rad, d)).first;
    }
    p.n_stages = (int)ia->second.first.size();
    for (int i = 0; i < p.n_stages; ++i) p.radix[i] = ia->second.first[i];
    p.twn = ia->second.second;
  }
  // frames too long for LDS work in global buffers (2 n double2 per frame), launched in slices of
  // frames whose buffers stay within 64 MiB
  int64_t per = n_frames;
  if (!pow2 && (size_t)n * 2 * sizeof(double2) > 160 * 1024 - 64) {
    per = std::max<int64_t>(1, std::min<int64_t>(n_frames, (int64_t)(64 << 20) / (2 * (int64_t)n * (int64_t)sizeof(double2))));
    if (int e = grow(c, &c->d_tr_scratch, &c->tr_scratch_cap, per * 2 * (int64_t)n)) return e;
    p.scratch = c->d_tr_scratch;
  }
  auto it = c->tr_tw.find(pow2 ? n : 0);
  if (pow2 && it == c->tr_tw.end()) {
    const int K = n / 2;
    std::vector<double2> t1(K / 2 > 0 ? K / 2 : 1), t2(K + 1);
    for (int m = 0; m < K / 2; ++m) t1[m] = make_double2(std::cos(2 * M_PI * m / K), -std::sin(2 * M_PI * m / K));
    for (int q = 0; q <= K; ++q) t2[q] = make_double2(std::cos(2 * M_PI * q / n), -std::sin(2 * M_PI * q / n));
    double2 *d1 = nullptr, *d2 = nullptr;
    int e = upload(c, &d1, t1);
    if (!e) e = upload(c, &d2, t2);
    if (e) return e;
    it = c->tr_tw.emplace(n, std::make_pair(d1, d2)).first;
  }
  std::vector<HostOut> outs;
  const void* dx = x;
  double* dout = out;
  if (mem == OMEGA_MEM_HOST) {
    const size_t el = f64 ? 8 : 4;
    int e = stage_in(c, 0, x, (size_t)((n_frames - 1) * frame_stride + n) * el, &dx);
    if (!e) e = stage_out(c, 1, out, (size_t)n_frames * kTransientCols, outs, &dout);
    if (e) return e;
  }
  p.f64 = f64 ? 1 : 0;
  p.n = n;
  p.frame_stride = frame_stride;
  p.sg = c->d_sg;
  p.fs = c->cfg.sample_rate;
  if (pow2) {
    p.x = dx;
    p.n_frames = n_frames;
    p.out = dout;
    p.tw = it->second.first;
    p.tw2 = it->second.second;
    HIPC(c, launch_transients(p, c->stream));
  } else {
    const size_t el = f64 ? 8 : 4;
    for (int64_t f0 = 0; f0 < n_frames; f0 += per) {
      TransientParams q = p;
      q.x = static_cast<const char*>(dx) + (size_t)(f0 * frame_stride) * el;
      q.n_frames = std::min(per, n_frames - f0);
      q.out = dout + f0 * kTransientCols;
      HIPC(c, launch_transients_any(q, c->stream));
    }
  }
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_drum_reset(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  if (!c->drum_bins) return 0;
  HIPC(c, hipSetDevice(c->device));
  for (int b = 0; b < 2; ++b) {
    HIPC(c, hipMemsetAsync(c->d_dlen[b], 0, kDrumBands * sizeof(int), c->stream));
    HIPC(c, hipMemsetAsync(c->d_dpos[b], 0, sizeof(long long), c->stream));
  }
  HIPC(c, hipStreamSynchronize(c->stream));
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_drum_features(omega_ctx* c, const float* mag, int64_t n_frames, int32_t n_bins, int64_t mag_stride,
                        double sensitivity, double* out, int mem) try {
  if (!c || !out) return OMEGA_EINVAL;
  if (!mag || n_frames < 0 || n_bins < 2 || mag_stride < n_bins)
    return fail(c, OMEGA_EINVAL, "drum features: bad magnitude layout (n_bins %d, stride %lld)", n_bins,
                (long long)mag_stride);
  if (c->drum_bins && c->drum_bins != n_bins)
    return fail(c, OMEGA_EINVAL, "drum features: the stream has %d bins per frame, got %d (omega_drum_reset "
                "does not change it; create another context)", c->drum_bins, n_bins);
  if (n_frames == 0) return 0;
  HIPC(c, hipSetDevice(c->device));
  if (!c->drum_bins) {
    for (int b = 0; b < 2; ++b) {
      int e = dalloc(c, &c->d_dprev[b], (size_t)n_bins);
      if (!e) e = dalloc(c, &c->d_dhist[b], (size_t)kDrumBands * kDrumHist);
      if (!e) e = dalloc(c, &c->d_dlen[b], kDrumBands);
      if (!e) e = dalloc(c, &c->d_dpos[b], 1);
      if (e) return e;
    }
    c->drum_bins = n_bins;
    const int e = omega_drum_reset(c);
    if (e) return e;
  }
  if (int e = grow(c, &c->d_dflux, &c->dflux_cap, n_frames * kDrumBands)) return e;
  std::vector<HostOut> outs;
  const float* dm = mag;
  double* dout = out;
  if (mem == OMEGA_MEM_HOST) {
    int e = stage_in(c, 0, mag, (size_t)((n_frames - 1) * mag_stride + n_bins) * sizeof(float),
                     reinterpret_cast<const void**>(&dm));
    if (!e) e = stage_out(c, 1, out, (size_t)n_frames * kDrumCols, outs, &dout);
    if (e) return e;
  }
  // drum_detection.py: bins int(f * len / nyquist) (:86-96, :240-259, :218-219), numpy slices clamp
  const double fs = c->cfg.sample_rate, ny = fs / 2;
  const double bands[kDrumBands][2] = {{20, 60}, {60, 120}, {2000, 5000}, {150, 400}, {400, 1000}, {2000, 8000},
                                       {8000, 15000}};
  const double mult[kDrumBands] = {2.8, 2.8, 2.8, 2.5, 2.3, 2.0, 0.0};  // :78, :295, :300, :305
  DrumParams p{};
  p.mag = dm;
  p.n = n_frames;
  p.stride = mag_stride;
  p.n_bins = n_bins;
  auto bin = [&](double f) { return std::min(n_bins, (int)(f * n_bins / ny)); };
  for (int b = 0; b < kDrumBands; ++b) {
    p.bs[b] = bin(bands[b][0]);
    p.be[b] = std::max(p.bs[b], bin(bands[b][1]));
    p.mult[b] = (float)(sensitivity * mult[b]);
  }
  p.cs = bin(150.0);
  p.ce = std::max(p.cs, bin(15000.0));
  p.fstep = 1.0 / ((2.0 * n_bins - 1.0) * (1.0 / fs));  // np.fft.rfftfreq(2 n - 1, 1 / fs) spacing
  const int a = c->drum_cur, b = a ^ 1;
  p.prev_in = c->d_dprev[a];
  p.prev_out = c->d_dprev[b];
  p.hist_in = c->d_dhist[a];
  p.hist_out = c->d_dhist[b];
  p.len_in = c->d_dlen[a];
  p.len_out = c->d_dlen[b];
  p.pos_in = c->d_dpos[a];
  p.pos_out = c->d_dpos[b];
  p.flux = c->d_dflux;
  p.out = dout;
  HIPC(c, launch_drum(p, c->stream));
  c->drum_cur = b;
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

// The leaves of numpy's pairwise float32 sum over n elements (numpy/_core/src/umath/loops_utils.h.src:
// up to 128 elements a leaf, above that halves split at a multiple of 8 below n / 2), in the
// recursion's depth-first order, as offset | length << 16 -- the table post_frame_kernel's range means
// read instead of walking the recursion per lane (numpy_emul.hpp np_leaf_sums_tab)
static void np_leaves(int off, int n, int depth, std::vector<unsigned>& out) {
  if (depth == 0 || n <= 128) {
    out.push_back((unsigned)off | (unsigned)n << 16);
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  np_leaves(off, n2, depth - 1, out);
  np_leaves(off + n2, n - n2, depth - 1, out);
}

int omega_post_configure(omega_ctx* c, int32_t n_bins, const double* curve, const uint8_t* bass,
                         const float* comp_instr, const float* comp_vocal, const float* vocal_sup,
                         const int32_t* ranges, int32_t p_lo, int32_t p_hi, float p_gamma,
                         const int32_t* band_start, const int32_t* band_end, const double* band_smooth,
                         int32_t n_bands) try {
  if (!c) return OMEGA_EINVAL;
  if (n_bins < 1 || n_bins > kPostMaxBins || n_bands < 0 || n_bands > kPostMaxBands || !curve || !bass ||
      !comp_instr || !comp_vocal || !vocal_sup || !ranges || (n_bands && (!band_start || !band_end || !band_smooth)))
    return fail(c, OMEGA_EINVAL, "post configure: bad tables (n_bins %d, n_bands %d)", n_bins, n_bands);
  if (p_lo < 0 || p_hi < p_lo || p_hi > p_lo + 1 || p_hi >= n_bins)
    return fail(c, OMEGA_EINVAL, "post configure: percentile ranks %d, %d outside %d bins", p_lo, p_hi, n_bins);
  for (int b = 0; b < n_bands; ++b)
    if (band_start[b] < 0 || band_start[b] >= n_bins || band_end[b] > n_bins || band_end[b] < band_start[b])
      return fail(c, OMEGA_EINVAL, "post configure: band %d [%d, %d) outside %d bins", b, band_start[b],
                  band_end[b], n_bins);
  std::vector<EmaCoef> coef((size_t)n_bands);
  for (int b = 0; b < n_bands; ++b) {
    const double f = band_smooth[b];
    if (!(f >= 0.0 && f <= 1.0)) return fail(c, OMEGA_EINVAL, "post configure: band %d smoothing factor %g outside [0, 1]", b, f);
    coef[b] = EmaCoef{f, 1.0 - f, (float)f, (float)(1.0 - f)};
  }
  HIPC(c, hipSetDevice(c->device));
  PostParams p{};
  p.T = n_bins;
  p.nb = n_bands;
  p.be = ranges[0];
  p.vs = ranges[1];
  p.ve = ranges[2];
  p.hs = ranges[3];
  p.p_lo = p_lo;
  p.p_hi = p_hi;
  p.p_g = p_gamma;
  auto up = [&](auto** d, const auto* h, size_t n) {
    int e = dalloc(c, d, n);
    if (!e && n) {
      const hipError_t he = hipMemcpy(*d, h, n * sizeof(**d), hipMemcpyHostToDevice);
      if (he != hipSuccess) e = fail(c, OMEGA_EHIP, "post configure: %s", hipGetErrorString(he));
    }
    return e;
  };
  double* dc = nullptr;
  unsigned char* db = nullptr;
  float *d0 = nullptr, *d1 = nullptr, *dv = nullptr;
  EmaCoef* dsf = nullptr;
  int *dbs = nullptr, *dbe = nullptr;
  int e = up(&dc, curve, (size_t)n_bins);
  if (!e) e = up(&db, bass, (size_t)n_bins);
  if (!e) e = up(&d0, comp_instr, (size_t)n_bins);
  if (!e) e = up(&d1, comp_vocal, (size_t)n_bins);
  if (!e) e = up(&dv, vocal_sup, (size_t)n_bins);
  if (!e) e = up(&dbs, band_start, (size_t)n_bands);
  if (!e) e = up(&dbe, band_end, (size_t)n_bands);
  if (!e) e = up(&dsf, coef.data(), (size_t)n_bands);
  // the content ranges' leaf tables: [w][0] the count (at most 17 for 2048 bins), [w][1 ..] the leaves
  std::vector<unsigned> leaf_tab(4 * 32, 0u);
  const int rn[4] = {p.be, p.ve - p.vs, n_bins - p.hs, n_bins};
  for (int w = 0; w < 4; ++w) {
    std::vector<unsigned> lv;
    np_leaves(0, std::min(std::max(rn[w], 0), n_bins), 6, lv);  // (a range past the bins is not read)
    leaf_tab[32 * w] = (unsigned)lv.size();
    for (size_t i = 0; i < lv.size() && i < 31; ++i) leaf_tab[32 * w + 1 + i] = lv[i];
  }
  unsigned* dlt = nullptr;
  if (!e) e = up(&dlt, leaf_tab.data(), leaf_tab.size());
  if (!e) e = dalloc(c, &p.prev, (size_t)std::max(n_bands, 1) * 2);  // two EMA state buffers
  if (!e) e = dalloc(c, &p.has_prev, 4);
  if (e) return e;
  p.prev_out = p.prev + std::max(n_bands, 1);
  p.has_prev_out = p.has_prev + 2;
  p.curve = dc;
  p.bass = db;
  p.comp[0] = d0;
  p.comp[1] = d1;
  p.vsup = dv;
  p.bs = dbs;
  p.bend = dbe;
  p.sf = dsf;
  p.leaf_tab = dlt;
  c->post = p;
  return omega_post_reset(c);
} catch (...) {
  return guard_fail(c);
}

int omega_post_reset(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  if (!c->post.T) return 0;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemsetAsync(std::min(c->post.has_prev, c->post.has_prev_out), 0, 4 * sizeof(int), c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_post_process(omega_ctx* c, const float* spectra, int64_t n_frames, int64_t stride, int32_t flags,
                       float bass_boost, float* spectrum_out, double* bands_out, int32_t* content_out) try {
  if (!c) return OMEGA_EINVAL;
  if (!c->post.T) return fail(c, OMEGA_EINVAL, "post process: omega_post_configure first");
  if (n_frames < 0 || stride < c->post.T || !spectra || !spectrum_out || (c->post.nb && !bands_out) ||
      n_frames > 0x7FFFFFFF)
    return fail(c, OMEGA_EINVAL, "post process: bad layout (n %lld, stride %lld, %d bins)", (long long)n_frames,
                (long long)stride, c->post.T);
  if (n_frames == 0) return 0;
  HIPC(c, hipSetDevice(c->device));
  PostParams p = c->post;
  p.in = spectra;
  p.n = n_frames;
  p.stride = stride;
  p.flags = flags;
  p.bass_boost = bass_boost;
  p.spec_out = spectrum_out;
  p.band_out = bands_out;
  p.content_out = content_out;
  // scratch: the raw band rows (+ the EMA's spare rows: post.hip post_ema_kernel), the per-frame dtype
  // flags, then (8-byte aligned) the EMA chunks' warm-up values at their boundaries and end values
  const int64_t rows = n_frames + kEmaSpareRows, nch = (n_frames + 63) / 64;
  const int64_t pre_off = (rows * (c->post.nb + 1) + 1) / 2 * 2;
  if (c->post.nb) {
    if (int e = grow(c, &c->d_post_raw, &c->post_raw_cap, pre_off + 4 * nch * c->post.nb + 4)) return e;
  }
  p.band_raw = c->d_post_raw;
  p.frame64 = reinterpret_cast<int*>(c->d_post_raw + rows * c->post.nb);
  p.ema_pre = reinterpret_cast<double*>(c->d_post_raw + pre_off);
  p.ema_end = p.ema_pre + nch * c->post.nb;
  HIPC(c, launch_post(p, c->stream));
  if (c->post.nb) {  // the EMA wrote the other state buffer: it is the next call's input
    std::swap(c->post.prev, c->post.prev_out);
    std::swap(c->post.has_prev, c->post.has_prev_out);
  }
  return 0;
} catch (...) {
  return guard_fail(c);
}

void omega_destroy(omega_ctx* c) try {
  if (!c) return;
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->pend && !flush_meters(c)) (void)hipStreamSynchronize(c->stream);  // (the last call's meters)
  if (c->own) (void)hipStreamSynchronize(c->own);
  if (c->fork[0]) (void)hipStreamSynchronize(c->fork[0]);
  for (void* p : c->allocs) (void)hipFree(p);
  for (auto& kv : c->chroma_mats) (void)hipFree(kv.second.first);
  for (void* q : {(void*)c->ctab.w4, (void*)c->ctab.w1, (void*)c->ctab.perm, (void*)c->ctab.goff,
                  (void*)c->ctab.rec})
    if (q) (void)hipFree(q);
  for (DevBuf& b : c->stage)
    if (b.p) (void)hipFree(b.p);
  for (DevBuf& b : c->pin)
    if (b.p) (void)hipHostFree(b.p);
  if (c->oarena.p) (void)hipFree(c->oarena.p);
  if (c->oarena_pin.p) (void)hipHostFree(c->oarena_pin.p);
  if (c->zc_pin.p) (void)hipHostFree(c->zc_pin.p);
  drop_graphs(c);
  if (c->h_err) (void)hipHostFree(c->h_err);
  if (c->d_tail) (void)hipFree(c->d_tail);
  if (c->d_mirror) (void)hipFree(c->d_mirror);
  for (hipStream_t st : {c->cap, c->fork[0]})
    if (st) (void)hipStreamDestroy(st);
  for (hipStream_t st : c->spare) (void)hipStreamDestroy(st);
  if (c->d_probe) (void)hipFree(c->d_probe);
  for (hipEvent_t ev : {c->ev_fork, c->ev_join[0], c->ev_join[1], c->ev_kw})
    if (ev) (void)hipEventDestroy(ev);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
} catch (...) {
}

const char* omega_last_error(const omega_ctx* c) { return c ? c->err : "null context"; }

int omega_set_stream(omega_ctx* c, void* s) try {
  if (!c) return OMEGA_EINVAL;
  const hipStream_t ns = static_cast<hipStream_t>(s);  // NULL = the null (default) stream, e.g. torch's
  if (ns != c->stream) {
    if (c->pend) {  // (a pending meter segment runs on its batch's stream)
      HIPC(c, hipSetDevice(c->device));
      if (int e = flush_meters(c)) return e;
    }
    // The work already enqueued on the old stream -- a batch's meter segment still reading the
    // per-context prep scratch and history, a query kernel -- must finish before the next call's work:
    // on one stream that is stream order, and the next meter prep on fork[0] waits for the next
    // batch's K-weighting count, i.e. for a batch that started after the previous one ended. Across a
    // stream switch nothing orders them, so the new stream and fork[0] wait once for the old stream.
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipEventRecord(c->ev_fork, c->stream));
    HIPC(c, hipStreamWaitEvent(ns, c->ev_fork, 0));
    HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_fork, 0));
    c->stream = ns;
    if (int e = side_stream_check(c)) return e;
  }
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_check_queues(omega_ctx* c, int* shared) try {
  if (!c) return OMEGA_EINVAL;
  HIPC(c, hipSetDevice(c->device));
  if (c->pend) {  // (the probe synchronises both streams; a pending segment launches first)
    if (int e = flush_meters(c)) return e;
  }
  if (int e = side_stream_check(c, true)) return e;
  if (shared) *shared = c->queue_shared ? 1 : 0;
  return 0;
} catch (...) {
  return guard_fail(c);
}

void* omega_get_stream(const omega_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int omega_get_config(const omega_ctx* c, omega_config* cfg, int* device) {
  if (!c) return OMEGA_EINVAL;
  if (cfg) *cfg = c->cfg;
  if (device) *device = c->device;
  return 0;
}

int omega_set_graphs(omega_ctx* c, int enable) try {
  if (!c) return OMEGA_EINVAL;
  if (c->pend) {
    HIPC(c, hipSetDevice(c->device));
    if (int e = flush_meters(c)) return e;
  }
  c->use_graph = (enable & 1) != 0;
  // bits 1-2: 0 default (one batch launch where eligible), else the full-chip kernels back to back with
  // the meters on a side stream
  c->layout = ((enable >> 1) & 3) ? 2 : 3;
  drop_graphs(c);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_synchronize(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  if (c->pend) {
    HIPC(c, hipSetDevice(c->device));
    if (int e = flush_meters(c)) return e;
  }
  HIPC(c, hipStreamSynchronize(c->stream));
  return check_device_err(c);
} catch (...) {
  return guard_fail(c);
}

int omega_meter_reset(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  if (int e = flush_meters(c)) return e;  // (the pending segment reads the state being reset)
  // a meter prep on the side stream may still be writing the next state after its count-in
  if (c->fork[0]) HIPC(c, hipStreamSynchronize(c->fork[0]));
  const int C = c->cfg.n_channels;
  for (int b = 0; b < 2; ++b) {
    HIPC(c, hipMemsetAsync(c->d_nl[b], 0, C * sizeof(int), c->stream));
    HIPC(c, hipMemsetAsync(c->d_nt[b], 0, C * sizeof(int), c->stream));
    HIPC(c, hipMemsetAsync(c->d_ns[b], 0, C * sizeof(int), c->stream));
    HIPC(c, hipMemsetAsync(c->d_t0[b], 0, C * sizeof(uint32_t), c->stream));
  }
  HIPC(c, hipStreamSynchronize(c->stream));
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_process_frames(omega_ctx* c, const float* x, int64_t n_frames, int64_t frame_stride, int64_t channel_stride,
                         const omega_outputs* out, int mem) try {
  if (!c || !out) return OMEGA_EINVAL;
  if (!x || n_frames < 0) return fail(c, OMEGA_EINVAL, "null input or negative frame count");
  if (int e = check_device_err(c)) return e;
  if (n_frames == 0) return 0;
  const int C = c->cfg.n_channels, W = c->cfg.frame_size, T = c->cfg.target_bins;
  const int64_t ncf = n_frames * C;
  if ((frame_stride & 1) || (channel_stride & 1))
    return fail(c, OMEGA_EINVAL, "frame_stride and channel_stride must be even (8-byte aligned frames)");
  if (ncf > 0x7FFFFFFF) return fail(c, OMEGA_EINVAL, "too many channel-frames");
  HIPC(c, hipSetDevice(c->device));
  // meter pipelining applies to direct device-memory calls; any other call runs a pending meter
  // segment first (before its staging buffers are touched)
  const bool pipe = c->pipe && mem == OMEGA_MEM_DEVICE && !c->use_graph;
  if (!pipe)
    if (int e = flush_meters(c)) return e;
  SpectralParams sp = spectral_params(c);
  sp.frame_stride = frame_stride;
  sp.chan_stride = channel_stride;
  sp.n_cf = ncf;
  std::vector<HostOut> outs;
  const float* dx = x;
  float* tp = out->true_peak_db;
  float* lufs = out->lufs_inst;
  double* meters = out->meters;
  float* comb = out->combined;
  float* weighted = out->weighted;
  float* mags[kMaxRes] = {};
  const size_t span = (size_t)((n_frames - 1) * frame_stride + (C - 1) * channel_stride + W);
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    // when every kernel of the call only stores its outputs, small ones go straight to page-locked
    // memory: not with meters (the meter path's true peaks are re-read across workgroups) nor with combine
    // targets owned by several resolutions (their o[t] += v reads back across kernels): device staging
    c->zc_ok = !meters && (!comb || c->res_independent);
    e = stage_in(c, 0, x, span * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 1, comb, ncf * T, outs, &comb);
    if (!e) e = stage_out(c, 2, out->lufs_inst, ncf, outs, &lufs);
    if (!e) e = stage_out(c, 3, out->true_peak_db, ncf, outs, &tp);
    if (!e) e = stage_out(c, 4, out->meters, ncf * 5, outs, &meters);
    if (!e) e = stage_out(c, 5, out->weighted, ncf * W, outs, &weighted);
    for (int r = 0; r < c->cfg.n_res && !e; ++r)
      e = stage_out(c, 6 + r, out->mag[r], ncf * (c->cfg.res[r].fft_size / 2 + 1), outs, &mags[r]);
    if (e) return e;
  } else {
    for (int r = 0; r < c->cfg.n_res; ++r) mags[r] = out->mag[r];
    if (!aligned8(x)) return fail(c, OMEGA_EINVAL, "input must be 8-byte aligned");
  }
  // meters need the instantaneous values even when the caller does not ask for them. Pipelined, the
  // meter prep and the deferred meter segment read them during the next call, so they read the
  // context's staging slots (two sets in turn) and never the caller's buffers, which the next call may
  // overwrite (the usual preallocated outputs): enqueue_frames points the batch's K-weighting and
  // true-peak roles at the slots and hands them the caller's buffers as copies.
  const int sl = pipe ? 2 * c->stage_par : 0;
  if (pipe && meters) c->stage_par ^= 1;
  float* lufs_st = nullptr;
  float* tp_st = nullptr;
  if (meters && (pipe || !lufs)) {
    e = stage_buf(c, 10 + sl, ncf * sizeof(float), reinterpret_cast<void**>(&lufs_st));
    if (e) return e;
    if (!lufs) lufs = lufs_st;
  }
  if (meters && (pipe || !tp)) {
    e = stage_buf(c, 11 + sl, ncf * sizeof(float), reinterpret_cast<void**>(&tp_st));
    if (e) return e;
    if (!tp) tp = tp_st;
  }
  sp.x = dx;
  sp.comb_out = comb;
  sp.tp_out = tp;
  for (int r = 0; r < c->cfg.n_res; ++r) sp.res[r].mag_out = mags[r];
  BiquadTab* tabs = nullptr;
  if (lufs || weighted) {
    e = get_kw_tab(c, W, &tabs);
    if (e) return e;
  }
  KWeightParams kp{dx, frame_stride, channel_stride, C, ncf, tabs, tabs ? tabs + 1 : nullptr, lufs, weighted, 0};
  if (mem == OMEGA_MEM_DEVICE && c->use_graph) {
    // replay a captured graph of this exact call (pointers, sizes, meter-state parity), capturing it on
    // first use: removes the per-launch host cost and runs the three branches concurrently
    const std::vector<uint64_t> key = {(uint64_t)dx, (uint64_t)n_frames, (uint64_t)frame_stride,
                                       (uint64_t)channel_stride, (uint64_t)comb, (uint64_t)lufs, (uint64_t)tp,
                                       (uint64_t)meters, (uint64_t)weighted, (uint64_t)mags[0], (uint64_t)mags[1],
                                       (uint64_t)mags[2], (uint64_t)mags[3], (uint64_t)c->cur};
    hipGraphExec_t exec = nullptr;
    for (auto& g : c->graphs)
      if (g.key == key) exec = g.exec;
    if (!exec) {
      if (c->graphs.size() >= 16) {
        for (auto& g : c->graphs) {
          (void)hipGraphExecDestroy(g.exec);
          (void)hipGraphDestroy(g.graph);
        }
        c->graphs.clear();
      }
      const int cur0 = c->cur;
      if (!c->cap) HIPC(c, hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking));
      HIPC(c, hipStreamBeginCapture(c->cap, hipStreamCaptureModeThreadLocal));
      e = enqueue_frames(c, sp, kp, W, n_frames, lufs, tp, meters, c->cap);
      hipGraph_t graph = nullptr;
      const hipError_t ce = hipStreamEndCapture(c->cap, &graph);
      if (e) return e;
      if (ce != hipSuccess) return fail(c, OMEGA_EHIP, "graph capture: %s", hipGetErrorString(ce));
      HIPC(c, hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      c->graphs.push_back({key, graph, exec});
      c->cur = cur0;  // capture advanced the parity; the replay below advances it for real
    }
    HIPC(c, hipGraphLaunch(exec, c->stream));
    if (meters) c->cur ^= (int)(((n_frames + kChunkFrames - 1) / kChunkFrames) & 1);
    return 0;
  }
  e = enqueue_frames(c, sp, kp, W, n_frames, lufs, tp, meters, c->stream, pipe, lufs_st, tp_st);
  if (e) {
    if (pipe && meters) c->stage_par ^= 1;  // (a still-pending segment reads the slots of the other parity)
    return e;
  }
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_set_meter_pipelining(omega_ctx* c, int enable) try {
  if (!c) return OMEGA_EINVAL;
  if (!enable && c->pend) {
    HIPC(c, hipSetDevice(c->device));
    if (int e = flush_meters(c)) return e;
  }
  c->pipe = enable != 0;
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_flush_meters(omega_ctx* c) try {
  if (!c) return OMEGA_EINVAL;
  if (!c->pend) return 0;
  HIPC(c, hipSetDevice(c->device));
  return flush_meters(c);
} catch (...) {
  return guard_fail(c);
}

int omega_process_stream(omega_ctx* c, const float* x, int64_t n_samples, int32_t hop, int64_t channel_stride,
                         const omega_outputs* out, int mem, int64_t* n_frames_out) try {
  if (!c) return OMEGA_EINVAL;
  if (n_frames_out) *n_frames_out = 0;
  if (hop < 1 || n_samples < 0) return fail(c, OMEGA_EINVAL, "hop must be >= 1 and n_samples >= 0");
  const int W = c->cfg.frame_size;
  const int64_t nf = n_samples < W ? 0 : (n_samples - W) / hop + 1;
  if (n_frames_out) *n_frames_out = nf;
  return omega_process_frames(c, x, nf, hop, channel_stride, out, mem);
} catch (...) {
  return guard_fail(c);
}

int omega_combine(omega_ctx* c, const float* const* mags, int64_t n_cf, float* out, int mem) try {
  if (!c || !mags || !out) return OMEGA_EINVAL;
  if (n_cf <= 0) return n_cf == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  const int T = c->cfg.target_bins;
  CombineParams p{};
  std::vector<HostOut> outs;
  float* dout = out;
  int e = 0;
  for (int r = 0; r < c->cfg.n_res; ++r) {
    p.nbins[r] = c->cfg.res[r].fft_size / 2 + 1;
    p.cw[r] = (float)c->cfg.res[r].weight;
    if (!mags[r]) continue;
    if (mem == OMEGA_MEM_HOST) {
      const void* d = nullptr;
      e = stage_in(c, 20 + r, mags[r], (size_t)n_cf * p.nbins[r] * sizeof(float), &d);
      if (e) return e;
      p.mag[r] = static_cast<const float*>(d);
    } else {
      p.mag[r] = mags[r];
    }
  }
  if (mem == OMEGA_MEM_HOST) {
    e = stage_out(c, 24, out, (size_t)n_cf * T, outs, &dout);
    if (e) return e;
  }
  p.n_cf = n_cf;
  p.T = T;
  p.own_off = c->d_own_off;
  p.own_rj = c->d_own_rj;
  p.own_frac = c->d_own_frac;
  p.out = dout;
  HIPC(c, launch_combine(p, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_true_peak(omega_ctx* c, const float* x, int64_t n, int32_t m, float* out_db, int mem) try {
  return omega_true_peak_os(c, x, n, m, 4, out_db, mem);
} catch (...) {
  return guard_fail(c);
}

// Plan of the any-length transform: radices (4s, then 2, 3, 5, 7, then the remaining primes) and the
// tables e^{-2 pi i m / N}, e^{2 pi i m / (4N)} in float64 rounded to float32
int get_any_plan(omega_ctx* c, int N, omega_ctx::AnyPlan** out) {
  auto it = c->any_plans.find(N);
  if (it == c->any_plans.end()) {
    omega_ctx::AnyPlan pl;
    int r = N;
    while (r % 4 == 0) pl.radix.push_back(4), r /= 4;
    for (int f : {2, 3, 5, 7})
      while (r % f == 0) pl.radix.push_back(f), r /= f;
    for (int f = 11; (int64_t)f * f <= r; f += 2)
      while (r % f == 0) pl.radix.push_back(f), r /= f;
    if (r > 1) pl.radix.push_back(r);
    if ((int)pl.radix.size() > kAnyMaxStages) return fail(c, OMEGA_EUNSUP, "length %d: too many factors", N);
    std::vector<float2> tw(N), rot(3 * (N / 2) + 1);
    for (int m = 0; m < N; ++m) tw[m] = make_float2((float)std::cos(2 * kPi * m / N), (float)-std::sin(2 * kPi * m / N));
    for (size_t m = 0; m < rot.size(); ++m)
      rot[m] = make_float2((float)std::cos(2 * kPi * (double)m / (4.0 * N)), (float)std::sin(2 * kPi * (double)m / (4.0 * N)));
    int e = upload(c, &pl.tw, tw);
    if (!e) e = upload(c, &pl.rot, rot);
    if (e) return e;
    it = c->any_plans.emplace(N, std::move(pl)).first;
  }
  *out = &it->second;
  return 0;
}

// launches the any-length kernel over n frames in slices whose global scratch (N > kAnyLdsMax) stays
// within 64 MiB; p.x / outputs advanced per slice
int run_any(omega_ctx* c, AnyFftParams p, int truepeak) {
  omega_ctx::AnyPlan* pl = nullptr;
  if (int e = get_any_plan(c, p.N, &pl)) return e;
  p.n_stages = (int)pl->radix.size();
  for (int s = 0; s < p.n_stages; ++s) p.radix[s] = pl->radix[s];
  p.tw = pl->tw;
  p.rot = pl->rot;
  for (int ph = 0; ph < 4; ++ph) p.nyq_cos[ph] = (float)std::cos(kPi * ph / 4.0);
  const int64_t n = p.n;
  int64_t per = n;
  if (p.N > kAnyLdsMax) {
    per = std::max<int64_t>(1, std::min<int64_t>(n, (int64_t)(8 << 20) / (3 * (int64_t)p.N)));
    if (int e = grow(c, &c->d_any, &c->any_cap, per * 3 * p.N)) return e;
    p.scratch = c->d_any;
  }
  const int nb = p.N / 2 + 1;
  for (int64_t f0 = 0; f0 < n; f0 += per) {
    AnyFftParams q = p;
    q.x = p.x + f0 * p.frame_stride;
    q.n = std::min(per, n - f0);
    if (q.tp_out) q.tp_out = p.tp_out + f0;
    if (q.mag) q.mag = p.mag + f0 * nb;
    if (q.cplx) q.cplx = p.cplx + f0 * nb * 2;
    HIPC(c, launch_any(q, truepeak, c->stream));
  }
  return 0;
}

int omega_true_peak_os(omega_ctx* c, const float* x, int64_t n, int32_t m, int32_t oversampling, float* out_db,
                       int mem) try {
  if (!c || !x || !out_db) return OMEGA_EINVAL;
  if (oversampling != 1 && oversampling != 2 && oversampling != 4)
    return fail(c, OMEGA_EUNSUP, "true peak: oversampling %d unsupported (1, 2, 4)", oversampling);
  if (m < 1) return fail(c, OMEGA_EINVAL, "true peak: frame length %d", m);
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  const bool any = !is_pow2_in(m, 512, 16384);
  HIPC(c, hipSetDevice(c->device));
  std::vector<HostOut> outs;
  const float* dx = x;
  float* dout = out_db;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)n * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 3, out_db, n, outs, &dout);
    if (e) return e;
  }
  if (any) {  // frames of other lengths (anyfft.hip)
    AnyFftParams ap{};
    ap.x = dx;
    ap.frame_stride = m;
    ap.n = n;
    ap.N = m;
    ap.phases = oversampling == 4 ? 0xE : (oversampling == 2 ? 0x4 : 0);
    ap.tp_out = dout;
    if ((e = run_any(c, ap, 1))) return e;
    if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
    return 0;
  }
  SpectralParams sp = spectral_params(c);
  sp.x = dx;
  sp.C = 1;
  sp.frame_stride = m;
  sp.chan_stride = 0;
  sp.n_cf = n;
  sp.comb_out = nullptr;
  for (int r = 0; r < kMaxRes; ++r) sp.res[r].mag_out = nullptr;
  sp.n_res = 0;
  sp.tp_out = dout;
  float2* rot = nullptr;
  e = get_rot(c, m, &rot);
  if (e) return e;
  sp.rot = rot;
  sp.tp_phases = oversampling == 4 ? 0xE : (oversampling == 2 ? 0x4 : 0);
  sp.tp_done = c->tp_count_to;  // (omega_calculate_lufs)
  HIPC(c, tp_launch(c, m, sp, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

// the batch kernel's float32 K-weighting (kweight_kernel) on its own, for power-of-two frames
int omega_k_weighting(omega_ctx* c, const float* x, int64_t n, int32_t m, float* weighted, float* lufs_inst,
                      int mem) try {
  if (!c || !x) return OMEGA_EINVAL;
  if (!is_pow2_in(m, 512, 16384)) return fail(c, OMEGA_EUNSUP, "k-weighting: frame length %d unsupported", m);
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  std::vector<HostOut> outs;
  const float* dx = x;
  float* dw = weighted;
  float* dl = lufs_inst;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)n * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 5, weighted, (size_t)n * m, outs, &dw);
    if (!e) e = stage_out(c, 2, lufs_inst, n, outs, &dl);
    if (e) return e;
  }
  BiquadTab* tabs = nullptr;
  if ((e = get_kw_tab(c, m, &tabs))) return e;
  KWeightParams kp{dx, m, 0, 1, n, tabs, tabs + 1, dl, dw, OMEGA_WEIGHT_K};
  HIPC(c, launch_kweight(m, kp, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

// The float64 filter cascade of a weighting mode for the context's sample rate
// (professional_meters.py:48-72, :74-127): K = {butter(2, 38 Hz, high), iirfilter(2, 1500 Hz, high)}
// blended 0.3; A = {butter(2, 20.598997, high), butter(1, 107.65265, high), butter(1, 737.86223, low),
// butter(2, min(12194.217 / nyq, 0.99), low)} x 2.5; C = {butter(2, 20.598997, high), butter(2, 12194.217, low)}.
W64Stage w64_stage(const BiquadCoef& q, int order) {
  W64Stage s{};
  s.b0 = q.b[0];
  s.b1 = q.b[1];
  s.b2 = q.b[2];
  s.a1 = q.a[1];
  s.a2 = q.a[2];
  // scipy.signal.lfilter_zi: solve (I - companion(a).T) zi = b[1:] - a[1:] b[0]
  const double B0 = s.b1 - s.a1 * s.b0, B1 = s.b2 - s.a2 * s.b0;
  s.zi0 = (B0 + B1) / (1.0 + s.a1 + s.a2);
  s.zi1 = B1 - s.a2 * s.zi0;
  s.E = 3 * (order + 1);  // filtfilt's default padlen 3 max(len(a), len(b))
  return s;
}

int get_w64_stages(omega_ctx* c, int mode, W64Stage** out) {
  if (c->w64[mode]) {
    *out = c->w64[mode];
    return 0;
  }
  const double fs = c->cfg.sample_rate, nyq = fs / 2;
  const double f1 = 20.598997, f2 = 107.65265, f3 = 737.86223, f4 = 12194.217;
  const double f4c = std::min(f4 / nyq, 0.99) * nyq;
  std::vector<W64Stage> t;
  if (mode == OMEGA_WEIGHT_K)
    t = {w64_stage(butter2_highpass(38.0, fs), 2), w64_stage(butter2_highpass(1500.0, fs), 2)};
  else if (mode == OMEGA_WEIGHT_A)
    t = {w64_stage(butter2_highpass(f1, fs), 2), w64_stage(butter1(f2, fs, true), 1),
         w64_stage(butter1(f3, fs, false), 1), w64_stage(butter2_lowpass(f4c, fs), 2)};
  else
    t = {w64_stage(butter2_highpass(f1, fs), 2), w64_stage(butter2_lowpass(f4c, fs), 2)};
  if (int e = upload(c, &c->w64[mode], t)) return e;
  *out = c->w64[mode];
  return 0;
}

int omega_weighting(omega_ctx* c, const float* x, int64_t n, int32_t m, int32_t mode, float* weighted,
                    float* lufs_inst, int mem) try {
  if (!c || !x) return OMEGA_EINVAL;
  if (mode < OMEGA_WEIGHT_K || mode > OMEGA_WEIGHT_Z) return fail(c, OMEGA_EINVAL, "weighting mode %d", mode);
  // scipy's filtfilt needs more samples than its padlen (9 for the first section of K, A and C)
  if (m < 1 || (mode != OMEGA_WEIGHT_Z && m <= 9))
    return fail(c, OMEGA_EINVAL, "weighting: the length of the input (%d) must be greater than padlen (9)", m);
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  std::vector<HostOut> outs;
  const float* dx = x;
  float* dw = weighted;
  float* dl = lufs_inst;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)n * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 5, weighted, (size_t)n * m, outs, &dw);
    if (!e) e = stage_out(c, 2, lufs_inst, n, outs, &dl);
    if (e) return e;
  }
  Weight64Params p{};
  p.M = m;
  p.mode = mode;
  if (mode != OMEGA_WEIGHT_Z) {
    if ((e = get_w64_stages(c, mode, &p.st))) return e;
    p.n_st = mode == OMEGA_WEIGHT_A ? 4 : 2;
  }
  // float64 working buffers per frame: the signal and its odd extension (at most 64 MiB per launch)
  p.scratch_stride = 2 * (int64_t)m + 32;
  const int64_t per_launch = std::max<int64_t>(1, std::min<int64_t>(n, (int64_t)(8 << 20) / p.scratch_stride));
  if ((e = grow(c, &c->d_w64, &c->w64_cap, per_launch * p.scratch_stride))) return e;
  p.scratch = c->d_w64;
  for (int64_t f0 = 0; f0 < n; f0 += per_launch) {
    p.x = dx + f0 * m;
    p.n = std::min(per_launch, n - f0);
    p.weighted_out = dw ? dw + f0 * m : nullptr;
    p.lufs_out = dl ? dl + f0 : nullptr;
    HIPC(c, launch_weight64(p, c->stream));
  }
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

// The meter aggregates on the caller's stream from device inputs. join_side: these kernels read the
// state a meter prep on the side stream may still be writing (after its count-in), so the caller's
// stream first waits for the side stream (a caller that has just joined it skips the second wait);
// order_side: the next batch's meter prep runs on the side stream and reads, before its K-weighting
// count, the state these kernels write, so the side stream is ordered after them (a host-memory
// caller does it after its copies back, which then follow the kernels without an event between).
int meter_update_dev(omega_ctx* c, const float* dl, const float* dt, int64_t n_frames, double* dm, bool join_side,
                     bool order_side, unsigned* wait_ctr = nullptr, unsigned wait_target = 0) {
  if (join_side) {
    HIPC(c, hipEventRecord(c->ev_join[1], c->fork[0]));
    HIPC(c, hipStreamWaitEvent(c->stream, c->ev_join[1], 0));
  }
  if (int e = meters_enqueue(c, dl, dt, n_frames, dm, c->stream, nullptr, wait_ctr, wait_target)) return e;
  if (order_side) {
    HIPC(c, hipEventRecord(c->ev_fork, c->stream));
    HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_fork, 0));
  }
  return 0;
}

int omega_meter_update(omega_ctx* c, const float* lufs_inst, const float* tp_db, int64_t n_frames, double* meters,
                       int mem) try {
  if (!c || !lufs_inst || !tp_db || !meters) return OMEGA_EINVAL;
  if (n_frames <= 0) return n_frames == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  if (int e = check_device_err(c)) return e;
  HIPC(c, hipSetDevice(c->device));
  if (int e = flush_meters(c)) return e;
  const int64_t ncf = n_frames * c->cfg.n_channels;
  std::vector<HostOut> outs;
  const float* dl = lufs_inst;
  const float* dt = tp_db;
  double* dm = meters;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 2, lufs_inst, ncf * sizeof(float), reinterpret_cast<const void**>(&dl));
    if (!e) e = stage_in(c, 3, tp_db, ncf * sizeof(float), reinterpret_cast<const void**>(&dt));
    if (!e) e = stage_out(c, 4, meters, ncf * 5, outs, &dm);
    if (e) return e;
  }
  if ((e = meter_update_dev(c, dl, dt, n_frames, dm, true, true))) return e;
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_meter_load_history(omega_ctx* c, const float* lufs_inst, int64_t n_l, const float* tp_db, int64_t n_t,
                             int mem) try {
  if (!c) return OMEGA_EINVAL;
  if (n_l < 0 || n_t < 0 || n_t > n_l) return fail(c, OMEGA_EINVAL, "need 0 <= n_t <= n_l");
  if ((n_l && !lufs_inst) || (n_t && !tp_db)) return fail(c, OMEGA_EINVAL, "null history");
  // rows older than the windows hold (integrated_len - 1 LUFS values, peak_len - 1 true peaks) leave no
  // trace in the state a replay of them would build: keep the last ones (a time-shard exchange hands over
  // up to 3599 / 59 rows whatever this context's window lengths are)
  if (n_l > c->HL) {
    lufs_inst += (n_l - c->HL) * (int64_t)c->cfg.n_channels;
    n_l = c->HL;
  }
  if (n_t > std::min<int64_t>(c->HT, n_l)) {
    const int64_t k = std::min<int64_t>(c->HT, n_l);
    tp_db += (n_t - k) * (int64_t)c->cfg.n_channels;
    n_t = k;
  }
  if (int e = check_device_err(c)) return e;
  HIPC(c, hipSetDevice(c->device));
  if (int e = flush_meters(c)) return e;  // (a pending segment reads the state being replaced)
  const int C = c->cfg.n_channels;
  const float* dl = lufs_inst;
  const float* dt = tp_db;
  if (mem == OMEGA_MEM_HOST) {
    int e = stage_in(c, 2, lufs_inst, (size_t)n_l * C * sizeof(float), reinterpret_cast<const void**>(&dl));
    if (!e) e = stage_in(c, 3, tp_db, (size_t)n_t * C * sizeof(float), reinterpret_cast<const void**>(&dt));
    if (e) return e;
  }
  // as omega_meter_update: after the side stream's last writes of the state, and before its next reads
  HIPC(c, hipEventRecord(c->ev_join[1], c->fork[0]));
  HIPC(c, hipStreamWaitEvent(c->stream, c->ev_join[1], 0));
  const int a = c->cur;
  MeterLoadParams p{dl, dt, (int)n_l, (int)n_t, C, c->HL, c->HT, (float)c->cfg.gate_lufs, c->d_hist_l[a],
                    c->d_hist_t[a], c->d_nl[a], c->d_nt[a], c->d_skeys[a], c->d_ns[a], c->d_t0[a]};
  HIPC(c, launch_meter_load(p, c->stream));
  HIPC(c, hipEventRecord(c->ev_fork, c->stream));
  HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_fork, 0));
  if (mem == OMEGA_MEM_HOST) HIPC(c, hipStreamSynchronize(c->stream));
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_calculate_lufs(omega_ctx* c, const float* x, int64_t n_frames, int32_t m, int32_t mode, int32_t oversampling,
                         float* lufs_inst, float* tp_db, double* meters, int mem) try {
  if (!c || !x || !meters) return OMEGA_EINVAL;
  if (n_frames <= 0) return n_frames == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  if (int e = check_device_err(c)) return e;
  HIPC(c, hipSetDevice(c->device));
  const int64_t ncf = n_frames * c->cfg.n_channels;
  std::vector<HostOut> outs;
  const float* dx = x;
  float* dl = lufs_inst;
  float* dt = tp_db;
  double* dm = meters;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)ncf * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 2, lufs_inst, ncf, outs, &dl);
    if (!e) e = stage_out(c, 3, tp_db, ncf, outs, &dt);
    if (!e) e = stage_out(c, 4, meters, ncf * 5, outs, &dm);
    if (e) return e;
  }
  // device scratch for the instantaneous values the caller does not want back
  if (!dl || !dt) {
    if ((e = grow(c, &c->d_lufs_scr, &c->lufs_scr_cap, 2 * ncf))) return e;
    if (!dl) dl = c->d_lufs_scr;
    if (!dt) dt = c->d_lufs_scr + ncf;
  }
  // The weighting and the true peak read the same input and write different outputs: the true peak
  // runs on the side stream beside the weighting's latency-bound float64 scans (per-call metering of
  // the app's 2048-sample frames: 37 + 14 us of kernels in sequence before). The aggregates read the
  // meter state, which a meter prep on the side stream may still be writing, and the true peaks.
  // Joining the side stream by an event costs ~5-10 us of idle GPU between kernels, so: when no meter
  // kernel went to the side stream since the last join (the app's steady state: nothing but these
  // calls; side_meters) there is nothing to join before, and the true peaks (power-of-two frames,
  // direct launches) count themselves in on a device counter that the first meter prep polls before it
  // reads them; otherwise events, as omega_meter_update.
  const bool capture = c->cap && c->stream == c->cap;
  const bool counted = !capture && is_pow2_in(m, 512, 16384);
  if (counted && c->side_meters) {
    HIPC(c, hipEventRecord(c->ev_join[1], c->fork[0]));
    HIPC(c, hipStreamWaitEvent(c->stream, c->ev_join[1], 0));
  }
  c->side_meters = false;
  HIPC(c, hipEventRecord(c->ev_fork, c->stream));
  HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_fork, 0));
  {
    const hipStream_t main = c->stream;
    c->stream = c->fork[0];
    c->tp_count_to = counted ? c->d_kw_done + 5 : nullptr;
    e = omega_true_peak_os(c, dx, ncf, m, oversampling, dt, OMEGA_MEM_DEVICE);
    c->tp_count_to = nullptr;
    c->stream = main;
    if (e) return e;
  }
  if (counted) c->lt_issued += (unsigned)ncf;
  if ((e = omega_weighting(c, dx, ncf, m, mode, nullptr, dl, OMEGA_MEM_DEVICE))) return e;
  if (!counted) {
    // the side stream's last work is the true peak, behind any earlier meter prep: one join serves
    // both (omega_meter_update's second wait is skipped)
    HIPC(c, hipEventRecord(c->ev_join[0], c->fork[0]));
    HIPC(c, hipStreamWaitEvent(c->stream, c->ev_join[0], 0));
  }
  if ((e = flush_meters(c))) return e;
  // for a host-memory call the side stream is ordered after the copies back (no event between the
  // aggregates and the copies)
  const bool host = mem == OMEGA_MEM_HOST;
  if ((e = meter_update_dev(c, dl, dt, n_frames, dm, false, !host, counted ? c->d_kw_done + 5 : nullptr,
                            c->lt_issued)))
    return e;
  if (host) {
    if ((e = finish_host(c, outs))) return e;
    HIPC(c, hipEventRecord(c->ev_fork, c->stream));
    HIPC(c, hipStreamWaitEvent(c->fork[0], c->ev_fork, 0));
    return 0;
  }
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_bands_create(omega_ctx* c, int op, const int32_t* starts, const int32_t* ends, int32_t n_bands,
                       int32_t n_out, const double* scale, const double* bin_scale, int32_t n_bins, omega_bands** out) try {
  if (!c || !starts || !ends || !out || n_bands < 0 || n_out < 0 || n_bins <= 0) return OMEGA_EINVAL;
  if (op != OMEGA_BANDS_MAX && op != OMEGA_BANDS_MEAN) return fail(c, OMEGA_EINVAL, "unknown band op %d", op);
  HIPC(c, hipSetDevice(c->device));
  omega_bands* b = new (std::nothrow) omega_bands();
  if (!b) return OMEGA_ENOMEM;
  b->ctx = c;
  b->op = op;
  b->n_bands = n_bands;
  b->n_out = n_out;
  b->n_bins = n_bins;
  // MAX (pipeline.py:207-220): bands min(num_bands, len(table)); each one that fits the spectrum.
  // MEAN (freq_mapper.py:184-194): stops at the first band running past the spectrum.
  int nv = std::min(n_bands, n_out);
  if (op == OMEGA_BANDS_MEAN) {
    for (int i = 0; i < nv; ++i)
      if (ends[i] > n_bins) {
        nv = i;
        break;
      }
  }
  b->n_valid = nv;
  std::vector<int32_t> s(starts, starts + n_bands), en(ends, ends + n_bands);
  if (s.empty()) {
    s.push_back(0);
    en.push_back(1);
  }
  int e = upload(c, &b->d_starts, s);
  if (!e) e = upload(c, &b->d_ends, en);
  b->d_scale = nullptr;
  b->d_bin_scale = nullptr;
  if (!e && scale) {
    std::vector<float> sc(std::max(n_out, 1), 1.0f);
    for (int i = 0; i < std::min(n_bands, n_out); ++i) sc[i] = (float)scale[i];
    e = upload(c, &b->d_scale, sc);
  }
  if (!e && bin_scale) {
    std::vector<float> bs(bin_scale, bin_scale + n_bins);
    e = upload(c, &b->d_bin_scale, bs);
  }
  if (e) {
    delete b;
    return e;
  }
  *out = b;
  return 0;
} catch (...) {
  return guard_fail(c);
}

void omega_bands_destroy(omega_bands* b) { delete b; }  // device tables are owned by the context

int omega_bands_apply(omega_ctx* c, omega_bands* b, const float* spec, int64_t n, int64_t spec_stride, float* out,
                      int mem) try {
  if (!c || !b || !spec || !out) return OMEGA_EINVAL;
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  std::vector<HostOut> outs;
  const float* ds = spec;
  float* dout = out;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, spec, ((n - 1) * spec_stride + b->n_bins) * sizeof(float), reinterpret_cast<const void**>(&ds));
    if (!e) e = stage_out(c, 1, out, (size_t)n * b->n_out, outs, &dout);
    if (e) return e;
  }
  BandParams p{ds, n, spec_stride, b->n_bins, b->n_out, b->d_starts, b->d_ends, b->d_scale, b->d_bin_scale, b->op,
               b->n_valid, dout};
  HIPC(c, launch_bands(p, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_chroma(omega_ctx* c, const float* spec, int64_t n, int32_t n_bins, double df, double* out_raw, int mem) try {
  if (!c || !spec || !out_raw || n_bins < 3 || !(df > 0)) return OMEGA_EINVAL;
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  auto it = c->chroma_mats.find(n_bins);
  if (it == c->chroma_mats.end() || c->chroma_df != df) {
    // chromagram.py:122-146 with transposition offset 0: bins 20 < f < 8000
    int lo = n_bins, hi = 0;
    for (int k = 0; k < n_bins; ++k) {
      const double f = k * df;
      if (f > 20 && f < 8000) {
        lo = std::min(lo, k);
        hi = std::max(hi, k + 1);
      }
    }
    if (hi <= lo) lo = hi = 0;
    const int nb = std::max(hi - lo, 1);
    std::vector<double> m(12 * (size_t)nb, 0.0);
    for (int k = lo; k < hi; ++k) {
      const double f = k * df;
      const double midi = 69 + 12 * std::log2(f / 440.0);
      double cb = std::fmod(midi, 12.0);
      if (cb < 0) cb += 12.0;
      const int base = (int)cb;
      const double sw = f < 100 ? 0.5 : (f < 1000 ? 1.0 : (f < 4000 ? 0.8 : 0.6));
      for (int o = -2; o <= 2; ++o) {
        const int tb = ((base + o) % 12 + 12) % 12;
        const double d = std::fabs(cb - (base + o));
        const double w = std::exp(-0.5 * (d / 0.5) * (d / 0.5));
        m[(size_t)tb * nb + (k - lo)] += w * sw;
      }
    }
    double* d = nullptr;
    HIPC(c, hipMalloc(&d, m.size() * sizeof(double)));
    HIPC(c, hipMemcpy(d, m.data(), m.size() * sizeof(double), hipMemcpyHostToDevice));
    if (it != c->chroma_mats.end()) (void)hipFree(it->second.first);
    c->chroma_mats[n_bins] = {d, {lo, hi}};
    c->chroma_df = df;
    it = c->chroma_mats.find(n_bins);
  }
  std::vector<HostOut> outs;
  const float* ds = spec;
  double* dout = out_raw;
  int e = 0;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, spec, (size_t)n * n_bins * sizeof(float), reinterpret_cast<const void**>(&ds));
    if (!e) e = stage_out(c, 1, out_raw, (size_t)n * 12, outs, &dout);
    if (e) return e;
  }
  HIPC(c, launch_chroma(ds, n, n_bins, it->second.second.first, it->second.second.second, it->second.first, dout,
                        c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_rfft(omega_ctx* c, const float* x, int64_t n, int32_t m, int32_t window, float* mag, float* cplx, int mem) try {
  if (!c || !x || (!mag && !cplx)) return OMEGA_EINVAL;
  if (m < 1) return fail(c, OMEGA_EINVAL, "rfft: length %d", m);
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  float* win = nullptr;
  int e = get_window(c, m, window, &win);
  if (e) return e;
  std::vector<HostOut> outs;
  const float* dx = x;
  float* dm = mag;
  float* dc = cplx;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)n * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e) e = stage_out(c, 1, mag, (size_t)n * (m / 2 + 1), outs, &dm);
    if (!e) e = stage_out(c, 2, cplx, (size_t)n * (m / 2 + 1) * 2, outs, &dc);
    if (e) return e;
  }
  if (!is_pow2_in(m, 512, 16384)) {  // other lengths: the mixed-radix transform (anyfft.hip)
    AnyFftParams ap{};
    ap.x = dx;
    ap.frame_stride = m;
    ap.n = n;
    ap.N = m;
    ap.win = win;
    ap.mag = dm;
    ap.cplx = dc;
    if ((e = run_any(c, ap, 0))) return e;
    if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
    return 0;
  }
  RfftParams p{};
  p.x = dx;
  p.n = n;
  p.win = win;
  p.mag = dm;
  p.cplx = dc;
  for (int l = 0; l < kMaxLog2; ++l) p.tw[l] = c->d_tw[l];
  HIPC(c, launch_rfft(m, p, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

int omega_spectra(omega_ctx* c, const float* x, int64_t n, int32_t m, int32_t window, omega_bands* bands,
                  float* bands_out, double* chroma_out, float* mag_out, int mem) try {
  if (!c || !x || (!bands_out && !chroma_out && !mag_out)) return OMEGA_EINVAL;
  if (m != 8192) return fail(c, OMEGA_EUNSUP, "spectra: frame length %d unsupported (8192)", m);
  if (bands_out && (!bands || bands->op != OMEGA_BANDS_MAX || bands->n_bins != m / 2 + 1 || bands->n_valid > 512))
    return fail(c, OMEGA_EINVAL, "spectra: needs a MAX band table over %d bins with at most 512 bands", m / 2 + 1);
  if (n <= 0) return n == 0 ? 0 : fail(c, OMEGA_EINVAL, "negative count");
  HIPC(c, hipSetDevice(c->device));
  float* win = nullptr;
  int e = get_window(c, m, window, &win);
  if (e) return e;
  const int nbins = m / 2 + 1;
  const double df = (double)c->cfg.sample_rate / m;
  if (c->ctab.n_bins != nbins || c->ctab.df != df) {
    // chromagram.py:122-146 with offset 0: bins 20 < f < 8000, base class floor((69 + 12 log2(f/440)) mod 12)
    int lo = nbins, hi = 0;
    for (int k = 0; k < nbins; ++k) {
      const double f = k * df;
      if (f > 20 && f < 8000) {
        lo = std::min(lo, k);
        hi = std::max(hi, k + 1);
      }
    }
    if (hi <= lo) lo = hi = 0;
    const int nb = hi - lo;
    if (nb > 1408) return fail(c, OMEGA_EUNSUP, "spectra: %d chroma bins (at most 1408)", nb);
    std::vector<float4> w4(std::max(nb, 1));
    std::vector<float> w1(std::max(nb, 1));
    std::vector<int> base(std::max(nb, 1));
    std::vector<float> ra(std::max(nb, 1)), rg(std::max(nb, 1));  // SpectraParams::crec's a, g
    for (int k = lo; k < hi; ++k) {
      const double f = k * df;
      double cb = std::fmod(69 + 12 * std::log2(f / 440.0), 12.0);
      if (cb < 0) cb += 12.0;
      const int b = (int)cb;
      const double sw = f < 100 ? 0.5 : (f < 1000 ? 1.0 : (f < 4000 ? 0.8 : 0.6));
      float w[5];
      for (int o = -2; o <= 2; ++o) {
        const double d = std::fabs(cb - (b + o));
        w[o + 2] = (float)(std::exp(-0.5 * (d / 0.5) * (d / 0.5)) * sw);
      }
      w4[k - lo] = make_float4(w[0], w[1], w[2], w[3]);
      w1[k - lo] = w[4];
      base[k - lo] = b;
      const double u = cb - b;
      ra[k - lo] = (float)(std::exp(-2.0 * u * u) * sw);
      rg[k - lo] = (float)std::exp(4.0 * u);
    }
    std::vector<unsigned short> perm;
    std::vector<int> goff(13, 0);
    for (int b = 0; b < 12; ++b) {
      goff[b] = (int)perm.size();
      for (int i = 0; i < nb; ++i)
        if (base[i] == b) perm.push_back((unsigned short)i);
    }
    goff[12] = (int)perm.size();
    if (perm.empty()) perm.push_back(0);
    std::vector<float> rec(3 * perm.size());
    for (size_t j = 0; j < perm.size(); ++j) {
      const int i = perm[j];
      const int bin = lo + i;
      rec[3 * j] = ra[i];
      rec[3 * j + 1] = rg[i];
      std::memcpy(&rec[3 * j + 2], &bin, sizeof bin);  // the bin index's bits
    }
    for (void* q : {(void*)c->ctab.w4, (void*)c->ctab.w1, (void*)c->ctab.perm, (void*)c->ctab.goff,
                    (void*)c->ctab.rec})
      if (q) (void)hipFree(q);
    c->ctab = omega_ctx::ChromaTab{};
    HIPC(c, hipMalloc(&c->ctab.rec, rec.size() * sizeof(float)));
    HIPC(c, hipMemcpy(c->ctab.rec, rec.data(), rec.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPC(c, hipMalloc(&c->ctab.w4, w4.size() * sizeof(float4)));
    HIPC(c, hipMalloc(&c->ctab.w1, w1.size() * sizeof(float)));
    HIPC(c, hipMalloc(&c->ctab.perm, perm.size() * sizeof(unsigned short)));
    HIPC(c, hipMalloc(&c->ctab.goff, goff.size() * sizeof(int)));
    HIPC(c, hipMemcpy(c->ctab.w4, w4.data(), w4.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->ctab.w1, w1.data(), w1.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->ctab.perm, perm.data(), perm.size() * sizeof(unsigned short), hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(c->ctab.goff, goff.data(), goff.size() * sizeof(int), hipMemcpyHostToDevice));
    c->ctab.n_bins = nbins;
    c->ctab.df = df;
    c->ctab.lo = lo;
    c->ctab.hi = hi;
  }
  if (!c->n_cu) {
    hipDeviceProp_t prop;
    HIPC(c, hipGetDeviceProperties(&prop, c->device));
    c->n_cu = prop.multiProcessorCount;
  }
  std::vector<HostOut> outs;
  const float* dx = x;
  float* db = bands_out;
  double* dcr = chroma_out;
  float* dm = mag_out;
  if (mem == OMEGA_MEM_HOST) {
    e = stage_in(c, 0, x, (size_t)n * m * sizeof(float), reinterpret_cast<const void**>(&dx));
    if (!e && bands_out) e = stage_out(c, 1, bands_out, (size_t)n * bands->n_out, outs, &db);
    if (!e && chroma_out) e = stage_out(c, 2, chroma_out, (size_t)n * 12, outs, &dcr);
    if (!e && mag_out) e = stage_out(c, 3, mag_out, (size_t)n * nbins, outs, &dm);
    if (e) return e;
  }
  SpectraParams p{};
  p.x = dx;
  p.n = n;
  p.stride = m;
  p.win = win;
  float4* wgen = nullptr;
  if (m == 8192 && (e = get_wingen(c, m, window, &wgen))) return e;
  p.wgen = wgen;
  p.mag_out = dm;
  if (bands_out) {
    p.n_out = bands->n_out;
    p.n_valid = bands->n_valid;
    p.starts = bands->d_starts;
    p.ends = bands->d_ends;
    p.scale = bands->d_scale;
    p.bands_out = db;
  }
  p.c_lo = c->ctab.lo;
  p.c_hi = c->ctab.hi;
  p.cw4 = c->ctab.w4;
  p.cw1 = c->ctab.w1;
  p.cperm = c->ctab.perm;
  p.cgoff = c->ctab.goff;
  p.crec = c->ctab.rec;
  p.chroma_out = dcr;
  for (int l = 0; l < kMaxLog2; ++l) p.tw[l] = c->d_tw[l];
  const int grid = (int)std::min<int64_t>(n, 2 * (int64_t)c->n_cu);
  if (m == 8192)
    HIPC(c, launch_spectra_rf(m, p, c->stream));
  else
    HIPC(c, launch_spectra(m, p, grid, c->stream));
  if (mem == OMEGA_MEM_HOST) return finish_host(c, outs);
  return 0;
} catch (...) {
  return guard_fail(c);
}

}  // extern "C"
