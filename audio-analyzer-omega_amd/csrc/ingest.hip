// Sustained-stream ingest: the capture byte stream straight into the stream
// layout of the hot path.
//
//   capture.py:546-600   parec float32le / s16le chunks of chunk_size samples (s16 / 32768.0)
//   capture.py:620-641   per-chunk noise gate: RMS, background EMA, silence counter -> zeros
//   omega4_main.py:648-688  input gain, ring buffer -> the analysed window
//
// Host side: the caller's bytes are memcpy'd into page-locked staging slots (the only host work);
// a full slot is one batch of batch_hops * hop samples per channel. Per batch, on the ingest's copy
// stream: one H2D of the raw interleaved bytes; on its compute stream (the context's stream): the gate
// RMS per capture chunk, the gate state scan, the unpack (carry of the previous batch's last samples +
// convert + gate + gain, planar), omega_process_stream over the batch's frames, and one D2H of the
// outputs into the slot's page-locked result block. The copy of batch b + 1 overlaps the analysis of
// batch b; the host never waits unless every staging slot is in flight.
//
// The gate runs as the reference's capture loop does with any channel count: it reads chunk_size
// samples of the interleaved stream at a time (capture.py:549-550: chunk_bytes = chunk_size * bytes
// per sample, whatever the channels), so a chunk holds chunk_size / C frames (or straddles frames), one
// RMS covers every channel of it, one background level and one silence counter (counting chunk_size
// interleaved samples per chunk) serve all channels, and a gated chunk zeroes all its samples.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <vector>

#include "../../include/omega.h"
#include "numpy_emul.hpp"

#pragma clang fp contract(off)

namespace omega {

struct IngestParams {
  const unsigned char* raw;  // [n_new][C] interleaved samples of `fmt`
  int fmt;                   // OMEGA_FMT_*
  int C;
  int64_t n_new;             // new samples per channel
  const float* prev;         // previous batch buffer; carry = prev[c * pitch + prev_off + i], i < carry
  int64_t prev_off, carry;
  float* dst;                // [C][pitch]: carry ++ new
  int64_t pitch;
  float gain;
  int gate;                  // noise gate on
  int chunk;                 // gate chunk (capture chunk_size), interleaved samples
  int64_t n_chunks;          // n_new * C / chunk
  float* rms;                // [n_chunks]
  unsigned char* zero;       // [n_chunks] chunk gated to zeros
  float* bg;                 // background level (float32 after its first update, as numpy computes it)
  int64_t* silence;          // silence_samples
  float nf2, nf, one_m_alpha, alpha;  // float32(noise_floor * 2), float32(noise_floor), float32(1 - a), float32(a)
  int64_t silence_threshold;
};

// interleaved sample k = frame * C + channel
__device__ __forceinline__ float ingest_sample(const IngestParams& p, int64_t k) {
  if (p.fmt == OMEGA_FMT_S16LE) {
    const short v = reinterpret_cast<const short*>(p.raw)[k];
    return (float)v / 32768.0f;  // astype(float32) / 32768.0 (capture.py:574)
  }
  return reinterpret_cast<const float*>(p.raw)[k];
}

// rms of one capture chunk (chunk_size interleaved samples): np.sqrt(np.mean(x ** 2)) in float32
// (capture.py:623)
__global__ __launch_bounds__(256) void ingest_rms_kernel(IngestParams p) {
  extern __shared__ float sq[];
  const int64_t k = blockIdx.x;
  for (int i = threadIdx.x; i < p.chunk; i += 256) {
    const float v = ingest_sample(p, k * p.chunk + i);
    sq[i] = v * v;
  }
  __syncthreads();
  if (threadIdx.x == 0) p.rms[k] = np_sqrt_f32(np_mean_f32(sq, p.chunk));
}

// the gate state machine of _process_audio_frame, chunk by chunk (one thread: the stream's state)
__global__ void ingest_gate_kernel(IngestParams p) {
  if (threadIdx.x != 0) return;
  float bg = *p.bg;
  int64_t sil = *p.silence;
  for (int64_t k = 0; k < p.n_chunks; ++k) {
    const float r = p.rms[k];
    // background_level = (1 - a) * bg + a * rms: Python floats times a float32 scalar stay float32
    if (r < p.nf2) bg = p.one_m_alpha * bg + p.alpha * r;
    const float b3 = bg * 3.0f;
    const float thr = b3 > p.nf ? b3 : p.nf;  // max(noise_floor, bg * 3)
    unsigned char z = 0;
    if (r < thr) {
      sil += p.chunk;
      z = sil > p.silence_threshold;
    } else {
      sil = 0;
    }
    p.zero[k] = z;
  }
  *p.bg = bg;
  *p.silence = sil;
}

// carry ++ gated, gain-scaled new samples, planar
__global__ __launch_bounds__(256) void ingest_unpack_kernel(IngestParams p) {
  const int c = blockIdx.y;
  const int64_t n = p.carry + p.n_new;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v;
    if (i < p.carry) {
      v = p.prev[c * p.pitch + p.prev_off + i];
    } else {
      const int64_t k = (i - p.carry) * p.C + c;
      v = ingest_sample(p, k);
      if (p.gate && p.zero[k / p.chunk]) v = 0.f;
      v = v * p.gain;  // audio_data * input_gain (omega4_main.py:660)
    }
    p.dst[c * p.pitch + i] = v;
  }
}

}  // namespace omega

using namespace omega;

struct omega_ingest {
  omega_ctx* ctx = nullptr;
  omega_ingest_config cfg{};
  int C = 0, W = 0, H = 0, B = 0, T = 0, bps = 4, device = 0;
  int64_t slot_samples = 0;  // B * H samples per channel
  size_t slot_bytes = 0;
  int64_t pitch = 0;
  hipStream_t comp = nullptr, copy = nullptr;
  // page-locked input staging: a slot is refilled once its H2D copy is done
  struct Slot {
    unsigned char* h_raw = nullptr;
    size_t fill = 0;
    bool inflight = false;
    hipEvent_t ev_h2d = nullptr;
  };
  // one batch's results: device outputs and their page-locked host copy, handed out in frame order
  struct Out {
    float *d_comb = nullptr, *d_li = nullptr, *d_tp = nullptr;
    double* d_met = nullptr;
    float *h_comb = nullptr, *h_li = nullptr, *h_tp = nullptr;
    double* h_met = nullptr;
    hipEvent_t ev_done = nullptr;
    int64_t n_frames = 0, consumed = 0;
  };
  std::vector<Slot> slots;
  int fill_slot = 0;
  std::vector<Out*> outs;        // every result block (owned)
  std::vector<Out*> free_outs;   // unused blocks
  std::deque<Out*> queue;        // launched batches in frame order, not yet fully polled
  int max_pending = 0;           // result blocks kept for the caller; beyond, the oldest are dropped
  unsigned char* d_raw[2] = {nullptr, nullptr};
  float* d_in[2] = {nullptr, nullptr};
  hipEvent_t ev_unpacked[2] = {nullptr, nullptr};
  int cur = 1;  // device buffer of the previous batch
  int64_t carry = 0, prev_off = 0;
  float *d_rms = nullptr, *d_bg = nullptr;
  unsigned char* d_zero = nullptr;
  int64_t* d_sil = nullptr;
  int64_t max_chunks = 0;
  omega_ingest_stats st{};
  char err[512] = {};  // omega_ingest_last_error (fixed: reporting an error allocates nothing)
};

namespace {

int ifail(omega_ingest* in, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (in) std::memcpy(in->err, buf, sizeof buf);
  return code;
}

#define IHIP(in, x)                                                                            \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return ifail(in, OMEGA_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// extern "C" entry points are function-try-blocks (the ABI contract, omega.h): what escapes becomes a
// status code and omega_ingest_last_error. Called only from inside a catch clause.
int iguard_fail(omega_ingest* in) noexcept {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    return ifail(in, OMEGA_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return ifail(in, OMEGA_EHIP, "internal error: %s", e.what());
  } catch (...) {
    return ifail(in, OMEGA_EHIP, "internal error: unknown exception");
  }
}

int ctx_call(omega_ingest* in, int code) {
  if (code) return ifail(in, code, "%s", omega_last_error(in->ctx));
  return 0;
}

int alloc_out(omega_ingest* in, omega_ingest::Out** out) {
  auto* o = new (std::nothrow) omega_ingest::Out();
  if (!o) return ifail(in, OMEGA_ENOMEM, "result block: out of host memory");
  in->outs.push_back(o);
  const size_t rows = (size_t)in->B * in->C;
  IHIP(in, hipEventCreateWithFlags(&o->ev_done, hipEventDisableTiming));
  const int w = in->cfg.want;
  if (w & OMEGA_INGEST_COMBINED) {
    IHIP(in, hipMalloc(&o->d_comb, rows * in->T * sizeof(float)));
    IHIP(in, hipHostMalloc(reinterpret_cast<void**>(&o->h_comb), rows * in->T * sizeof(float), hipHostMallocDefault));
  }
  if (w & (OMEGA_INGEST_LUFS | OMEGA_INGEST_METERS)) {  // (the meters need the instantaneous values)
    IHIP(in, hipMalloc(&o->d_li, rows * sizeof(float)));
    IHIP(in, hipHostMalloc(reinterpret_cast<void**>(&o->h_li), rows * sizeof(float), hipHostMallocDefault));
  }
  if (w & (OMEGA_INGEST_TRUE_PEAK | OMEGA_INGEST_METERS)) {
    IHIP(in, hipMalloc(&o->d_tp, rows * sizeof(float)));
    IHIP(in, hipHostMalloc(reinterpret_cast<void**>(&o->h_tp), rows * sizeof(float), hipHostMallocDefault));
  }
  if (w & OMEGA_INGEST_METERS) {
    IHIP(in, hipMalloc(&o->d_met, rows * OMEGA_N_METERS * sizeof(double)));
    IHIP(in, hipHostMalloc(reinterpret_cast<void**>(&o->h_met), rows * OMEGA_N_METERS * sizeof(double),
                           hipHostMallocDefault));
  }
  *out = o;
  return 0;
}

// a result block for the next batch: a free one, a new one, or -- max_pending reached -- the oldest
// unpolled one, whose remaining frames are dropped (the capture buffer's policy, capture.py:579-580)
int take_out(omega_ingest* in, omega_ingest::Out** out) {
  if (!in->free_outs.empty()) {
    *out = in->free_outs.back();
    in->free_outs.pop_back();
    return 0;
  }
  if ((int)in->outs.size() < in->max_pending) return alloc_out(in, out);
  omega_ingest::Out* o = in->queue.front();
  in->queue.pop_front();
  IHIP(in, hipEventSynchronize(o->ev_done));
  in->st.dropped_frames += o->n_frames - o->consumed;
  *out = o;
  return 0;
}

// analyse the first n_new samples per channel of slot s (whole gate chunks)
int launch_slot(omega_ingest* in, int s, int64_t n_new) {
  omega_ingest::Slot& sl = in->slots[s];
  omega_ingest::Out* ob = nullptr;
  if (int e = take_out(in, &ob)) return e;
  const int k = in->cur ^ 1;
  const size_t bytes = (size_t)n_new * in->C * in->bps;
  // H2D on the copy stream, once the unpack of the batch that last used d_raw[k] is done
  IHIP(in, hipStreamWaitEvent(in->copy, in->ev_unpacked[k], 0));
  IHIP(in, hipMemcpyAsync(in->d_raw[k], sl.h_raw, bytes, hipMemcpyHostToDevice, in->copy));
  IHIP(in, hipEventRecord(sl.ev_h2d, in->copy));
  sl.inflight = true;
  IHIP(in, hipStreamWaitEvent(in->comp, sl.ev_h2d, 0));
  IngestParams p{};
  p.raw = in->d_raw[k];
  p.fmt = in->cfg.format;
  p.C = in->C;
  p.n_new = n_new;
  p.prev = in->d_in[in->cur];
  p.prev_off = in->prev_off;
  p.carry = in->carry;
  p.dst = in->d_in[k];
  p.pitch = in->pitch;
  p.gain = in->cfg.gain;
  p.gate = in->cfg.gate;
  p.chunk = in->cfg.chunk_size;
  p.n_chunks = n_new * in->C / in->cfg.chunk_size;
  p.rms = in->d_rms;
  p.zero = in->d_zero;
  p.bg = in->d_bg;
  p.silence = in->d_sil;
  const double nf = in->cfg.noise_floor, a = in->cfg.background_alpha;
  p.nf2 = (float)(nf * 2);
  p.nf = (float)nf;
  p.one_m_alpha = (float)(1 - a);
  p.alpha = (float)a;
  p.silence_threshold = (int64_t)(in->cfg.sample_rate * in->cfg.silence_threshold_seconds);
  if (p.gate && p.n_chunks > 0) {
    hipLaunchKernelGGL(ingest_rms_kernel, dim3((unsigned)p.n_chunks), dim3(256), (size_t)p.chunk * sizeof(float),
                       in->comp, p);
    hipLaunchKernelGGL(ingest_gate_kernel, dim3(1), dim3(64), 0, in->comp, p);
  }
  const int64_t n = in->carry + n_new;
  const unsigned gx = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(ingest_unpack_kernel, dim3(gx, (unsigned)in->C), dim3(256), 0, in->comp, p);
  IHIP(in, hipGetLastError());
  IHIP(in, hipEventRecord(in->ev_unpacked[k], in->comp));
  const int64_t F = n < in->W ? 0 : (n - in->W) / in->H + 1;
  if (F > 0) {
    omega_outputs o{};
    o.combined = ob->d_comb;
    o.lufs_inst = ob->d_li;
    o.true_peak_db = ob->d_tp;
    o.meters = ob->d_met;
    int64_t got = 0;
    if (int e = ctx_call(in, omega_process_stream(in->ctx, in->d_in[k], n, in->H, in->pitch, &o, OMEGA_MEM_DEVICE, &got)))
      return e;
    const size_t rows = (size_t)F * in->C;
    if (o.combined) IHIP(in, hipMemcpyAsync(ob->h_comb, ob->d_comb, rows * in->T * sizeof(float), hipMemcpyDeviceToHost, in->comp));
    if (o.lufs_inst) IHIP(in, hipMemcpyAsync(ob->h_li, ob->d_li, rows * sizeof(float), hipMemcpyDeviceToHost, in->comp));
    if (o.true_peak_db) IHIP(in, hipMemcpyAsync(ob->h_tp, ob->d_tp, rows * sizeof(float), hipMemcpyDeviceToHost, in->comp));
    if (o.meters) IHIP(in, hipMemcpyAsync(ob->h_met, ob->d_met, rows * OMEGA_N_METERS * sizeof(double), hipMemcpyDeviceToHost, in->comp));
  }
  IHIP(in, hipEventRecord(ob->ev_done, in->comp));
  in->carry = n - F * in->H;
  in->prev_off = F * in->H;
  in->cur = k;
  ob->n_frames = F;
  ob->consumed = 0;
  in->queue.push_back(ob);
  in->st.frames += F;
  in->st.batches += 1;
  return 0;
}

// the slot the next bytes go to: wait for its previous H2D copy (backpressure on the copy engine only)
int take_fill_slot(omega_ingest* in, int* out) {
  const int s = in->fill_slot;
  omega_ingest::Slot& sl = in->slots[s];
  if (sl.inflight) {
    IHIP(in, hipEventSynchronize(sl.ev_h2d));
    sl.inflight = false;
    sl.fill = 0;
  }
  *out = s;
  return 0;
}

}  // namespace

extern "C" {

void omega_ingest_config_default(omega_ingest_config* c) try {
  if (!c) return;
  *c = omega_ingest_config{};
  c->format = OMEGA_FMT_F32LE;
  c->sample_rate = 48000;
  c->hop = 512;
  c->batch_hops = 64;
  c->ring_slots = 4;
  c->max_pending_batches = 64;
  c->chunk_size = 512;
  c->gain = 4.0f;  // omega4_main.py:152
  c->gate = 1;
  c->noise_floor = 0.001;  // capture.py:36-39
  c->silence_threshold_seconds = 0.25;
  c->background_alpha = 0.001;
  c->want = OMEGA_INGEST_COMBINED | OMEGA_INGEST_LUFS | OMEGA_INGEST_TRUE_PEAK | OMEGA_INGEST_METERS;
} catch (...) {
}

int omega_ingest_create(omega_ctx* ctx, const omega_ingest_config* cfg, omega_ingest** out) try {
  if (!ctx || !cfg || !out) return OMEGA_EINVAL;
  *out = nullptr;
  omega_config cc{};
  int device = 0;
  if (omega_get_config(ctx, &cc, &device)) return OMEGA_EINVAL;
  auto* in = new (std::nothrow) omega_ingest();
  if (!in) return OMEGA_ENOMEM;
  in->ctx = ctx;
  in->cfg = *cfg;
  in->C = cc.n_channels;
  in->W = cc.frame_size;
  in->H = cfg->hop;
  in->B = cfg->batch_hops;
  in->T = cc.target_bins;
  in->device = device;
  auto bad = [&](const char* m) {
    delete in;
    (void)m;
    return OMEGA_EINVAL;
  };
  if (cfg->format != OMEGA_FMT_F32LE && cfg->format != OMEGA_FMT_S16LE) return bad("format: float32le or s16le");
  in->bps = cfg->format == OMEGA_FMT_S16LE ? 2 : 4;
  if (in->C < 1 || in->W < 512 || in->T < 2) return bad("channels / frame size / target bins");
  if (in->H < 4 || in->H % 4) return bad("hop must be a positive multiple of 4");
  if (in->B < 1 || cfg->ring_slots < 2) return bad("batch_hops >= 1 and ring_slots >= 2");
  if (cfg->chunk_size < 1 || cfg->chunk_size > 8192) return bad("chunk_size 1..8192 (capture.py:64)");
  in->slot_samples = (int64_t)in->B * in->H;
  if (in->slot_samples * in->C % cfg->chunk_size)
    return bad("batch_hops * hop * channels must be a multiple of chunk_size (whole capture chunks per batch)");
  in->slot_bytes = (size_t)in->slot_samples * in->C * in->bps;
  in->pitch = ((int64_t)in->W + in->slot_samples + 3) / 4 * 4;
  in->max_chunks = in->slot_samples * in->C / cfg->chunk_size;
  *out = in;
  IHIP(in, hipSetDevice(device));
  IHIP(in, hipStreamCreateWithFlags(&in->comp, hipStreamNonBlocking));
  IHIP(in, hipStreamCreateWithFlags(&in->copy, hipStreamNonBlocking));
  if (int e = ctx_call(in, omega_set_stream(ctx, in->comp))) return e;
  for (int k = 0; k < 2; ++k) {
    IHIP(in, hipMalloc(&in->d_raw[k], in->slot_bytes));
    IHIP(in, hipMalloc(&in->d_in[k], (size_t)in->C * in->pitch * sizeof(float)));
    IHIP(in, hipEventCreateWithFlags(&in->ev_unpacked[k], hipEventDisableTiming));
    IHIP(in, hipEventRecord(in->ev_unpacked[k], in->comp));
  }
  IHIP(in, hipMalloc(&in->d_rms, (size_t)in->max_chunks * sizeof(float)));
  IHIP(in, hipMalloc(&in->d_zero, (size_t)in->max_chunks));
  IHIP(in, hipMalloc(&in->d_bg, sizeof(float)));
  IHIP(in, hipMalloc(&in->d_sil, sizeof(int64_t)));
  IHIP(in, hipMemset(in->d_bg, 0, sizeof(float)));
  IHIP(in, hipMemset(in->d_sil, 0, sizeof(int64_t)));
  in->slots.resize(cfg->ring_slots);
  for (auto& sl : in->slots) {
    IHIP(in, hipHostMalloc(reinterpret_cast<void**>(&sl.h_raw), in->slot_bytes, hipHostMallocDefault));
    IHIP(in, hipEventCreateWithFlags(&sl.ev_h2d, hipEventDisableTiming));
  }
  in->max_pending = std::max(cfg->max_pending_batches, 2);
  IHIP(in, hipStreamSynchronize(in->comp));
  return 0;
} catch (...) {
  return iguard_fail(out ? *out : nullptr);
}

int omega_ingest_push(omega_ingest* in, const void* bytes, int64_t n_bytes) try {
  if (!in || (!bytes && n_bytes > 0) || n_bytes < 0) return OMEGA_EINVAL;
  IHIP(in, hipSetDevice(in->device));
  const unsigned char* b = static_cast<const unsigned char*>(bytes);
  while (n_bytes > 0) {
    int s;
    if (int e = take_fill_slot(in, &s)) return e;
    omega_ingest::Slot& sl = in->slots[s];
    const size_t take = std::min<size_t>((size_t)n_bytes, in->slot_bytes - sl.fill);
    std::memcpy(sl.h_raw + sl.fill, b, take);
    sl.fill += take;
    b += take;
    n_bytes -= (int64_t)take;
    in->st.bytes_in += (int64_t)take;
    if (sl.fill == in->slot_bytes) {
      if (int e = launch_slot(in, s, in->slot_samples)) return e;
      in->fill_slot = (s + 1) % (int)in->slots.size();
    }
  }
  return 0;
} catch (...) {
  return iguard_fail(in);
}

int omega_ingest_flush(omega_ingest* in) try {
  if (!in) return OMEGA_EINVAL;
  IHIP(in, hipSetDevice(in->device));
  omega_ingest::Slot& sl = in->slots[in->fill_slot];
  if (sl.inflight || sl.fill == 0) return 0;
  // whole frames that make whole capture chunks: a multiple of chunk / gcd(chunk, C) frames
  int g = in->cfg.chunk_size, cc = in->C;
  while (cc) {
    const int r = g % cc;
    g = cc;
    cc = r;
  }
  const size_t unit = (size_t)in->C * in->bps * (size_t)(in->cfg.chunk_size / g);
  const size_t whole = sl.fill / unit * unit;
  if (whole == 0) return 0;
  const size_t rest = sl.fill - whole;
  std::vector<unsigned char> tail(sl.h_raw + whole, sl.h_raw + sl.fill);
  const int s = in->fill_slot;
  if (int e = launch_slot(in, s, (int64_t)(whole / ((size_t)in->C * in->bps)))) return e;
  in->fill_slot = (s + 1) % (int)in->slots.size();
  if (rest) {
    in->st.bytes_in -= (int64_t)rest;  // moved, not new
    return omega_ingest_push(in, tail.data(), (int64_t)rest);
  }
  return 0;
} catch (...) {
  return iguard_fail(in);
}

int omega_ingest_poll(omega_ingest* in, int64_t max_frames, const omega_outputs* out, int wait, int64_t* n_frames_out) try {
  if (!in || !out || max_frames < 0) return OMEGA_EINVAL;
  if (n_frames_out) *n_frames_out = 0;
  IHIP(in, hipSetDevice(in->device));
  int64_t done = 0;
  const int C = in->C, T = in->T, w = in->cfg.want;
  while (!in->queue.empty() && done < max_frames) {
    omega_ingest::Out* ob = in->queue.front();
    if (wait) {
      IHIP(in, hipEventSynchronize(ob->ev_done));
    } else {
      const hipError_t q = hipEventQuery(ob->ev_done);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) return ifail(in, OMEGA_EHIP, "hipEventQuery: %s", hipGetErrorString(q));
    }
    const int64_t take = std::min(ob->n_frames - ob->consumed, max_frames - done);
    const size_t r0 = (size_t)ob->consumed * C, rn = (size_t)take * C, o0 = (size_t)done * C;
    if (out->combined && (w & OMEGA_INGEST_COMBINED))
      std::memcpy(out->combined + o0 * T, ob->h_comb + r0 * T, rn * T * sizeof(float));
    if (out->lufs_inst && (w & OMEGA_INGEST_LUFS)) std::memcpy(out->lufs_inst + o0, ob->h_li + r0, rn * sizeof(float));
    if (out->true_peak_db && (w & OMEGA_INGEST_TRUE_PEAK))
      std::memcpy(out->true_peak_db + o0, ob->h_tp + r0, rn * sizeof(float));
    if (out->meters && (w & OMEGA_INGEST_METERS))
      std::memcpy(out->meters + o0 * OMEGA_N_METERS, ob->h_met + r0 * OMEGA_N_METERS, rn * OMEGA_N_METERS * sizeof(double));
    ob->consumed += take;
    done += take;
    if (ob->consumed == ob->n_frames) {
      in->queue.pop_front();
      in->free_outs.push_back(ob);
    }
  }
  if (n_frames_out) *n_frames_out = done;
  in->st.frames_polled += done;
  return 0;
} catch (...) {
  return iguard_fail(in);
}

int omega_ingest_get_stats(const omega_ingest* in, omega_ingest_stats* out) {
  if (!in || !out) return OMEGA_EINVAL;
  *out = in->st;
  return 0;
}

const char* omega_ingest_last_error(const omega_ingest* in) { return in ? in->err : "null ingest"; }

void omega_ingest_destroy(omega_ingest* in) try {
  if (!in) return;
  (void)hipSetDevice(in->device);
  if (in->comp) (void)hipStreamSynchronize(in->comp);
  if (in->copy) (void)hipStreamSynchronize(in->copy);
  if (in->ctx) {
    (void)omega_synchronize(in->ctx);
    (void)omega_set_stream(in->ctx, nullptr);  // (the context must outlive the ingest)
  }
  for (auto& sl : in->slots) {
    if (sl.h_raw) (void)hipHostFree(sl.h_raw);
    if (sl.ev_h2d) (void)hipEventDestroy(sl.ev_h2d);
  }
  for (omega_ingest::Out* o : in->outs) {
    for (void* p : {(void*)o->h_comb, (void*)o->h_li, (void*)o->h_tp, (void*)o->h_met})
      if (p) (void)hipHostFree(p);
    for (void* p : {(void*)o->d_comb, (void*)o->d_li, (void*)o->d_tp, (void*)o->d_met})
      if (p) (void)hipFree(p);
    if (o->ev_done) (void)hipEventDestroy(o->ev_done);
    delete o;
  }
  for (int k = 0; k < 2; ++k) {
    if (in->d_raw[k]) (void)hipFree(in->d_raw[k]);
    if (in->d_in[k]) (void)hipFree(in->d_in[k]);
    if (in->ev_unpacked[k]) (void)hipEventDestroy(in->ev_unpacked[k]);
  }
  for (void* p : {(void*)in->d_rms, (void*)in->d_zero, (void*)in->d_bg, (void*)in->d_sil})
    if (p) (void)hipFree(p);
  if (in->comp) (void)hipStreamDestroy(in->comp);
  if (in->copy) (void)hipStreamDestroy(in->copy);
  delete in;
} catch (...) {
}

}  // extern "C"
