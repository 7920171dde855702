/*
 * omega.h -- C ABI of libomega.so, the MI355X (gfx950) engine for the OMEGA-4 per-frame audio
 * analysis hot path: multi-resolution windowed R2C FFT + psychoacoustic weighting + interpolated
 * combine, K-weighted LUFS (zero-phase biquads), 4x true peak, the per-stream meter aggregates,
 * perceptual/mel band reductions and chromagram binning.
 *
 * Each entry point replaces one reference Python surface (reference repo paths, file:line):
 *
 *   omega_process_frames   MultiResolutionFFT.process_audio_chunk     omega4/audio/multi_resolution_fft.py:228-302
 *                          + combine_results_optimized                 multi_resolution_fft.py:335-408
 *                          + ProfessionalMetering.calculate_lufs       omega4/panels/professional_meters.py:231-281
 *                          (batched over channel-frames; the reference calls these once per display frame,
 *                           omega4_main.py:707-717 and professional_meters.py:348-351)
 *   omega_process_stream   the same over the stream layout: frame f = samples [f*hop, f*hop + W) of one
 *                          buffer per channel (the CircularBuffer.read_latest(N) view of :52-133 once
 *                          W samples have arrived)
 *   omega_combine          combine_results_optimized                   multi_resolution_fft.py:335-408
 *   omega_true_peak        ProfessionalMetering.calculate_true_peak    professional_meters.py:283-299
 *   omega_true_peak_os     calculate_true_peak(x, oversampling)         professional_meters.py:283-299
 *   omega_k_weighting      ProfessionalMetering.apply_k_weighting      professional_meters.py:129-153
 *                          (+ the instantaneous LUFS of calculate_lufs :236-246)
 *   omega_meter_*          the momentary/short-term/integrated/range/true-peak deques  professional_meters.py:19-25, :248-279
 *   omega_bands_*          AudioProcessingPipeline.map_to_bands       omega4/audio/pipeline.py:295-335 (max-reduce)
 *                          PrecomputedFrequencyMapper.map_spectrum_to_bars omega4/optimization/freq_mapper.py:165-196 (mean-reduce)
 *   omega_chroma           ChromagramAnalyzer.compute_chromagram      omega4/panels/chromagram.py:109-159
 *   omega_rfft             BatchedFFTProcessor process_batch (CPU/CuPy branches) omega4/optimization/batched_fft_processor.py:148-285
 *   omega_spectra          omega_rfft -> omega_bands_apply (MAX) + omega_chroma fused in one pass (cfg3)
 *   omega_drum_features    EnhancedKickDetector / EnhancedSnareDetector band flux, adaptive thresholds and
 *                          spectral centroid  omega4/analyzers/drum_detection.py:47-103, :212-305 (§8(f) row 1)
 *   omega_weighting        ProfessionalMetering.apply_weighting (K / A / C / Z) professional_meters.py:74-229
 *   omega_calculate_lufs   ProfessionalMetering.calculate_lufs (weighting + TP + aggregates) professional_meters.py:231-281
 *                          at scipy's float64 precision, any frame length above filtfilt's padlen
 *   omega_post_*           the app's spectrum post-processing          omega4_main.py:748-1056 (§8(f) row 2)
 *   omega_vu_*             VUMetersPanel.update ballistics             omega4/panels/vu_meters.py:55-99 (§8(f) row 2)
 *   omega_ingest_*         capture chunks -> ring -> analysis          omega4/audio/capture.py:512-600,
 *                          omega4_main.py:648-688 (§8(f) row 3)
 *   omega_transients       TransientAnalyzer.analyze_transients        omega4/analyzers/transient.py:19-108 (§8(f) row 4)
 *
 * Conventions:
 *   - every function returns 0 on success and a negative omega_status on error; the message is
 *     available from omega_last_error(ctx). No C++ exception and no abort crosses the ABI.
 *   - all buffers are caller-owned. `mem` says whether the data pointers are host (OMEGA_MEM_HOST:
 *     the call stages through context-owned device buffers and returns when outputs are in host
 *     memory) or device (OMEGA_MEM_DEVICE: the call enqueues on the context stream and returns
 *     immediately; synchronize with omega_synchronize).
 *   - one context per host thread (contexts own a HIP stream and the per-channel meter state);
 *     a context is not internally locked.
 *   - channel-frame index cf = f * n_channels + c; input sample n of channel-frame (f, c) lives at
 *     x[f * frame_stride + c * channel_stride + n] (materialized layout: frame_stride = C*W,
 *     channel_stride = W; stream layout with hop H over planar channels: frame_stride = H,
 *     channel_stride = samples per channel).
 */
#ifndef OMEGA_H
#define OMEGA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMEGA_ABI_VERSION 3
#define OMEGA_MAX_RES 4
#define OMEGA_N_METERS 5 /* momentary, short_term, integrated, range, true_peak */

typedef enum {
  OMEGA_OK = 0,
  OMEGA_EINVAL = -1,  /* bad argument / config (the reference raises ValueError) */
  OMEGA_EHIP = -2,    /* HIP runtime error */
  OMEGA_ENOMEM = -3,
  OMEGA_EUNSUP = -4   /* valid for the reference, not supported by this build (e.g. a batch frame size W
                         that is not a power of two 512..16384) */
} omega_status;

typedef enum { OMEGA_MEM_HOST = 0, OMEGA_MEM_DEVICE = 1 } omega_mem;

typedef enum {
  OMEGA_WIN_BLACKMAN = 0, /* np.blackman, multi_resolution_fft.py:177-178 */
  OMEGA_WIN_HANN = 1,     /* np.hanning, batched_fft_processor.py:94 */
  OMEGA_WIN_HAMMING = 2,  /* np.hamming */
  OMEGA_WIN_RECT = 3      /* ones */
} omega_window;

/* One FFT resolution: FFTConfig (multi_resolution_fft.py:26-44). */
typedef struct {
  double freq_lo, freq_hi; /* inclusive range [lo, hi] in Hz */
  int32_t fft_size;        /* power of two, 2..frame_size (below 512: mrfft_small_kernel) */
  int32_t hop_size;        /* kept for fidelity (CircularBuffer sizing); the frame API is stateless */
  double weight;           /* base psychoacoustic weight and combine weight */
  int32_t window;          /* omega_window */
} omega_resolution;

typedef struct {
  int32_t sample_rate;     /* fs */
  double max_freq;         /* combine grid top: min(max_freq, fs/2) (multi_resolution_fft.py:146) */
  int32_t n_res;           /* 1..OMEGA_MAX_RES */
  omega_resolution res[OMEGA_MAX_RES];
  int32_t apply_weighting; /* process_audio_chunk(apply_weighting=...) */
  int32_t target_bins;     /* T of combine_results_optimized, 2..4096 */
  int32_t frame_size;      /* W = metering window M: power of two 512..16384 */
  int32_t n_channels;      /* independent streams; one meter state each */
  double gate_lufs;        /* -70 (professional_meters.py:36) */
  int32_t momentary_len, short_len, integrated_len, peak_len; /* 24, 180, 3600, 60 (:20-25) */
} omega_config;

/* Per-call outputs; any pointer may be NULL to skip that stage. */
typedef struct {
  float* combined;              /* [n_cf, T] combine_results_optimized magnitude */
  float* lufs_inst;             /* [n_cf] instantaneous K-weighted LUFS (-100 when silent) */
  float* true_peak_db;          /* [n_cf] calculate_true_peak (dBTP, -100 when silent) */
  double* meters;               /* [n_cf, 5] calculate_lufs dict values; advances the meter state */
  float* mag[OMEGA_MAX_RES];    /* [n_cf, N_r/2+1] weighted magnitude per resolution (full-magnitude mode) */
  float* weighted;              /* [n_cf, W] K-weighted signal (apply_k_weighting) */
} omega_outputs;

typedef struct omega_ctx omega_ctx;

/* Reference defaults: the four resolutions of multi_resolution_fft.py:149-154, fs 48000,
 * max_freq 20000, T 1024, W 4096, one channel, gate/deques of professional_meters.py:20-36. */
void omega_config_default(omega_config* cfg);

int omega_create(const omega_config* cfg, int device, omega_ctx** out);
void omega_destroy(omega_ctx* ctx);
const char* omega_last_error(const omega_ctx* ctx);
const char* omega_version(void);
/* Enqueue on a caller-owned hipStream_t (NULL = the null/default stream, e.g. PyTorch's default
 * stream). Contexts start on a private non-blocking stream. Switching streams orders the new stream
 * (and the context's side stream) after the work already enqueued on the old one, once.
 *
 * Concurrency precondition of the default layout (omega_set_graphs): the batch kernel on this stream
 * and the meter prep on the context's side stream wait for each other through device counters, so the
 * two must be able to run at once. Each context owns two streams (its private one and the side stream;
 * a graph-capture stream only once graphs are enabled); HIP maps streams onto GPU_MAX_HW_QUEUES
 * hardware queues per process. omega_create and every stream switch here probe the pair (a waiter on
 * the side stream that must see a value stored by a kernel enqueued after it on this stream) and, on a
 * shared queue, move the side stream to a new one (the next queue), up to three times (each distinct
 * stream once; omega_check_queues re-probes). Should that fail,
 * or another tenant hold every CU, the wait is bounded (OMEGA_POLL_LIMIT polls): that call's meter
 * aggregates may be stale and OMEGA_EHIP is returned -- by the call itself for host memory, by the
 * next call or omega_synchronize for device memory. Layouts other than 0 order the side stream by
 * events and carry no such condition (but serialise on a shared queue). A stream switch synchronises
 * both streams once (the probe). */
int omega_set_stream(omega_ctx* ctx, void* hip_stream);
/* Probe the context's stream and its side stream again, whatever was probed before (a stream switch
 * probes each distinct stream once): streams created since -- an RCCL communicator's, another library's
 * -- may share a hardware queue with the side stream. Moves the side stream as omega_set_stream does;
 * *shared (optional) = 1 if no independent queue was found (the device waits then run to their bound;
 * omega_last_error says so), else 0. Synchronises both streams (a pending meter segment launches
 * first). Not part of the reference surface: the multi-GPU host calls it once its collectives exist. */
int omega_check_queues(omega_ctx* ctx, int* shared);
/* flags: bit 0 = HIP graphs: device-memory omega_process_frames calls are captured once per distinct
 * argument set and replayed afterwards (default off: measured slower than direct launches on MI355X,
 * see DESIGN.md); bits 1-2 = stream layout:
 * 0 default: 16384-sample frames on direct launches run as ONE batch kernel (K-weighting, true peak,
 * every resolution and -- up to 2048 frames per channel -- the meter aggregates as workgroup roles of
 * one grid) with the meter prep on a side stream ordered by device counters instead of stream events;
 * other calls (and graph capture) as below;
 * any other value: the full-chip kernels back to back on the stream, the latency-bound meter prep and
 * LUFS query kernels on a side stream joined by events. Every layout gives the same outputs bitwise. */
int omega_set_graphs(omega_ctx* ctx, int flags);
/* The stream calls enqueue on (omega_set_stream), and the context's configuration and device. */
void* omega_get_stream(const omega_ctx* ctx);
int omega_get_config(const omega_ctx* ctx, omega_config* cfg, int* device);
/* Waits for the work enqueued on the context's stream (a pending meter segment launched first). */
int omega_synchronize(omega_ctx* ctx);

/* Meter pipelining (default off; ABI 3). When on, a direct device-memory omega_process_frames /
 * omega_process_stream call on the default layout with meters (up to 2048 frames per channel) leaves
 * its meter aggregates (out->meters) PENDING: the next such call's one batch launch computes them
 * first in its grid -- their inputs are complete once that batch starts -- instead of this launch
 * ending with them, so consecutive calls overlap the meters of one with the transforms of the next.
 * Every other output of a call is complete when its stream work is, as always; its meters are complete
 * when the stream work of the NEXT call, omega_flush_meters or omega_synchronize is. Any other use of
 * the meter state (omega_meter_update / omega_meter_reset / omega_calculate_lufs, a host-memory,
 * graph or other-layout call, omega_set_stream, omega_set_graphs, disabling pipelining,
 * omega_destroy) launches a pending segment first, on the stream of its batch. The caller keeps the
 * pending call's meters buffer alive and unwritten until then (the segment writes it). The segment
 * and the meter prep read the batch's LUFS_inst / true-peak values from the context's own staging
 * (two sets in turn), never from the caller's lufs_inst / true_peak_db buffers, which are free to be
 * reused by the next call as soon as this call's stream work completes (they receive copies).
 * Outputs are bitwise those of the default. In this mode the batch kernel never waits for the side
 * stream (the meter prep follows it there behind a stream wait on the batch's last workgroup; only the
 * next launch's meter segment waits for the prep). */
int omega_set_meter_pipelining(omega_ctx* ctx, int enable);
/* Enqueue a pending meter segment now (no-op without one); complete with the stream's work. */
int omega_flush_meters(omega_ctx* ctx);

/* The fused per-channel-frame hot path over n_frames x n_channels frames of W samples. */
int omega_process_frames(omega_ctx* ctx, const float* x, int64_t n_frames, int64_t frame_stride,
                         int64_t channel_stride, const omega_outputs* out, int mem);

/* Stream layout: n_samples per channel (channel c at x + c*channel_stride), one frame per hop
 * samples once a full window has arrived: n_frames = n_samples < W ? 0 : (n_samples - W)/hop + 1,
 * frame f = x[f*hop, f*hop + W). hop must be even; *n_frames_out (may be NULL) receives the count. */
int omega_process_stream(omega_ctx* ctx, const float* x, int64_t n_samples, int32_t hop, int64_t channel_stride,
                         const omega_outputs* out, int mem, int64_t* n_frames_out);

/* combine_results_optimized over externally supplied weighted magnitudes; mags[r] may be NULL
 * (resolution absent from the results dict). out: [n_cf, T]. */
int omega_combine(omega_ctx* ctx, const float* const* mags, int64_t n_cf, float* out, int mem);

/* calculate_true_peak(x, 4) for n frames of length m (power of two 512..16384), contiguous. */
int omega_true_peak(omega_ctx* ctx, const float* x, int64_t n, int32_t m, float* out_db, int mem);
/* calculate_true_peak(x, oversampling) (professional_meters.py:283-299) for oversampling 1, 2 or 4:
 * max |resample(x, oversampling * m)| over the phases n + p / oversampling; other factors return
 * OMEGA_EUNSUP. n frames of any length m >= 1, contiguous: powers of two 512..16384 on the
 * register-FFT / Stockham kernels, every other length on the mixed-radix transform (anyfft.hip). */
int omega_true_peak_os(omega_ctx* ctx, const float* x, int64_t n, int32_t m, int32_t oversampling, float* out_db,
                       int mem);

/* apply_k_weighting for n frames of length m (power of two 512..16384): weighted [n, m] (may be
 * NULL) and the instantaneous LUFS [n] (may be NULL). */
int omega_k_weighting(omega_ctx* ctx, const float* x, int64_t n, int32_t m, float* weighted,
                      float* lufs_inst, int mem);

/* apply_weighting + instantaneous LUFS for a weighting mode (professional_meters.py:220-229):
 * K (0, :129-153), A (1, :155-192: four cascaded Butterworth filtfilt sections, x 2.5), C (2, :194-218:
 * two sections) and Z (3: the signal itself, no gate). The A and C coefficients are built for the
 * context's sample rate (create_a/c_weighting_filter, :74-127). */
typedef enum { OMEGA_WEIGHT_K = 0, OMEGA_WEIGHT_A = 1, OMEGA_WEIGHT_C = 2, OMEGA_WEIGHT_Z = 3 } omega_weighting_mode;
int omega_weighting(omega_ctx* ctx, const float* x, int64_t n, int32_t m, int32_t mode, float* weighted,
                    float* lufs_inst, int mem);

/* Meter aggregates from precomputed instantaneous values: feeds n_frames x n_channels values
 * (cf-major) through the per-channel state and writes meters [n_cf, 5]. */
int omega_meter_update(omega_ctx* ctx, const float* lufs_inst, const float* tp_db, int64_t n_frames,
                       double* meters, int mem);
int omega_meter_reset(omega_ctx* ctx);
/* The meter state of a stream whose last n_l frames had the instantaneous LUFS lufs_inst [n_l, C] and
 * whose last n_t of them (n_t <= n_l) the true peaks tp_db [n_t, C] (time order, frame-major), the next
 * frame following them: what omega_meter_reset + omega_meter_update over those n_l frames (the true
 * peaks of the n_l - n_t older ones -100 dBTP) leave, written by one kernel without computing their
 * aggregates (a time-sharded stream's rank loads the history before its shard; SURVEY §8(e),
 * omega_gpu/dist.py meter_time_shard). Rows beyond the windows (n_l > integrated_len - 1, n_t >
 * peak_len - 1) are older than anything the state keeps: the last ones are used. Replaces the reference's deques
 * (professional_meters.py:20-25) filled by calculate_lufs calls. */
int omega_meter_load_history(omega_ctx* ctx, const float* lufs_inst, int64_t n_l, const float* tp_db, int64_t n_t,
                             int mem);

/* ProfessionalMetering.calculate_lufs (professional_meters.py:231-281) in one call: weighting `mode`
 * (LUFS_inst only, as omega_weighting), calculate_true_peak(x, oversampling) (as omega_true_peak_os)
 * and the meter aggregates (as omega_meter_update) for n_frames x n_channels channel-frames of length
 * m (frame-major, contiguous), with one host round trip when mem = OMEGA_MEM_HOST (the three entry
 * points each stage, launch and synchronize on their own). lufs_inst / tp_db may be NULL (device
 * scratch), meters [n_cf, 5] is required. The true peak runs on the context's side stream beside the
 * weighting; for power-of-two frame lengths it counts in on a device counter that the aggregates
 * poll (bounded, OMEGA_EHIP on expiry), so the caller's stream joins the side stream by an event only
 * when other meter work went there since the last call. Outputs are bitwise those of the three calls. */
int omega_calculate_lufs(omega_ctx* ctx, const float* x, int64_t n_frames, int32_t m, int32_t mode,
                         int32_t oversampling, float* lufs_inst, float* tp_db, double* meters, int mem);

/* ---- band reductions (A10/A11) ---- */
typedef struct omega_bands omega_bands;
typedef enum { OMEGA_BANDS_MAX = 0, OMEGA_BANDS_MEAN = 1 } omega_band_op;
/* n_bands bands [starts[i], ends[i]) over spectra of n_bins bins. MAX: out[i] = max(spec[s:e]) *
 * scale[i] (pipeline.py:313-324); MEAN: out[i] = mean((spec*bin_scale)[s:e]) (freq_mapper.py:180-194).
 * scale / bin_scale may be NULL (ones). Bands whose end exceeds n_bins are 0 (MAX) or stop the
 * table (MEAN, freq_mapper.py:188-189), exactly as the reference. */
int omega_bands_create(omega_ctx* ctx, int op, const int32_t* starts, const int32_t* ends,
                       int32_t n_bands, int32_t n_out, const double* scale, const double* bin_scale,
                       int32_t n_bins, omega_bands** out);
void omega_bands_destroy(omega_bands* b);
int omega_bands_apply(omega_ctx* ctx, omega_bands* b, const float* spec, int64_t n, int64_t spec_stride,
                      float* out, int mem);

/* ---- chromagram (A12) over n spectra of n_bins bins with uniform rfftfreq spacing df ---- */
int omega_chroma(omega_ctx* ctx, const float* spec, int64_t n, int32_t n_bins, double df,
                 double* out_raw, int mem);

/* ---- windowed R2C FFT (A13): magnitude [n, m/2+1] and/or complex [n, m/2+1] (interleaved) ---- */
int omega_rfft(omega_ctx* ctx, const float* x, int64_t n, int32_t m, int32_t window, float* mag,
               float* cplx, int mem);

/* ---- fused spectrum analysis (BASELINE cfg3): per frame of m samples (m = 8192), the windowed
 * rfft magnitude (A13), the log-band max of a MAX band table (A10, before smoothing; bands may be
 * NULL) and the chromagram before its temporal blend (A12, bins at df = sample_rate / m), reading
 * each frame once. Any output may be NULL: bands_out [n, n_out], chroma_out [n, 12], mag_out
 * [n, m/2+1]. Replaces the BatchedFFTProcessor -> map_to_bands / compute_chromagram chain
 * (batched_fft_processor.py:148-285, pipeline.py:295-335, chromagram.py:109-159). ---- */
/* Drum-detection spectral features of consecutive magnitude frames of ONE stream (SURVEY.md §8(f)
 * row 1) -- replaces the per-frame feature part of omega4/analyzers/drum_detection.py
 * EnhancedKickDetector.detect_kick_onset :80-103 (calculate_band_flux :47-67,
 * calculate_adaptive_threshold :69-78) and EnhancedSnareDetector.detect_snare_onset :268-305
 * (calculate_multi_band_flux :231-266, calculate_spectral_centroid :212-229); the onset decisions read
 * the wall clock and stay with the caller. mag: n_frames rows of n_bins float32 magnitudes, row
 * stride mag_stride floats. out: [n_frames, 14] float64 = kick sub/body/click flux, kick sub/body/click
 * threshold, snare fundamental/body/snap/rattle flux, snare fundamental/body/snap threshold, snare
 * spectral centroid (Hz). The context keeps the stream state (previous frame, 21-deep flux histories)
 * across calls; omega_drum_reset starts a new stream. n_bins is fixed per context. */
int omega_drum_features(omega_ctx* ctx, const float* mag, int64_t n_frames, int32_t n_bins, int64_t mag_stride,
                        double sensitivity, double* out, int mem);
int omega_drum_reset(omega_ctx* ctx);

/* App spectrum post-processing of combined spectra -- replaces the per-frame
 * part of omega4_main.ProfessionalLiveAudioAnalyzer after combine_results_optimized:
 * process_multi_resolution_fft :748-752 (equal-loudness curve, bass boost), update_content_type
 * :805-840, process_audio_spectrum :991-1056 (98th-percentile normalisation,
 * apply_frequency_compensation :855-926, optional max normalisation, band means -> sqrt -> clamp,
 * frequency-dependent band EMA). omega_post_configure uploads the host-built tables (host memory):
 * curve[T] equal-loudness by position, bass[T] (combine frequency < 250 Hz), comp_instr / comp_vocal
 * [T] compensation factors, vocal_sup[T], ranges {bass_end, vocal_start, vocal_end, high_start},
 * the percentile's sorted ranks and float32 gamma, bands [n_bands] (start, end) already truncated
 * as the reference's loop does, band_smooth[n_bands] = the EMA factor f of each band (in [0, 1]).
 * omega_post_process (device memory only): n_frames spectra at row stride `stride` -> spectrum_out
 * [n, T] float32, bands_out [n, n_bands] float64 (after the EMA, which runs across frames in order and
 * across calls), content_out [n] (0 instrumental, 1 vocal, 2 bass-heavy; may be NULL). flags:
 * OMEGA_POST_*. Bands are numpy's values bit for bit: a frame's band list is float32, or float64 when
 * a band clamps to the Python int 1 (:1034: max(0, min(1, v)) returns the int), and the EMA
 * (:1041-1054) runs in the dtypes numpy gives each term -- bands_out holds both exactly. (A frame
 * whose every band clamps would make numpy's array int64; after the 98th-percentile normalisation
 * to 0.8 no frame reaches that.) */
enum {
  OMEGA_POST_PSYCHO = 1,      /* equal-loudness curve + bass boost */
  OMEGA_POST_FREQ_COMP = 2,   /* apply_frequency_compensation */
  OMEGA_POST_NORMALIZE = 4,   /* final max normalisation */
  OMEGA_POST_SMOOTH = 8       /* band EMA */
};
int omega_post_configure(omega_ctx* ctx, int32_t n_bins, const double* curve, const uint8_t* bass,
                         const float* comp_instr, const float* comp_vocal, const float* vocal_sup,
                         const int32_t* ranges, int32_t p_lo, int32_t p_hi, float p_gamma,
                         const int32_t* band_start, const int32_t* band_end, const double* band_smooth,
                         int32_t n_bands);
int omega_post_process(omega_ctx* ctx, const float* spectra, int64_t n_frames, int64_t stride, int32_t flags,
                       float bass_boost, float* spectrum_out, double* bands_out, int32_t* content_out);
int omega_post_reset(omega_ctx* ctx);
int omega_spectra(omega_ctx* ctx, const float* x, int64_t n, int32_t m, int32_t window, omega_bands* bands,
                  float* bands_out, double* chroma_out, float* mag_out, int mem);


/* VU meter ballistics, VUMetersPanel.update (omega4/panels/vu_meters.py:55-99), for n_updates
 * consecutive update(audio, dt) calls of every channel (one stream each; the reference duplicates its
 * mono input into L and R): update u of channel c reads chunk samples at x + u*update_stride +
 * c*channel_stride (float32, or float64 when f64 != 0 -- the app passes its float64 windowed frame);
 * dt[n_updates] in seconds. out [n_updates, C, 3] float64: the VU level (dBFS + 18 over the last
 * int(0.3 fs) samples, -60 + 18 when silent), the damped display value and the peak hold. The sample
 * history and the needle state carry over between calls; omega_vu_reset starts over. */
int omega_vu_update(omega_ctx* ctx, const void* x, int32_t f64, int64_t n_updates, int32_t chunk, int64_t update_stride,
                    int64_t channel_stride, const double* dt, double* out, int mem);
int omega_vu_reset(omega_ctx* ctx);

/* TransientAnalyzer.analyze_transients (omega4/analyzers/transient.py:19-108) for n_frames frames of
 * n samples (any n >= 64, as the reference; float32, or float64 when f64 != 0), frame f at x + f*frame_stride,
 * in float64 like scipy: Hilbert envelope, Savitzky-Golay (21, 3) smoothing, attack points where the
 * envelope's derivative exceeds twice its standard deviation. out [n_frames, 6] float64:
 * transients_detected, attack_time (ms), punch_factor, envelope_peak, envelope_rms and the smoothed
 * envelope's mean (the value the reference appends to its envelope_history). */
int omega_transients(omega_ctx* ctx, const void* x, int32_t f64, int64_t n_frames, int32_t n, int64_t frame_stride,
                     double* out, int mem);

/* ---- Sustained-stream ingest ------------------------------------------
 * The capture byte stream of omega4/audio/capture.py:546-600 (parec float32le / s16le, fixed chunks
 * of chunk_size samples, s16 scaled by 1/32768), its per-chunk noise gate (:620-641: RMS, background
 * EMA, silence counter -> zeros) and the app's input gain + ring buffer (omega4_main.py:648-688),
 * feeding omega_process_stream: frame f of every channel covers stream samples [f*hop, f*hop + W).
 * Bytes are interleaved over the context's n_channels. The gate works as the reference's capture
 * loop does for any channel count: a chunk is chunk_size interleaved samples (capture.py:549-550,
 * chunk_size / C frames), one RMS over all its channels, one background level and one silence
 * counter (+chunk_size per quiet chunk) for the stream, a gated chunk zeroes every channel of it.
 * The gate's float32 arithmetic is numpy >= 2's (NEP 50: a Python float times a float32 scalar stays
 * float32; the golden vectors were recorded with numpy 2.2.6). omega_ingest_push memcpy's them into
 * page-locked staging slots; each full slot (batch_hops * hop samples per channel) is copied to the
 * device on a copy stream and analysed on the ingest's compute stream (bound to the context with
 * omega_set_stream; destroy the ingest before the context, and before using the context directly
 * again), overlapping the next slot's copy. push blocks only while the slot it fills is still being
 * copied to the device. Results come back through omega_ingest_poll in frame order; when
 * max_pending_batches batches wait unpolled, the oldest one's frames are dropped and counted (the
 * capture buffer's drop policy, capture.py:579-580). */
typedef enum { OMEGA_FMT_F32LE = 0, OMEGA_FMT_S16LE = 1 } omega_sample_format;
enum { OMEGA_INGEST_COMBINED = 1, OMEGA_INGEST_LUFS = 2, OMEGA_INGEST_TRUE_PEAK = 4, OMEGA_INGEST_METERS = 8 };

typedef struct {
  int32_t format;                   /* omega_sample_format */
  int32_t sample_rate;              /* for the gate's silence threshold (capture.py:227) */
  int32_t hop;                      /* frame hop H, multiple of 4 */
  int32_t batch_hops;               /* hops per device batch; batch_hops * hop * n_channels % chunk_size == 0 */
  int32_t ring_slots;               /* page-locked input staging slots, >= 2 */
  int32_t max_pending_batches;      /* result blocks kept until polled (>= 2); beyond, the oldest drop */
  int32_t chunk_size;               /* capture chunk (noise-gate block), 1..8192 (capture.py:28, :64) */
  float gain;                       /* input_gain (omega4_main.py:152, :660) */
  int32_t gate;                     /* apply the capture noise gate */
  double noise_floor;               /* 0.001 (capture.py:36) */
  double silence_threshold_seconds; /* 0.25 */
  double background_alpha;          /* 0.001 */
  int32_t want;                     /* OMEGA_INGEST_* outputs */
} omega_ingest_config;

typedef struct {
  int64_t bytes_in, batches, frames, frames_polled, dropped_frames;
} omega_ingest_stats;

typedef struct omega_ingest omega_ingest;

void omega_ingest_config_default(omega_ingest_config* cfg);
/* On an error after allocation *out is set: read omega_ingest_last_error, then omega_ingest_destroy. */
int omega_ingest_create(omega_ctx* ctx, const omega_ingest_config* cfg, omega_ingest** out);
int omega_ingest_push(omega_ingest* in, const void* bytes, int64_t n_bytes);
/* Analyse the whole capture chunks buffered so far in whole frames (the rest stays buffered). */
int omega_ingest_flush(omega_ingest* in);
/* Up to max_frames completed frames (per channel) in frame order into host buffers laid out like
 * omega_outputs ([frames * C, T], [frames * C], [frames * C, 5]; NULL pointers skip); wait != 0
 * blocks until the launched batches are done. */
int omega_ingest_poll(omega_ingest* in, int64_t max_frames, const omega_outputs* out, int wait, int64_t* n_frames_out);
int omega_ingest_get_stats(const omega_ingest* in, omega_ingest_stats* out);
const char* omega_ingest_last_error(const omega_ingest* in);
void omega_ingest_destroy(omega_ingest* in);

#ifdef __cplusplus
}
#endif
#endif /* OMEGA_H */
