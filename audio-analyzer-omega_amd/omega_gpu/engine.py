"""Engine: one libomega context (one HIP stream + per-channel meter state) and the batched
entry points. Inputs may be numpy arrays (host memory: the call stages through device buffers and
returns host arrays) or torch tensors on an MI355X (device memory: the call enqueues on torch's
current stream and returns device tensors). torch is used only as a device-memory/stream carrier."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L


@dataclass(frozen=True)
class Resolution:
    """One FFT resolution (FFTConfig, multi_resolution_fft.py:26-44)."""

    freq_range: Tuple[float, float]
    fft_size: int
    hop_size: int
    weight: float
    window: str = "blackman"


DEFAULT_RESOLUTIONS = (  # multi_resolution_fft.py:149-154
    Resolution((20, 200), 4096, 1024, 1.5),
    Resolution((200, 1000), 2048, 512, 1.2),
    Resolution((1000, 5000), 1024, 256, 1.0),
    Resolution((5000, 20000), 1024, 256, 1.5),
)
NORTHSTAR_RESOLUTIONS = (  # BASELINE.json north-star sizes, same ranges/weights
    Resolution((20, 200), 16384, 1024, 1.5),
    Resolution((200, 1000), 8192, 512, 1.2),
    Resolution((1000, 5000), 4096, 256, 1.0),
    Resolution((5000, 20000), 1024, 256, 1.5),
)
METER_KEYS = ("momentary", "short_term", "integrated", "range", "true_peak")


def _is_torch(a) -> bool:
    return hasattr(a, "data_ptr") and hasattr(a, "is_cuda")


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if _is_torch(a):
        return a.data_ptr()
    return a.ctypes.data


class Engine:
    def __init__(self, resolutions: Sequence[Resolution] = DEFAULT_RESOLUTIONS, sample_rate: int = 48000,
                 max_freq: float = 20000, target_bins: int = 1024, frame_size: Optional[int] = None,
                 n_channels: int = 1, apply_weighting: bool = True, device: int = 0,
                 meter_windows: Optional[Sequence[int]] = None):
        self._ctx = C.c_void_p()
        cfg = L.Config()
        lib = L.lib()
        lib.omega_config_default(C.byref(cfg))
        if meter_windows is not None:  # (momentary, short, integrated, peak) window lengths in frames
            cfg.momentary_len, cfg.short_len, cfg.integrated_len, cfg.peak_len = (int(v) for v in meter_windows)
        resolutions = list(resolutions)
        cfg.sample_rate = int(sample_rate)
        cfg.max_freq = float(max_freq)
        cfg.n_res = len(resolutions)
        if not 1 <= cfg.n_res <= L.MAX_RES:
            raise ValueError(f"1..{L.MAX_RES} resolutions supported")
        for i, r in enumerate(resolutions):
            cfg.res[i] = L.Resolution(float(r.freq_range[0]), float(r.freq_range[1]), int(r.fft_size),
                                      int(r.hop_size), float(r.weight), L.WIN.get(r.window, 0))
        cfg.apply_weighting = 1 if apply_weighting else 0
        cfg.target_bins = int(target_bins)
        cfg.frame_size = int(frame_size or max(r.fft_size for r in resolutions))
        cfg.n_channels = int(n_channels)
        self.cfg = cfg
        self.resolutions = tuple(resolutions)
        self.W, self.C, self.T = cfg.frame_size, cfg.n_channels, cfg.target_bins
        self.device = device
        self._ingests = []  # weak references: stream ingests bound to this context, closed before it
        # meter pipelining: the outputs of the last pipelined device call, held until its deferred meter
        # segment is enqueued (the next call, a flush, synchronize, reset or close): the segment writes
        # that call's meters, so their memory must not return to torch's caching allocator before then
        self._pipe = False
        self._held = None
        code = lib.omega_create(C.byref(cfg), int(device), C.byref(self._ctx))
        if code != L.OK:
            msg = lib.omega_last_error(self._ctx).decode()
            lib.omega_destroy(self._ctx)
            self._ctx = C.c_void_p()
            if code == L.EINVAL:
                raise ValueError(msg)
            raise (L.UnsupportedError if code == L.EUNSUP else L.OmegaError)(code, msg)

    # -- lifecycle --
    def close(self):
        for r in getattr(self, "_ingests", ()):
            ing = r()
            if ing is not None:
                ing.close()
        if self._ctx:
            L.lib().omega_destroy(self._ctx)
            self._ctx = C.c_void_p()
        self._held = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, code):
        L.check(self._ctx, code)

    def synchronize(self):
        self._check(L.lib().omega_synchronize(self._ctx))
        self._held = None

    def _bind_stream(self, tensor):
        """Enqueue on torch's current stream of the tensor's device, which must be this context's GPU
        (a pointer on another device would be read by this device's kernels)."""
        import torch
        if not tensor.is_cuda or tensor.device.index != self.device:
            raise ValueError(f"device tensor on {tensor.device}, but this engine runs on cuda:{self.device}")
        self._check(L.lib().omega_set_stream(self._ctx, C.c_void_p(torch.cuda.current_stream(tensor.device).cuda_stream)))

    def check_queues(self) -> bool:
        """Probe this context's stream and side stream again (omega_check_queues): call once other
        components -- an RCCL communicator, another library -- have created their streams. True if the
        two run on independent hardware queues (False: the batch path's device waits run to their
        bound; omega_last_error says so)."""
        shared = C.c_int(0)
        self._check(L.lib().omega_check_queues(self._ctx, C.byref(shared)))
        return shared.value == 0

    def reset_meters(self):
        self._check(L.lib().omega_meter_reset(self._ctx))
        self._held = None  # (the reset enqueued a pending segment first)

    def set_meter_pipelining(self, enable: bool = True):
        """omega_set_meter_pipelining: a batch call's meter aggregates are completed by the next batch
        call's launch (or flush_meters / synchronize) instead of its own (omega.h)."""
        self._check(L.lib().omega_set_meter_pipelining(self._ctx, int(bool(enable))))
        self._pipe = bool(enable)
        if not enable:
            self._held = None

    def flush_meters(self):
        """Enqueue a pending meter segment on the context's stream (omega_flush_meters)."""
        self._check(L.lib().omega_flush_meters(self._ctx))
        self._held = None

    # -- helpers --
    def _alloc(self, like, shape, dtype):
        if _is_torch(like):
            import torch
            tdt = {np.float32: torch.float32, np.float64: torch.float64}[dtype]
            return torch.empty(shape, dtype=tdt, device=like.device)
        return np.empty(shape, dtype=dtype)

    # -- the fused per-channel-frame path --
    def process_stream(self, x, n_samples: int, hop: int, channel_stride: int = 0, **kw) -> Dict:
        """Stream layout (omega_process_stream): one frame per `hop` samples once W samples have
        arrived; channel c at x[c * channel_stride:]. Same keywords and outputs as process_frames."""
        n_frames = 0 if n_samples < self.W else (n_samples - self.W) // hop + 1
        return self.process_frames(x, n_frames, hop, channel_stride, _stream=(n_samples, hop), **kw)

    def process_frames(self, x, n_frames: int, frame_stride: int, channel_stride: int, *, combined=True,
                       lufs=True, true_peak=True, meters=False, mags=False, weighted=False,
                       out: Optional[Dict] = None, _stream=None) -> Dict:
        """Run the hot path over n_frames x n_channels channel-frames of x (flat float32, host numpy
        or device torch). Returns a dict of the requested outputs (numpy or torch, like x)."""
        dev = _is_torch(x)
        if not dev:
            x = np.ascontiguousarray(x, dtype=np.float32)
        ncf = n_frames * self.C
        o = dict(out or {})
        if combined and "combined" not in o:
            o["combined"] = self._alloc(x, (ncf, self.T), np.float32)
        if lufs and "lufs_inst" not in o:
            o["lufs_inst"] = self._alloc(x, (ncf,), np.float32)
        if true_peak and "true_peak_db" not in o:
            o["true_peak_db"] = self._alloc(x, (ncf,), np.float32)
        if meters and "meters" not in o:
            o["meters"] = self._alloc(x, (ncf, L.N_METERS), np.float64)
        if weighted and "weighted" not in o:
            o["weighted"] = self._alloc(x, (ncf, self.W), np.float32)
        if mags:
            sel = range(len(self.resolutions)) if mags is True else mags
            for r in sel:
                o.setdefault(f"mag{r}", self._alloc(x, (ncf, self.resolutions[r].fft_size // 2 + 1), np.float32))
        outs = L.Outputs()
        outs.combined = _ptr(o.get("combined"))
        outs.lufs_inst = _ptr(o.get("lufs_inst"))
        outs.true_peak_db = _ptr(o.get("true_peak_db"))
        outs.meters = _ptr(o.get("meters"))
        outs.weighted = _ptr(o.get("weighted"))
        for r in range(len(self.resolutions)):
            outs.mag[r] = _ptr(o.get(f"mag{r}"))
        if dev:
            self._bind_stream(x)
        mem = L.MEM_DEVICE if dev else L.MEM_HOST
        if _stream is not None:
            got = C.c_int64(0)
            self._check(L.lib().omega_process_stream(self._ctx, _ptr(x), int(_stream[0]), int(_stream[1]),
                                                     int(channel_stride), C.byref(outs), mem, C.byref(got)))
            assert got.value == n_frames
        else:
            self._check(L.lib().omega_process_frames(self._ctx, _ptr(x), int(n_frames), int(frame_stride),
                                                     int(channel_stride), C.byref(outs), mem))
        # the previous pipelined call's segment is enqueued by now (this call, or the flush a non-pipelined
        # call runs first); this call's may be pending: hold its outputs (see __init__)
        self._held = o if (self._pipe and dev and meters) else None
        return o

    def combine(self, mags: Dict[int, np.ndarray], n_cf: int = 1) -> np.ndarray:
        """combine_results_optimized on the device over the given weighted magnitudes."""
        arrs = {i: np.ascontiguousarray(m, dtype=np.float32) for i, m in mags.items()}
        ptrs = (C.c_void_p * L.MAX_RES)()
        for i in range(L.MAX_RES):
            ptrs[i] = arrs[i].ctypes.data if i in arrs else None
        out = np.empty((n_cf, self.T), np.float32)
        self._check(L.lib().omega_combine(self._ctx, ptrs, int(n_cf), out.ctypes.data, L.MEM_HOST))
        return out

    def true_peak(self, x: np.ndarray, oversampling: int = 4) -> np.ndarray:
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        out = np.empty(x.shape[0], np.float32)
        self._check(L.lib().omega_true_peak_os(self._ctx, x.ctypes.data, x.shape[0], x.shape[1], int(oversampling),
                                               out.ctypes.data, L.MEM_HOST))
        return out

    def weighting(self, x: np.ndarray, mode: str = "K", weighted: bool = True):
        """apply_weighting (+ instantaneous LUFS) for n frames [n, m]."""
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        w = np.empty_like(x) if weighted else None
        li = np.empty(x.shape[0], np.float32)
        self._check(L.lib().omega_weighting(self._ctx, x.ctypes.data, x.shape[0], x.shape[1], L.WEIGHT[mode],
                                            w.ctypes.data if w is not None else None, li.ctypes.data, L.MEM_HOST))
        return w, li

    def k_weighting(self, x: np.ndarray, weighted: bool = True):
        return self.weighting(x, "K", weighted)

    def k_weighting_scan(self, x: np.ndarray, weighted: bool = True):
        """The batch path's float32 chunked-scan K-weighting on its own (omega_k_weighting,
        kweight_kernel: power-of-two frames 512..16384) -- what omega_process_frames computes LUFS_inst
        with; ``k_weighting`` / ``weighting`` run scipy's float64 cascade instead."""
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        w = np.empty_like(x) if weighted else None
        li = np.empty(x.shape[0], np.float32)
        self._check(L.lib().omega_k_weighting(self._ctx, x.ctypes.data, x.shape[0], x.shape[1],
                                              w.ctypes.data if w is not None else None, li.ctypes.data, L.MEM_HOST))
        return w, li

    def load_meter_history(self, lufs_inst, tp_db):
        """omega_meter_load_history: the meter state after a stream whose last frames had the LUFS_inst
        rows lufs_inst [n_l, C] and, for the last n_t of them, the true-peak rows tp_db [n_t, C]
        (time order; device torch float32 tensors or host numpy)."""
        if _is_torch(lufs_inst):
            import torch
            li, tp = lufs_inst.contiguous(), tp_db.contiguous()
            if li.dtype != torch.float32 or tp.dtype != torch.float32:
                raise ValueError("load_meter_history: float32 rows")
            if li.numel():
                self._bind_stream(li)
            mem = L.MEM_DEVICE
        else:
            li = np.ascontiguousarray(lufs_inst, dtype=np.float32)
            tp = np.ascontiguousarray(tp_db, dtype=np.float32)
            mem = L.MEM_HOST
        n_l, n_t = li.shape[0] if li.ndim else 0, tp.shape[0] if tp.ndim else 0
        if li.ndim != 2 or li.shape[1] != self.C or (n_t and (tp.ndim != 2 or tp.shape[1] != self.C)):
            raise ValueError(f"load_meter_history: [n, {self.C}] rows")
        self._check(L.lib().omega_meter_load_history(self._ctx, _ptr(li) if n_l else None, int(n_l),
                                                     _ptr(tp) if n_t else None, int(n_t), mem))
        self._held = None  # (the load ran a pending meter segment first)

    def meter_update(self, lufs_inst, tp_db, n_frames: int):
        """The A9 aggregates of n_frames x C injected (LUFS_inst, true peak) values in frame order
        (host numpy, or device torch float32 tensors: then the result is a device tensor too)."""
        if _is_torch(lufs_inst):
            import torch
            li, tp = lufs_inst.contiguous(), tp_db.contiguous()
            if li.dtype != torch.float32 or tp.dtype != torch.float32 or li.numel() != n_frames * self.C \
                    or tp.numel() != n_frames * self.C:
                raise ValueError(f"meter_update: float32 values for {n_frames} x {self.C} channel-frames")
            self._bind_stream(li)
            out = torch.empty((n_frames * self.C, L.N_METERS), dtype=torch.float64, device=li.device)
            self._check(L.lib().omega_meter_update(self._ctx, _ptr(li), _ptr(tp), int(n_frames), _ptr(out),
                                                   L.MEM_DEVICE))
            return out
        li = np.ascontiguousarray(lufs_inst, dtype=np.float32)
        tp = np.ascontiguousarray(tp_db, dtype=np.float32)
        out = np.empty((n_frames * self.C, L.N_METERS), np.float64)
        self._check(L.lib().omega_meter_update(self._ctx, li.ctypes.data, tp.ctypes.data, int(n_frames),
                                               out.ctypes.data, L.MEM_HOST))
        return out

    def calculate_lufs(self, x: np.ndarray, mode: str = "K", oversampling: int = 4):
        """Weighting (LUFS_inst) + true peak + meter aggregates of frames x [n_frames * C, m] in one
        host round trip (omega_calculate_lufs). Returns (lufs_inst [n_cf], tp_db [n_cf], meters [n_cf, 5])."""
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        ncf, m = x.shape
        li = np.empty(ncf, np.float32)
        tp = np.empty(ncf, np.float32)
        met = np.empty((ncf, L.N_METERS), np.float64)
        self._check(L.lib().omega_calculate_lufs(self._ctx, x.ctypes.data, ncf // self.C, m, L.WEIGHT[mode],
                                                 int(oversampling), li.ctypes.data, tp.ctypes.data,
                                                 met.ctypes.data, L.MEM_HOST))
        return li, tp, met

    def rfft(self, x: np.ndarray, window: str = "hann", magnitude=True, complex_out=True):
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        n, m = x.shape
        mag = np.empty((n, m // 2 + 1), np.float32) if magnitude else None
        cp = np.empty((n, m // 2 + 1), np.complex64) if complex_out else None
        self._check(L.lib().omega_rfft(self._ctx, x.ctypes.data, n, m, L.WIN.get(window, 3),
                                       mag.ctypes.data if mag is not None else None,
                                       cp.ctypes.data if cp is not None else None, L.MEM_HOST))
        return mag, cp

    def spectra(self, x, window: str = "hann", bands: Optional["BandTable"] = None, chroma: bool = True,
                mags: bool = False, out: Optional[Dict] = None) -> Dict:
        """Fused cfg3 analysis (omega_spectra) of frames x [n, 8192] (host numpy or device torch):
        'bands' [n, n_out] (A10 without smoothing, needs a MAX BandTable over 4097 bins), 'chroma'
        [n, 12] (A12 before the temporal blend), 'mag' [n, 4097] (A13 magnitude)."""
        dev = _is_torch(x)
        if not dev:
            x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
        n, m = x.shape
        o = dict(out or {})
        if bands is not None and "bands" not in o:
            o["bands"] = self._alloc(x, (n, bands.n_out), np.float32)
        if chroma and "chroma" not in o:
            o["chroma"] = self._alloc(x, (n, 12), np.float64)
        if mags and "mag" not in o:
            o["mag"] = self._alloc(x, (n, m // 2 + 1), np.float32)
        if dev:
            self._bind_stream(x)
        self._check(L.lib().omega_spectra(self._ctx, _ptr(x), n, m, L.WIN.get(window, 1),
                                          bands._h if bands is not None else None, _ptr(o.get("bands")),
                                          _ptr(o.get("chroma")), _ptr(o.get("mag")),
                                          L.MEM_DEVICE if dev else L.MEM_HOST))
        return o

    def drum_features(self, mags, sensitivity: float = 1.0, out=None):
        """Kick + snare spectral features of consecutive magnitude frames of one stream (omega_drum_features):
        [F, 14] float64 in DRUM_COLUMNS order; the stream state carries over to the next call
        (reset_drums starts a new stream). mags: [F, n_bins] float32, host numpy or device torch."""
        dev = _is_torch(mags)
        if not dev:
            mags = np.ascontiguousarray(mags, dtype=np.float32)
        F, n = mags.shape
        o = out if out is not None else self._alloc(mags, (F, 14), np.float64)
        if dev:
            self._bind_stream(mags)
        self._check(L.lib().omega_drum_features(self._ctx, _ptr(mags), int(F), int(n), int(mags.stride(0) if dev else n),
                                                float(sensitivity), _ptr(o), L.MEM_DEVICE if dev else L.MEM_HOST))
        return o

    def reset_drums(self):
        self._check(L.lib().omega_drum_reset(self._ctx))

    def chroma_raw(self, spec: np.ndarray, df: float) -> np.ndarray:
        s = np.ascontiguousarray(np.atleast_2d(spec), dtype=np.float32)
        out = np.empty((s.shape[0], 12), np.float64)
        self._check(L.lib().omega_chroma(self._ctx, s.ctypes.data, s.shape[0], s.shape[1], float(df),
                                         out.ctypes.data, L.MEM_HOST))
        return out


class BandTable:
    """A device band table bound to an engine (omega_bands_*)."""

    def __init__(self, engine: Engine, op: int, starts, ends, n_out: int, n_bins: int, scale=None, bin_scale=None):
        self.engine = engine
        s = np.ascontiguousarray(starts, dtype=np.int32)
        e = np.ascontiguousarray(ends, dtype=np.int32)
        sc = None if scale is None else np.ascontiguousarray(scale, dtype=np.float64)
        bs = None if bin_scale is None else np.ascontiguousarray(bin_scale, dtype=np.float64)
        self.n_out, self.n_bins = int(n_out), int(n_bins)
        self._h = C.c_void_p()
        engine._check(L.lib().omega_bands_create(engine._ctx, op, s.ctypes.data, e.ctypes.data, len(s), self.n_out,
                                                 sc.ctypes.data if sc is not None else None,
                                                 bs.ctypes.data if bs is not None else None, self.n_bins,
                                                 C.byref(self._h)))

    def apply(self, spec: np.ndarray) -> np.ndarray:
        s = np.ascontiguousarray(np.atleast_2d(spec), dtype=np.float32)
        if s.shape[1] != self.n_bins:
            raise ValueError(f"band table built for {self.n_bins} bins, got {s.shape[1]}")
        out = np.empty((s.shape[0], self.n_out), np.float32)
        self.engine._check(L.lib().omega_bands_apply(self.engine._ctx, self._h, s.ctypes.data, s.shape[0],
                                                     s.shape[1], out.ctypes.data, L.MEM_HOST))
        return out

    def __del__(self):
        try:
            if self._h:
                L.lib().omega_bands_destroy(self._h)
        except Exception:
            pass
