"""Sustained-stream ingest over libomega.so (omega_ingest_*).

The step before the hot path: the capture's byte stream (omega4/audio/capture.py:546-600: parec
float32le / s16le in fixed chunks, with the per-chunk noise gate of :620-641) and the app's input gain
and ring buffer (omega4_main.py:648-688), fed to the engine's stream layout -- frame f of every channel
covers stream samples [f*hop, f*hop + W). ``push`` only memcpy's bytes into page-locked staging slots;
the H2D copy of each full slot overlaps the analysis of the previous one on the device.

    eng = Engine(NORTHSTAR_RESOLUTIONS, 96000, 20000, target_bins=512, n_channels=8)
    ing = StreamIngest(eng, hop=1024, batch_hops=64)
    for chunk in capture:                 # interleaved float32le bytes (or a numpy array)
        ing.push(chunk)
        res = ing.poll()                  # completed frames so far: dict of [frames * C, ...] arrays
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Dict

import numpy as np

from . import _lib as L
from .engine import Engine


class StreamIngest:
    def __init__(self, engine: Engine, hop: int = 512, batch_hops: int = 64, ring_slots: int = 4,
                 max_pending_batches: int = 64, chunk_size: int = 512, gain: float = 4.0, gate: bool = True, audio_format: str = "float32le",
                 noise_floor: float = 0.001, silence_threshold_seconds: float = 0.25,
                 background_alpha: float = 0.001, want=("combined", "lufs_inst", "true_peak_db", "meters")):
        self.engine = engine
        cfg = L.IngestConfig()
        lib = L.lib()
        lib.omega_ingest_config_default(C.byref(cfg))
        if audio_format not in L.FMT:
            raise ValueError(f"audio_format must be one of {sorted(L.FMT)}")
        cfg.format = L.FMT[audio_format]
        cfg.sample_rate = int(engine.cfg.sample_rate)
        cfg.hop, cfg.batch_hops, cfg.ring_slots, cfg.chunk_size = int(hop), int(batch_hops), int(ring_slots), int(chunk_size)
        cfg.max_pending_batches = int(max_pending_batches)
        cfg.gain = float(gain)
        cfg.gate = 1 if gate else 0
        cfg.noise_floor, cfg.silence_threshold_seconds = float(noise_floor), float(silence_threshold_seconds)
        cfg.background_alpha = float(background_alpha)
        bits = {"combined": L.INGEST_COMBINED, "lufs_inst": L.INGEST_LUFS, "true_peak_db": L.INGEST_TRUE_PEAK,
                "meters": L.INGEST_METERS}
        cfg.want = sum(bits[w] for w in want)
        self.want = tuple(want)
        self.cfg = cfg
        self.C, self.T = engine.C, engine.T
        self.bytes_per_sample = 2 if audio_format == "s16le" else 4
        self._dtype = np.int16 if audio_format == "s16le" else np.float32
        self._h = C.c_void_p()
        engine._ingests.append(weakref.ref(self))
        code = lib.omega_ingest_create(engine._ctx, C.byref(cfg), C.byref(self._h))
        if code != L.OK:
            msg = lib.omega_ingest_last_error(self._h).decode() if self._h else "invalid ingest configuration"
            self.close()
            if code == L.EINVAL:
                raise ValueError(msg)
            raise L.OmegaError(code, msg)

    def _check(self, code):
        if code != L.OK:
            raise L.OmegaError(code, L.lib().omega_ingest_last_error(self._h).decode())

    def push(self, data) -> None:
        """Raw capture bytes (interleaved over the engine's channels) or a numpy array of samples."""
        if isinstance(data, np.ndarray):
            buf = np.ascontiguousarray(data, dtype=self._dtype)
            self._check(L.lib().omega_ingest_push(self._h, buf.ctypes.data, buf.nbytes))
        else:
            mv = memoryview(data).cast("B")
            arr = np.frombuffer(mv, np.uint8)
            self._check(L.lib().omega_ingest_push(self._h, arr.ctypes.data if len(arr) else None, len(arr)))

    def flush(self) -> None:
        self._check(L.lib().omega_ingest_flush(self._h))

    def poll(self, max_frames: int = 1 << 30, wait: bool = False) -> Dict[str, np.ndarray]:
        """Completed frames in order: {'combined': [F*C, T], 'lufs_inst': [F*C], 'true_peak_db': [F*C],
        'meters': [F*C, 5]} (the requested outputs), F <= max_frames."""
        st = self.stats()
        avail = min(int(max_frames), st["frames"] - st["frames_polled"] - st["dropped_frames"])
        n = max(avail, 0)
        o = {}
        if "combined" in self.want:
            o["combined"] = np.empty((n * self.C, self.T), np.float32)
        if "lufs_inst" in self.want:
            o["lufs_inst"] = np.empty(n * self.C, np.float32)
        if "true_peak_db" in self.want:
            o["true_peak_db"] = np.empty(n * self.C, np.float32)
        if "meters" in self.want:
            o["meters"] = np.empty((n * self.C, L.N_METERS), np.float64)
        outs = L.Outputs()
        for k in ("combined", "lufs_inst", "true_peak_db", "meters"):
            setattr(outs, k, o[k].ctypes.data if k in o else None)
        got = C.c_int64(0)
        self._check(L.lib().omega_ingest_poll(self._h, n, C.byref(outs), 1 if wait else 0, C.byref(got)))
        return {k: v[: got.value * self.C] for k, v in o.items()}

    def stats(self) -> Dict[str, int]:
        s = L.IngestStats()
        self._check(L.lib().omega_ingest_get_stats(self._h, C.byref(s)))
        return {f: int(getattr(s, f)) for f, _ in L.IngestStats._fields_}

    def close(self):
        if self._h:
            L.lib().omega_ingest_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
