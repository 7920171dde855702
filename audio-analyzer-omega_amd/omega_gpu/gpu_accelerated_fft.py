"""GPUAcceleratedFFT over libomega.so (omega4/optimization/gpu_accelerated_fft.py:22-370).

The reference's CuPy class (still called by optimization/parallel_panel_updater.py:242-250 and by
its own benchmark) with the same names, arguments and return shapes, on the MI355X:

  compute_fft(audio, window_type, return_complex)   :92-177  window * audio -> rfft -> |.|
  compute_multi_resolution_fft(audio, {name: N}, w) :179-226 last N samples (zero-padded at the end
                                                             when shorter), freqs for 48 kHz (:213)
  prepare_batch_arrays(B, N) / process_fft_batch(x) :286-340 device batch in, device complex out

The window is numpy's (np.hanning / np.hamming / else np.blackman, cast to float32, :59-63,
:113-125) and the transform runs in float32 on the device for every input dtype (the reference's CPU
branch follows a float64 input's dtype; its CuPy branch casts to float32 like this one). The
reference's result cache is kept as it is: keyed by (length, window, first 100 bytes of the input),
ten entries, oldest evicted first (:103-111, :163-174) -- two inputs that share their first 100 bytes
get the first one's spectrum, as in the reference. Every length runs on the device: powers of two
512-16384 on the radix-16 / Stockham kernels, the others on the mixed-radix transform (anyfft.hip).
"""
from __future__ import annotations

import ctypes as C
import logging
import threading
from typing import Any, Dict, Optional, Tuple

import numpy as np

from . import _lib as L
from .engine import Engine, Resolution, _is_torch

logger = logging.getLogger(__name__)
_SIZES = (512, 1024, 2048, 4096, 8192, 16384)


def _supported(n: int) -> bool:
    return n >= 1


class GPUAcceleratedFFT:
    def __init__(self, max_fft_size: int = 16384, device: int = 0):
        self.max_fft_size = max_fft_size
        self.gpu_available = True
        self.fft_cache: Dict[tuple, Dict[str, Any]] = {}
        self.cache_lock = threading.Lock()
        self.device = device
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], 48000, 20000, target_bins=2, frame_size=512,
                           device=device)
        self.windows = {name: {n: fn(n).astype(np.float32) for n in _SIZES}
                        for name, fn in (("hann", np.hanning), ("hamming", np.hamming), ("blackman", np.blackman))}

    @staticmethod
    def _win_code(window_type: str) -> int:
        return L.WIN.get(window_type if window_type in ("hann", "hamming") else "blackman")

    def compute_fft(self, audio_data: np.ndarray, window_type: str = "hann",
                    return_complex: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        n = len(audio_data)
        key = (n, window_type, np.asarray(audio_data).tobytes()[:100])
        with self.cache_lock:
            hit = self.fft_cache.get(key)
            if hit is not None:
                return hit["magnitude"], (hit["complex"] if return_complex else None)
        if _supported(n):
            mag, cp = self._eng.rfft(np.asarray(audio_data, np.float32), window=window_type if window_type in
                                     ("hann", "hamming") else "blackman", magnitude=True, complex_out=True)
            mag, cp = mag[0], cp[0]
        else:
            logger.error("GPUAcceleratedFFT.compute_fft: empty input")
            mag, cp = np.zeros(n // 2 + 1, np.float32), np.zeros(n // 2 + 1, np.complex64)
        with self.cache_lock:
            self.fft_cache[key] = {"magnitude": mag, "complex": cp if return_complex else None,
                                   "timestamp": threading.current_thread().ident}
            if len(self.fft_cache) > 10:
                del self.fft_cache[next(iter(self.fft_cache))]
        return mag, (cp if return_complex else None)

    def compute_multi_resolution_fft(self, audio_data: np.ndarray, resolutions: Dict[str, int],
                                     window_type: str = "hann") -> Dict[str, Dict[str, np.ndarray]]:
        out = {}
        for name, n in resolutions.items():
            chunk = audio_data[-n:] if len(audio_data) >= n else np.pad(audio_data, (0, n - len(audio_data)))
            mag, cp = self.compute_fft(chunk, window_type, return_complex=True)
            out[name] = {"magnitude": mag, "complex": cp, "freqs": np.fft.rfftfreq(n, 1 / 48000)}
        return out

    def clear_cache(self):
        with self.cache_lock:
            self.fft_cache.clear()

    def get_gpu_memory_info(self) -> Dict[str, float]:
        try:
            import torch
            used = torch.cuda.memory_allocated(self.device)
            total = torch.cuda.memory_reserved(self.device)
            return {"available": True, "used_mb": used / 2 ** 20, "total_mb": total / 2 ** 20,
                    "utilization": used / total if total > 0 else 0}
        except Exception:
            return {"available": False}

    def prepare_batch_arrays(self, batch_size: int, fft_size: int):
        """(input [B, N] float32, output [B, N/2+1] complex64) on this device (torch tensors)."""
        import torch
        dev = torch.device("cuda", self.device)
        return (torch.zeros((batch_size, fft_size), dtype=torch.float32, device=dev),
                torch.zeros((batch_size, fft_size // 2 + 1), dtype=torch.complex64, device=dev))

    def process_fft_batch(self, input_batch, window_type: str = "hann"):
        """rfft of window * each row of a device batch [B, N] -> complex64 [B, N/2+1] on the device
        (None on error, as the reference)."""
        try:
            import torch
            if input_batch is None:
                return None
            if not _is_torch(input_batch):
                input_batch = torch.as_tensor(np.ascontiguousarray(input_batch, np.float32)).to(
                    torch.device("cuda", self.device))
            x = input_batch.to(torch.float32).contiguous()
            b, n = x.shape
            if not _supported(n):
                raise ValueError(f"FFT size {n} not supported on the device")
            out = torch.empty((b, n // 2 + 1), dtype=torch.complex64, device=x.device)
            self._eng._bind_stream(x)
            self._eng._check(L.lib().omega_rfft(self._eng._ctx, x.data_ptr(), b, n, self._win_code(window_type),
                                                None, out.data_ptr(), L.MEM_DEVICE))
            return out
        except Exception as e:
            logger.error("Batch FFT processing failed: %s", e)
            return None

    def setup_memory_pool(self, size_mb: int = 256):
        """The reference caps CuPy's pool; device memory here is the caller's (torch) -- nothing to set."""

    def enable_zero_copy(self):
        """The reference switches CuPy to managed memory; the entry points here take host or device
        pointers directly (mem flag), so there is nothing to switch."""
