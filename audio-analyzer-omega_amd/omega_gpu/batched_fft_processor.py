"""BatchedFFTProcessor over libomega.so (omega4/optimization/batched_fft_processor.py:37-360).

The reference's GPU seam (CuPy cuFFT with host windowing and an H2D/D2H per request) becomes one
device launch per FFT size over all pending requests; request bookkeeping keeps the reference's
API: prepare_batch -> request id, process_batch -> count, distribute_results -> {id: result}.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict
from typing import Dict, Optional

import numpy as np

from .engine import Engine, Resolution


class FFTRequest:
    def __init__(self, request_id: str, audio_data: np.ndarray, fft_size: int, window_type: str = "hann"):
        self.request_id = request_id
        self.audio_data = audio_data
        self.fft_size = fft_size
        self.window_type = window_type
        self.result = None
        self.completed = False


class BatchedFFTProcessor:
    def __init__(self, gpu_memory_limit_mb: int = 256, device: int = 0):
        self.gpu_available = True
        self.gpu_memory_limit = gpu_memory_limit_mb * 1024 * 1024
        self.pending_requests: Dict[str, FFTRequest] = {}
        self.request_lock = threading.Lock()
        self.common_fft_sizes = [512, 1024, 2048, 4096, 8192, 16384]
        self.batch_times = []
        self.last_batch_size = 0
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], 48000, 20000, target_bins=2, frame_size=512,
                           device=device)
        self._seq = 0

    def prepare_batch(self, panel_id: str, audio_data: np.ndarray, fft_size: int, window_type: str = "hann") -> str:
        """batched_fft_processor.py:119-146 (pads or keeps the last fft_size samples)."""
        self._seq += 1
        request_id = f"{panel_id}_{fft_size}_{time.time()}_{self._seq}"
        if len(audio_data) > fft_size:
            audio_data = audio_data[-fft_size:]
        elif len(audio_data) < fft_size:
            audio_data = np.pad(audio_data, (0, fft_size - len(audio_data)))
        with self.request_lock:
            self.pending_requests[request_id] = FFTRequest(request_id, audio_data, fft_size, window_type)
        return request_id

    def process_batch(self) -> int:
        with self.request_lock:
            if not self.pending_requests:
                return 0
            groups = defaultdict(list)
            for r in self.pending_requests.values():
                if not r.completed:
                    groups[(r.fft_size, r.window_type)].append(r)
        start = time.perf_counter()
        total = 0
        for (n, w), reqs in groups.items():
            x = np.stack([np.asarray(r.audio_data, np.float32) for r in reqs])
            mag, cp = self._eng.rfft(x, w if w in ("hann", "hamming", "blackman") else "rect")
            freqs = np.fft.rfftfreq(n, 1 / 48000)  # hard-coded 48 kHz, as the reference (:230, :257)
            for i, r in enumerate(reqs):
                r.result = {"magnitude": mag[i], "complex": cp[i], "frequencies": freqs}
                r.completed = True
            total += len(reqs)
        self.batch_times.append((time.perf_counter() - start) * 1000)
        if len(self.batch_times) > 60:
            self.batch_times.pop(0)
        self.last_batch_size = total
        return total

    def distribute_results(self) -> Dict[str, Dict[str, np.ndarray]]:
        out = {}
        with self.request_lock:
            done = [k for k, r in self.pending_requests.items() if r.completed]
            for k in done:
                out[k] = self.pending_requests.pop(k).result
        return out

    def get_result_for_panel(self, request_id: str) -> Optional[Dict[str, np.ndarray]]:
        with self.request_lock:
            r = self.pending_requests.get(request_id)
            if r and r.completed:
                return self.pending_requests.pop(request_id).result
        return None
