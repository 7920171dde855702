"""ctypes binding of libomega.so (include/omega.h). No torch types cross this boundary: plain
pointers and sizes. The library is loaded from the package's in-tree ``lib/`` and the import fails
loudly when it is missing -- there is no CPU fallback."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libomega.so")

MAX_RES = 4
N_METERS = 5
MEM_HOST, MEM_DEVICE = 0, 1
WIN = {"blackman": 0, "hann": 1, "hamming": 2, "rect": 3}
BANDS_MAX, BANDS_MEAN = 0, 1
WEIGHT = {"K": 0, "A": 1, "C": 2, "Z": 3}
OK, EINVAL, EHIP, ENOMEM, EUNSUP = 0, -1, -2, -3, -4


class Resolution(C.Structure):
    _fields_ = [("freq_lo", C.c_double), ("freq_hi", C.c_double), ("fft_size", C.c_int32),
                ("hop_size", C.c_int32), ("weight", C.c_double), ("window", C.c_int32)]


class Config(C.Structure):
    _fields_ = [("sample_rate", C.c_int32), ("max_freq", C.c_double), ("n_res", C.c_int32),
                ("res", Resolution * MAX_RES), ("apply_weighting", C.c_int32), ("target_bins", C.c_int32),
                ("frame_size", C.c_int32), ("n_channels", C.c_int32), ("gate_lufs", C.c_double),
                ("momentary_len", C.c_int32), ("short_len", C.c_int32), ("integrated_len", C.c_int32),
                ("peak_len", C.c_int32)]


class Outputs(C.Structure):
    _fields_ = [("combined", C.c_void_p), ("lufs_inst", C.c_void_p), ("true_peak_db", C.c_void_p),
                ("meters", C.c_void_p), ("mag", C.c_void_p * MAX_RES), ("weighted", C.c_void_p)]


class IngestConfig(C.Structure):
    _fields_ = [("format", C.c_int32), ("sample_rate", C.c_int32), ("hop", C.c_int32), ("batch_hops", C.c_int32),
                ("ring_slots", C.c_int32), ("max_pending_batches", C.c_int32), ("chunk_size", C.c_int32), ("gain", C.c_float), ("gate", C.c_int32),
                ("noise_floor", C.c_double), ("silence_threshold_seconds", C.c_double),
                ("background_alpha", C.c_double), ("want", C.c_int32)]


class IngestStats(C.Structure):
    _fields_ = [("bytes_in", C.c_int64), ("batches", C.c_int64), ("frames", C.c_int64),
                ("frames_polled", C.c_int64), ("dropped_frames", C.c_int64)]


FMT = {"float32le": 0, "s16le": 1}
INGEST_COMBINED, INGEST_LUFS, INGEST_TRUE_PEAK, INGEST_METERS = 1, 2, 4, 8


class OmegaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libomega error {code}: {msg}")
        self.code = code


class UnsupportedError(OmegaError):
    """A valid reference call this build does not cover (e.g. a non power-of-two frame)."""


EXPORTS = {
    "omega_version": (C.c_char_p, []),
    "omega_config_default": (None, [C.POINTER(Config)]),
    "omega_create": (C.c_int, [C.POINTER(Config), C.c_int, C.POINTER(C.c_void_p)]),
    "omega_destroy": (None, [C.c_void_p]),
    "omega_last_error": (C.c_char_p, [C.c_void_p]),
    "omega_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "omega_check_queues": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "omega_synchronize": (C.c_int, [C.c_void_p]),
    "omega_set_meter_pipelining": (C.c_int, [C.c_void_p, C.c_int]),
    "omega_flush_meters": (C.c_int, [C.c_void_p]),
    "omega_get_stream": (C.c_void_p, [C.c_void_p]),
    "omega_get_config": (C.c_int, [C.c_void_p, C.POINTER(Config), C.POINTER(C.c_int)]),
    "omega_vu_update": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_int64,
                                  C.c_void_p, C.c_void_p, C.c_int]),
    "omega_vu_reset": (C.c_int, [C.c_void_p]),
    "omega_transients": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_void_p,
                                   C.c_int]),
    "omega_ingest_config_default": (None, [C.POINTER(IngestConfig)]),
    "omega_ingest_create": (C.c_int, [C.c_void_p, C.POINTER(IngestConfig), C.POINTER(C.c_void_p)]),
    "omega_ingest_push": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    "omega_ingest_flush": (C.c_int, [C.c_void_p]),
    "omega_ingest_poll": (C.c_int, [C.c_void_p, C.c_int64, C.POINTER(Outputs), C.c_int, C.POINTER(C.c_int64)]),
    "omega_ingest_get_stats": (C.c_int, [C.c_void_p, C.POINTER(IngestStats)]),
    "omega_ingest_last_error": (C.c_char_p, [C.c_void_p]),
    "omega_ingest_destroy": (None, [C.c_void_p]),
    "omega_set_graphs": (C.c_int, [C.c_void_p, C.c_int]),
    "omega_process_frames": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                       C.POINTER(Outputs), C.c_int]),
    "omega_process_stream": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int64,
                                       C.POINTER(Outputs), C.c_int, C.POINTER(C.c_int64)]),
    "omega_spectra": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                C.c_void_p, C.c_void_p, C.c_int]),
    "omega_combine": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int64, C.c_void_p, C.c_int]),
    "omega_true_peak": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int]),
    "omega_true_peak_os": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_int]),
    "omega_k_weighting": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p,
                                    C.c_int]),
    "omega_weighting": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p,
                                  C.c_void_p, C.c_int]),
    "omega_meter_update": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]),
    "omega_meter_reset": (C.c_int, [C.c_void_p]),
    "omega_meter_load_history": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int]),
    "omega_calculate_lufs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "omega_bands_create": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                     C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "omega_bands_destroy": (None, [C.c_void_p]),
    "omega_bands_apply": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_int]),
    "omega_chroma": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_double, C.c_void_p, C.c_int]),
    "omega_drum_features": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int64, C.c_double,
                                      C.c_void_p, C.c_int]),
    "omega_drum_reset": (C.c_int, [C.c_void_p]),
    "omega_post_configure": (C.c_int, [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_int32, C.c_int32, C.c_float]
                             + [C.c_void_p] * 3 + [C.c_int32]),
    "omega_post_process": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_float,
                                     C.c_void_p, C.c_void_p, C.c_void_p]),
    "omega_post_reset": (C.c_int, [C.c_void_p]),
    "omega_rfft": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                             C.c_int]),
}

_lib = None


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process. torch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7,
    like /opt/rocm's). If libomega loaded first it would bind /opt/rocm's copy and torch would then
    load a second runtime (torch reports "No HIP GPUs are available", and torch streams/events would
    not order libomega's kernels). Preloading torch's copy by path, without importing torch, makes
    libomega's NEEDED libamdhip64.so.7 resolve to the runtime torch uses."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)
            return


def use_development_library(name: str) -> None:
    """Kernel-development tools only (tools/stamps.py, tools/wgtrace.py): load lib/<name> (e.g.
    libomega_dev.so from `make dev`) instead of libomega.so. Must run before the first lib() call; the
    product path never calls it and reads no environment variable to pick its library."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libomega is already loaded")
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", name)


def lib() -> C.CDLL:
    """Load libomega.so once (raises if the HIP library was not built: no fallback)."""
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libomega.so not found at {LIB_PATH}; run `make -C audio-analyzer-omega_amd` "
                              "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        dev = os.path.basename(LIB_PATH) != "libomega.so"
        for name, (res, args) in EXPORTS.items():
            if dev and not hasattr(L, name):  # (an older build in an A/B: its ABI's entry points only)
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(ctx, code: int) -> None:
    if code != OK:
        msg = lib().omega_last_error(ctx).decode() if ctx else ""
        raise (UnsupportedError if code == EUNSUP else OmegaError)(code, msg)
