"""CPU-side checks of the drop-in boundary: libomega.so loads, exports every function include/omega.h
declares, the ctypes structs match the C layout, and config validation mirrors the reference's
ValueErrors (validation runs before any HIP call, so this needs no GPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO


def _declared():
    h = open(os.path.join(REPO, "include", "omega.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    return sorted(set(re.findall(r"\b(omega_[a-z_]+)\s*\(", h)))


def test_library_exports_every_declared_symbol():
    import omega_gpu
    lib = omega_gpu.lib()
    names = _declared()
    assert len(names) >= 18
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from omega_gpu import _lib
    assert set(names) == set(_lib.EXPORTS), set(names) ^ set(_lib.EXPORTS)


def test_version_and_defaults():
    import omega_gpu
    from omega_gpu import _lib as L
    assert omega_gpu.lib().omega_version().startswith(b"omega-mi355x")
    cfg = L.Config()
    omega_gpu.lib().omega_config_default(C.byref(cfg))
    assert (cfg.sample_rate, cfg.max_freq, cfg.n_res, cfg.target_bins) == (48000, 20000.0, 4, 1024)
    got = [(cfg.res[i].freq_lo, cfg.res[i].freq_hi, cfg.res[i].fft_size, cfg.res[i].hop_size, cfg.res[i].weight)
           for i in range(4)]
    # multi_resolution_fft.py:149-154
    assert got == [(20, 200, 4096, 1024, 1.5), (200, 1000, 2048, 512, 1.2), (1000, 5000, 1024, 256, 1.0),
                   (5000, 20000, 1024, 256, 1.5)]
    assert (cfg.gate_lufs, cfg.momentary_len, cfg.short_len, cfg.integrated_len, cfg.peak_len) == (-70.0, 24, 180, 3600, 60)


def test_struct_layout():
    from omega_gpu import _lib as L
    # omega_resolution: 2 doubles, 2 int32, 1 double, 1 int32 (+pad) = 40 bytes on LP64
    assert C.sizeof(L.Resolution) == 40
    assert C.sizeof(L.Outputs) == 9 * 8


@pytest.mark.parametrize("bad, msg", [
    (dict(freq_range=(200, 20)), "Invalid frequency range"),
    (dict(fft_size=1000), "FFT size must be power of 2"),
    (dict(hop_size=0), "Hop size must be positive"),
    (dict(weight=0.0), "Weight must be positive"),
])
def test_config_validation_mirrors_reference(bad, msg):
    from omega_gpu import Engine, Resolution
    kw = dict(freq_range=(20, 200), fft_size=1024, hop_size=256, weight=1.0)
    kw.update(bad)
    with pytest.raises(ValueError, match=msg):
        Engine([Resolution(**kw)])


def test_sample_rate_and_nyquist_validation():
    from omega_gpu import Engine, Resolution
    r = [Resolution((20, 200), 1024, 256, 1.0)]
    with pytest.raises(ValueError, match="Sample rate must be positive"):
        Engine(r, sample_rate=0)
    with pytest.raises(ValueError, match="Nyquist"):
        Engine(r, sample_rate=48000, max_freq=30000)


def test_facade_constructor_errors():
    from omega_gpu.multi_resolution_fft import FFTConfig, MultiResolutionFFT
    with pytest.raises(ValueError):
        FFTConfig((20, 200), 1000, 256, 1.0)
    with pytest.raises(ValueError):
        MultiResolutionFFT(sample_rate=-1)
    with pytest.raises(ValueError):
        MultiResolutionFFT(48000, max_freq=24001)


def test_unsupported_sizes_are_reported_not_faked():
    from omega_gpu import Engine, Resolution, UnsupportedError
    with pytest.raises(UnsupportedError):
        Engine([Resolution((20, 200), 1024, 256, 1.0)], frame_size=256)  # frames below 512 samples


def test_no_gpu_fails_loudly():
    """Without a device the product path raises; it never falls back to a CPU computation."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from omega_gpu import Engine, OmegaError
    with pytest.raises(OmegaError):
        Engine()


def test_product_package_does_not_import_oracle():
    pkg = os.path.join(REPO, "audio-analyzer-omega_amd", "omega_gpu")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert not re.search(r"^\s*(from|import)\s+(oracle|scipy)\b", src, flags=re.M), f


def test_abi_guard_maps_host_allocation_failure(tmp_path):
    """include/omega.h's contract -- no C++ exception crosses the ABI -- through public entry points:
    tests/abi/abi_guard.cpp replaces operator new with one that throws std::bad_alloc while armed and
    calls omega_create and omega_post_configure (a host-side table build) armed; both return
    OMEGA_ENOMEM with a message instead of terminating the process (no GPU needed)."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    lib = os.path.join(REPO, "audio-analyzer-omega_amd", "lib")
    exe = str(tmp_path / "abi_guard")
    subprocess.run(["g++", "-std=c++17", "-O1", "-o", exe, os.path.join(REPO, "tests", "abi", "abi_guard.cpp"),
                    f"-L{lib}", "-lomega", f"-Wl,-rpath,{lib}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")
