"""§8(f) row 4: TransientAnalyzer.analyze_transients on the device (omega_transients, float64) against
the reference's own outputs (golden: float64 windowed 2048-sample frames, float32 1024-sample frames,
one analyzer so the envelope history carries over) and the oracle; the oracle is pinned on the CPU."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import omega_ref as R

KEYS = ("transients_detected", "attack_time", "punch_factor", "envelope_peak", "envelope_rms")


def test_transient_oracle_matches_reference_golden():
    g = load_golden("transients")
    st = R.TransientState(48000)
    rec = [[r[k] for k in KEYS] for r in (st.analyze(fr) for fr in list(g["x64"]) + list(g["x32"]))]
    np.testing.assert_array_equal(np.array(rec), g["out"])
    short = st.analyze(np.ones(40))
    np.testing.assert_array_equal([short[k] for k in KEYS[:3]], g["short"])
    np.testing.assert_array_equal(list(st.envelope_history), g["history"])


ANY_GROUPS = ("f64_4800", "f32_1000", "f64_1021", "f64_9600", "f32_100", "zeros_3000")


def test_transient_oracle_any_length_golden():
    """Lengths that are not powers of two: the oracle against the reference."""
    g = load_golden("transients_any")
    for name in ANY_GROUPS:
        st = R.TransientState(48000)
        rec = [[r[k] for k in KEYS] for r in (st.analyze(fr) for fr in g[f"{name}/x"])]
        np.testing.assert_array_equal(np.array(rec), g[f"{name}/out"], err_msg=name)
        np.testing.assert_array_equal(list(st.envelope_history), g[f"{name}/history"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ANY_GROUPS)
def test_transients_any_length_golden(name):
    """transient_any_kernel (complex mixed-radix float64 transform; 9600 samples on global working
    buffers) against the reference: counts exact, the rest to float64 rounding (float32 frames: 1e-6)."""
    from omega_gpu.transient import TransientAnalyzer
    g = load_golden("transients_any")
    ta = TransientAnalyzer(48000)
    x = g[f"{name}/x"]
    if name.startswith("f32"):
        x = x.astype(np.float32)
    got = ta.analyze_batch(x)[:, :5]
    ref = g[f"{name}/out"]
    np.testing.assert_array_equal(got[:, 0], ref[:, 0])
    tol = 1e-6 if name.startswith("f32") else 1e-9
    np.testing.assert_allclose(got[:, 1:], ref[:, 1:], rtol=tol, atol=1e-12)
    np.testing.assert_allclose(ta.get_envelope_history(), g[f"{name}/history"], rtol=tol, atol=1e-15)


@pytest.mark.gpu
def test_transients_golden():
    """Counts exact; times, punch and envelope statistics to float64 rounding for the float64 frames
    (1e-9 relative: the device's FFT and sums run in another order than scipy's pocketfft and numpy's
    pairwise sums) and to float32 rounding for the float32 frames (scipy's hilbert transforms a float32
    frame in complex64 before its complex128 inverse; the device stays in float64: 1e-6 relative)."""
    from omega_gpu.transient import TransientAnalyzer
    g = load_golden("transients")
    ta = TransientAnalyzer(48000)
    got = [[r[k] for k in KEYS] for r in (ta.analyze_transients(fr) for fr in g["x64"])]
    got += [list(r[:5]) for r in ta.analyze_batch(g["x32"])]
    got = np.array(got)
    np.testing.assert_array_equal(got[:, 0], g["out"][:, 0])
    n64 = len(g["x64"])
    np.testing.assert_allclose(got[:n64, 1:], g["out"][:n64, 1:], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(got[n64:, 1:], g["out"][n64:, 1:], rtol=1e-6, atol=1e-12)
    assert ta.analyze_transients(np.ones(40)) == {"transients_detected": 0, "attack_time": 0.0, "punch_factor": 0.0}
    np.testing.assert_allclose(ta.get_envelope_history(), g["history"], rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [64, 512, 8192])
def test_transients_sizes_vs_oracle(n):
    import torch
    from omega_gpu.transient import TransientAnalyzer
    rng = np.random.default_rng(n)
    x = rng.standard_normal((5, n)) * np.exp(-np.arange(n) / (n / 8))[None, :]
    x[:, n // 3:n // 3 + 8] += 3.0
    ta = TransientAnalyzer(44100)
    got = ta.analyze_batch(x)
    st = R.TransientState(44100)
    for f in range(5):
        r = st.analyze(x[f])
        assert got[f, 0] == r["transients_detected"]
        np.testing.assert_allclose(got[f, 1:5], [r[k] for k in KEYS[1:]], rtol=1e-9, atol=1e-15)
    xd = torch.from_numpy(x.astype(np.float32)).cuda()
    gd = ta.analyze_batch(xd).cpu().numpy()
    st32 = R.TransientState(44100)
    for f in range(5):
        r = st32.analyze(x[f].astype(np.float32).astype(np.float64))
        assert gd[f, 0] == r["transients_detected"]
    z = ta.analyze_transients(np.zeros(3000))  # a length off the packed transform (transient_any_kernel)
    assert z == {"transients_detected": 0, "attack_time": 0.0, "punch_factor": 0.0, "envelope_peak": 0.0,
                 "envelope_rms": 0.0}


@pytest.mark.gpu
def test_transients_any_length_sliced_scratch():
    """Frames too long for LDS run on global working buffers in slices of frames (64 MiB of scratch
    per launch): 420 frames of 10000 samples span three slices (209 frames each) and equal the same
    frames analysed in single-frame calls bitwise; a few frames against the oracle to float32 rounding."""
    from omega_gpu.transient import TransientAnalyzer
    rng = np.random.default_rng(42)
    n, F = 10000, 420
    x = (rng.standard_normal((F, n)) * np.linspace(0.05, 0.9, F)[:, None]).astype(np.float32)
    x[:, 3000:3050] *= 8.0
    ta = TransientAnalyzer(48000)
    got = ta.analyze_batch(x)
    for f in (0, 208, 209, 210, 418, 419):
        one = TransientAnalyzer(48000).analyze_batch(x[f:f + 1])
        np.testing.assert_array_equal(got[f], one[0], err_msg=str(f))
    st = R.TransientState(48000)
    for f in (0, 209, 419):
        r = st.analyze(x[f])
        assert got[f, 0] == r[KEYS[0]]
        np.testing.assert_allclose(got[f, 1:5], [r[k] for k in KEYS[1:5]], rtol=1e-6, atol=1e-12)
