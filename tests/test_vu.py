"""§8(f) row 2 remainder: VU meter ballistics (omega_vu_update) against the reference's own
VUMetersPanel sequence (golden: float64 windowed frames, then float32 chunks) and the oracle on
random batches; the oracle itself is pinned to the golden on the CPU."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import omega_ref as R

# The device runs the window sums and the needle in float64. The reference follows its deque's dtype:
# float32 arithmetic once the 300 ms window holds only float32 samples (rms, log10, damping), which puts
# it ~1e-6 dB from the float64 values -- far below a displayable difference.
VU_TOL_DB = 2e-5


def test_vu_oracle_matches_reference_golden():
    g = load_golden("vu")
    st = R.VUState(48000)
    rec = [st.update(fr, 1 / 60) for fr in g["x64"]]
    rec += [st.update(fr, float(dt)) for fr, dt in zip(g["x32"], g["dt32"])]
    np.testing.assert_allclose(np.array(rec), g["out"][:, :3], rtol=0, atol=1e-9)
    np.testing.assert_array_equal(g["out"][:, 0], g["out"][:, 3])  # mono input: both needles equal


@pytest.mark.gpu
def test_vu_golden_sequence_one_call_and_per_call():
    from omega_gpu.vu_meters import VUMeters
    g = load_golden("vu")
    vu = VUMeters(48000, n_channels=2)
    a = vu.update_batch(np.repeat(g["x64"][:, None, :], 2, axis=1), np.full(len(g["x64"]), 1 / 60))
    b = vu.update_batch(np.repeat(g["x32"][:, None, :], 2, axis=1), g["dt32"])
    got = np.concatenate([a, b])
    np.testing.assert_allclose(got[:, 0, :], g["out"][:, :3], rtol=0, atol=VU_TOL_DB)
    np.testing.assert_array_equal(got[:, 0, :], got[:, 1, :])
    # the panel-style per-call facade (mono input drives both needles)
    v1 = VUMeters(48000)
    for fr in g["x64"][:100]:
        v1.update(fr, 1 / 60)
    assert abs(v1.vu_left_display - g["out"][99, 1]) < VU_TOL_DB
    assert abs(v1.vu_right_peak_db - g["out"][99, 2]) < VU_TOL_DB
    v1.update(np.zeros(0), 1 / 60)  # empty: no change
    assert abs(v1.vu_left_display - g["out"][99, 1]) < VU_TOL_DB


@pytest.mark.gpu
def test_vu_random_batches_channels_and_device_input():
    import torch
    from omega_gpu.vu_meters import VUMeters
    rng = np.random.default_rng(8)
    C, n, m = 3, 90, 700
    lv = np.abs(rng.standard_normal((n, C, 1))) * np.linspace(1, 0.001, n)[:, None, None]
    x = (rng.standard_normal((n, C, m)) * lv).astype(np.float32)
    x[30:50, 1] = 0.0
    dts = rng.uniform(0.01, 0.1, n)
    vu = VUMeters(44100, n_channels=C)
    parts = [vu.update_batch(x[a:e], dts[a:e]) for a, e in ((0, 1), (1, 37), (37, n))]
    got = np.concatenate(parts)
    for c in range(C):
        st = R.VUState(44100)
        ref = np.array([st.update(x[u, c], dts[u]) for u in range(n)])
        np.testing.assert_allclose(got[:, c, :], ref, rtol=0, atol=VU_TOL_DB)
    vu.reset()
    xd = torch.from_numpy(x).cuda()
    gd = vu.update_batch(xd, dts)
    torch.cuda.synchronize()
    np.testing.assert_allclose(gd.cpu().numpy(), got, rtol=0, atol=1e-12)
