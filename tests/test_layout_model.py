"""The register-FFT LDS layouts (csrc/regfft.hpp) as an index model (tools/model/regfft_model.py): each
plan reproduces np.fft.fft, each exchange is a bijection onto its slots, and no exchange has LDS bank
conflicts beyond the known 2-way natural-order reads -- for the padded K = 4096 / 8192 layouts and the tight
32 KiB K = 4096 one (RegFFT<4096, true>)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "model"))
import regfft_model as M  # noqa: E402


def _check(pl, n_slots_max, allowed=("x3m",)):
    rng = np.random.default_rng(3)
    x = rng.standard_normal(pl.K) + 1j * rng.standard_normal(pl.K)
    ref = np.fft.fft(x)
    assert np.max(np.abs(pl.fft(x) - ref)) / np.max(np.abs(ref)) < 1e-12
    c = pl.check_conflicts()
    assert all(v == 0 for k, v in c.items() if k not in allowed), c
    assert all(c[k] <= 2 for k in allowed), c
    s3 = {pl.a3(n) for n in range(pl.K)}
    assert len(s3) == pl.K and max(s3) < n_slots_max


def test_padded_layouts():
    # (the padded natural-order spectrum reads cost one extra cycle on a few lane groups)
    _check(M.Plan(4096), 4352, ("x3m",))
    _check(M.Plan(8192), 8712, ("x3r", "x3m"))


def test_natural_order_4096_separable_forms():
    """RegFFT<4096>'s natural-order slots as the kernel addresses them (regfft.hpp s3 / o3 / s3m / s3o /
    o3o: a per-thread base plus an immediate offset per register) equal the model's a3 -- the XOR
    swizzle -- for the untangle's reads, their mirrors and pass 3's stores."""
    pl = M.Plan(4096)
    s3 = lambda t: t ^ ((t >> 4) & 15)  # noqa: E731
    for t in range(256):
        for r in range(16):
            assert pl.a3(t + 256 * r) == s3(t) + 256 * r
            if t:
                assert pl.a3(4096 - t - 256 * r) == s3(256 - t) + 256 * (15 - r)
    for s_ in range(256):
        for m in range(16):
            assert pl.a3(pl.out_index(s_, m)) == ((s_ >> 4) ^ (s_ & 15)) + 16 * (s_ & 15) + 256 * m
    # t = 0: the mirror of register r = 0 is bin K (slot 4096, inside the exchange buffer: the callers
    # take bin 0's real and imaginary parts instead)
    assert s3(256) + 256 * 15 == 4096 < 4352


def test_half_buffer_layout():
    """RegFFT<4096>::run_half: the same maps in float units through one 4352-float buffer, every access a
    32-lane ds_read_b32 / ds_write_b32 -- conflict-free except one extra cycle on the mirror reads."""
    _check(M.HalfPlan4096(), 4352, ("x3m",))


def test_tight_layout():
    pl = M.TightPlan4096()
    _check(pl, 4096)
    M.check_tight()


def test_exchange2_is_wave_local():
    """regfft.hpp drops the workgroup barriers around exchange 2: every slot a wave writes or reads
    there lies in its own exchange-1 rows, which no other wave reads."""
    for K in (8192, 4096):
        assert M.wave_local_exchange2(K) == 0


def test_meter_prep_model_matches_oracle():
    """The meter prep / query index algebra (tools/model/meter_model.py restates meters.hip's core /
    extras split by rank, the time-order prefixes and the next sorted history) equals the oracle's
    MeterState over random batches: gated and ungated values, ties, a silent stretch, batch sizes
    across the 3600-frame window's eviction."""
    import numpy as np
    import meter_model as MM
    from oracle import omega_ref as R
    rng = np.random.default_rng(4)
    n = 4300
    li = rng.uniform(-85, -5, n).astype(np.float32)
    li[500:900] = -95.0
    li[1000:1100] = np.float32(-23.0)
    tp = rng.uniform(-40, 0, n).astype(np.float32)
    m = MM.Model()
    cuts = [0, 1, 7, 300, 1324, 2400, 3900, 4299, n]
    got = np.concatenate([m.batch(li[a:b], tp[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    st = R.MeterState(48000)
    ref = np.array([list(st.update(np.ones(1), float(li[f]), float(tp[f])).values()) for f in range(n)])
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-9)



def test_post_top16_select_model():
    """The app post-processing's percentile select for frames up to 512 bins (csrc/post.hip
    wave_top16 / merge_top16, modelled lane for lane in tools/model/post_select_model.py): each wave's
    top 16 come out as its 16 largest keys in order, and the fold of the four gives np.sort's key at
    each rank of the frame's top 16, with heavy ties, frames shorter than a wave and frames of one bin."""
    import post_select_model as P
    rng = np.random.default_rng(4)
    for trial in range(400):
        t = int(rng.integers(1, 513)) if trial > 2 else (1, 16, 512)[trial]
        keys = rng.integers(1, 2 ** 32 if trial % 2 else 12, size=t).astype(np.uint64)
        for w in range(4):
            part = np.concatenate([keys[128 * w:128 * w + 128], np.zeros(128, np.uint64)])[:128]
            np.testing.assert_array_equal(P.wave_top16(keys, w), np.sort(part)[-16:])
        ref = np.sort(keys)
        for r in range(max(t - 16, 0), t):
            assert P.select(keys, r) == ref[r], (t, r)
