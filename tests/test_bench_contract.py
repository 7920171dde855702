"""bench.py's synthetic workload equals the oracle's cfg2 generator (so the CPU-baseline sample sees
the same frames as the GPU), and its constants are the SURVEY.md §8(d) figures."""
import numpy as np


def test_bench_input_matches_oracle_generator():
    import bench
    from oracle import signals as S
    np.testing.assert_array_equal(bench.cfg2_input(3, seed_l=4, seed_r=5), S.cfg2_batch(3, seed_l=4, seed_r=5))


def test_bench_algorithmic_figures():
    import bench
    assert round(bench.FLOP_TP / 1e6, 2) == 3.33
    assert round(bench.FLOP_FFT / 1e6, 2) == 1.09
    assert round(bench.FLOP_KW / 1e6, 2) == 0.67
    assert bench.BYTES_CF == 67592


def test_cfg3_input_matches_oracle_generator():
    import bench
    from oracle import signals as S
    np.testing.assert_array_equal(bench.cfg3_input(8, 8192), S.cfg3_batch(8))


def test_cfg5_input_matches_oracle_generator():
    import bench
    from oracle import signals as S
    np.testing.assert_array_equal(bench.cfg5_input(5000, 8, 96000), S.cfg5_stream(5000, 8, 96000))
