#!/usr/bin/env python3
"""Numeric comparison of two tools/lib_outputs.py dumps (a build whose arithmetic differs, e.g. packed
FP32: not bitwise, so the largest normwise / absolute differences per output)."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in sorted(a.files):
    x, y = a[k].astype(np.float64), b[k].astype(np.float64)
    fin = np.isfinite(x) & np.isfinite(y)
    d = np.abs(x - y)[fin]
    nw = np.linalg.norm((x - y)[fin]) / max(np.linalg.norm(x[fin]), 1e-30)
    print(f"{k:16s} shape {str(x.shape):14s} max|d| {d.max() if d.size else 0:.3e}  normwise {nw:.3e}  "
          f"nonfinite-mismatch {int((np.isfinite(x) != np.isfinite(y)).sum())}")
