#!/usr/bin/env python3
"""Run bench.py's side lines (cfg3, drums, app_post) once each for a profiler: python tools/side_lines.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402

d = torch.device("cuda", 0)
for fn in (bench.cfg3_line, bench.drums_line, bench.post_line):
    r = fn(d)
    print(json.dumps({"workload": r["workload"][:40], "value": r["value"], "frac": r["roofline"]["frac"]}))
