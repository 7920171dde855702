#!/usr/bin/env python3
"""Device time of loading a time-sharded stream's meter history: omega_meter_load_history
(one kernel) against the round-4 replay (reset + omega_meter_update over the history as pseudo-frames),
a full 3599-frame LUFS / 59-frame true-peak history of a stereo stream, HIP events on the stream."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "audio-analyzer-omega_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from omega_gpu import Engine, Resolution
    from omega_gpu import dist as D
    rng = np.random.default_rng(3)
    hl = torch.from_numpy(rng.uniform(-90, -5, (3599, 2)).astype(np.float32)).cuda()
    ht = torch.from_numpy(rng.uniform(-40, 0, (59, 2)).astype(np.float32)).cuda()
    e = Engine([Resolution((20, 20000), 512, 256, 1.0)], 48000, 20000, 2, frame_size=512, n_channels=2)
    rl, rt = D.history_frames(hl, ht)
    rl, rt = rl.contiguous(), rt.contiguous()

    def load():
        e.load_meter_history(hl, ht)

    def replay():
        e.reset_meters()
        e.meter_update(rl, rt, rl.shape[0])

    for name, f in (("load_meter_history", load), ("reset + meter_update replay", replay)):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            f()
        t.record()
        torch.cuda.synchronize()
        print(f"{name:28s} {s.elapsed_time(t) / 50 * 1e3:8.1f} us per history (3599 x 2 LUFS, 59 x 2 TP)")


if __name__ == "__main__":
    main()
