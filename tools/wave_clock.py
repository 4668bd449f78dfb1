"""Pass-1 wave timeline of config 3 (MTE_WAVE_CLOCK): per-pair start / end
(s_memrealtime, 100 MHz) -> tail statistics.  Usage on the GPU box:
  MTE_WAVE_CLOCK=gpurun_out/wclock.bin python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  python3 tools/wave_clock.py gpurun_out/wclock.bin"""
import sys

import numpy as np

w = np.fromfile(sys.argv[1], np.uint64).reshape(-1, 2).astype(np.int64)
t0 = w[:, 0].min()
start = (w[:, 0] - t0) / 100.0  # us
end = (w[:, 1] - t0) / 100.0
dur = end - start
q = np.percentile(end, [0, 10, 50, 90, 99, 100])
print(f"pairs {len(w)}  start max {start.max():.1f} us")
print("end   pct 0/10/50/90/99/100 (us):", " ".join(f"{x:.0f}" for x in q))
print("dur   mean {:.0f} std {:.0f} min {:.0f} max {:.0f} us".format(dur.mean(), dur.std(), dur.min(), dur.max()))
print(f"busy fraction of the pass (mean end / max end): {end.mean() / end.max():.3f}")
