"""PER sampling probe: n per_sample calls at a 1M-row ring (for rocprofv3 --stats)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd"))
import numpy as np
import torch  # noqa: F401
from sacmi import Config, Context
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ctx = Context(Config(4, 1, 4, max_batch=4096, capacity=n, replay="per"), 0)
ctx.push(np.zeros((n, 4), np.float32), np.zeros((n, 1), np.float32), np.zeros(n, np.float32),
         np.zeros((n, 4), np.float32), np.zeros(n, np.uint8))
for _ in range(3):
    ctx.per_sample(4096)
t = time.perf_counter()
for _ in range(20):
    ctx.per_sample(4096)
print("per_sample us (incl. host copies)", (time.perf_counter() - t) / 20 * 1e6)
