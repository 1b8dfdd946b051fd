"""select_action latency probe: drop-in agent vs raw ctx.act, Humanoid shapes."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd"))
import numpy as np
import torch
from sac_imp import SAC
agent = SAC(376, 17, hidden_dim=512, device="cuda", capacity=10000, max_batch=256, seed=1)
s = np.random.default_rng(0).standard_normal(376).astype(np.float32)
for f, name in ((lambda: agent.select_action(s), "agent.select_action"),
                (lambda: agent._ctx.act(s.reshape(1, -1), False), "ctx.act"),
                (lambda: agent._ctx.act(s.reshape(1, -1), True), "ctx.act det")):
    for _ in range(20):
        f()
    t = time.perf_counter()
    for _ in range(500):
        f()
    print(f"{name}: {(time.perf_counter() - t) / 500 * 1e6:.1f} us")
