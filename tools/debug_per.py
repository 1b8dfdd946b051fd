import sys
sys.path.insert(0, "."); sys.path.insert(0, "humanoid-walking-with-sac_amd")
import numpy as np, torch
from oracle.sac_step import NETS, OracleSAC, SacConfig, init_params, synthetic_rows
from sacmi import Config, Context
cfg = SacConfig(24, 4, 64)
params = init_params(cfg, 81, bias_scale=0.05)
for nrows, cap in ((200, 256), (300, 256)):
    rows = synthetic_rows(cfg, nrows, 82, state_scale=0.5)
    def mk(kind):
        c = Context(Config(24, 4, 64, max_batch=64, capacity=cap, replay=kind), 0)
        for n in NETS: c.set_net(n, params[n])
        c.push(*rows)
        if kind == "per":
            L = min(nrows, cap)
            c.per_update(np.arange(L), np.linspace(0.1, 3, L).astype(np.float32))
            c.set_mt(1, np.arange(624, dtype=np.uint32), 624)
        return c
    z = np.zeros((64, 4), np.float32)
    a = mk("per"); idx, w = a.per_sample(64)
    b = mk("per"); lb = b.step(64, eps1=z, eps2=z)
    head = 0 if nrows < cap else nrows % cap
    pos = (idx - head) % cap
    u = mk("uniform"); lu = u.step(64, idx=pos, eps1=z, eps2=z)
    s, aa, r, s2, d = a.get_slots(idx)
    o = OracleSAC(cfg, params, torch.float64).step(s, aa, r, s2, d, z, z)
    print(nrows, cap, "per-step", lb, "uniform+pos", lu, "oracle", [o[k] for k in o])
    print("   idx[:10]", idx[:10], "w[:4]", w[:4])
