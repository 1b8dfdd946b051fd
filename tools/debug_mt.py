import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "humanoid-walking-with-sac_amd")
import numpy as np, torch
from oracle.pyrandom import MT19937, sample_indices
from oracle.sac_step import SacConfig, NETS, param_shapes
from sacmi import Config, Context
z = np.load("tests/golden/step_small.npz")
S, A, H, B, N = (int(x) for x in z["cfg"])
rows = [z[f"rows.{k}"] for k in ("s", "a", "r", "s2", "d")]
ref = sample_indices(MT19937(z["step0.mt_key"], int(z["step0.mt_pos"])), N, B)
for ng in ("0", "1"):
    os.environ["SACMI_NO_GRAPH"] = ng
    ctx = Context(Config(S, A, H, max_batch=B, capacity=N), 0)
    ctx.push(*rows)
    print("len", len(ctx))
    ctx.set_mt(0, z["step0.mt_key"], int(z["step0.mt_pos"]))
    k, p = ctx.get_mt(0); print("mt roundtrip", np.array_equal(k, z["step0.mt_key"]), p)
    got = ctx.sample_indices(B)
    print("nograph", ng, "sample_indices equal:", np.array_equal(got, ref), got[:8], ref[:8])
    k2, p2 = ctx.get_mt(0)
    m = MT19937(z["step0.mt_key"], int(z["step0.mt_pos"])); sample_indices(m, N, B)
    print("post state equal", np.array_equal(k2, m.key), p2, m.pos)
