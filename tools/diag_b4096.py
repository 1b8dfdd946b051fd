"""Diagnose the batch-4096 critic fc1 gradient error: where (rows / columns) it sits."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
from test_gpu_parity import run_case, rel
from oracle.sac_step import SacConfig, init_params, synthetic_rows
cfg = SacConfig(376, 17, 512, n_hidden=int(sys.argv[2]) if len(sys.argv) > 2 else 2)
params = init_params(cfg, 101, bias_scale=0.02)
rows = synthetic_rows(cfg, 6000, 102, state_scale=0.1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
_, out = run_case(cfg, params, rows, B=B, steps=1, seed=103)
res = out[0]
gg, g32, g64 = res["gpu"][2], res["o32"][2], res["o64"][2]
for k in sorted(g64):
    if k == "log_alpha":
        continue
    print(k, "gpu", rel(gg[k], g64[k]), "o32", rel(g32[k], g64[k]), "norm", np.linalg.norm(g64[k]))
k = sys.argv[3] if len(sys.argv) > 3 else "q1.fc1.weight"
d = (gg[k].astype(np.float64) - g64[k]); d32 = (g32[k].astype(np.float64) - g64[k])
col = np.linalg.norm(d, axis=0); rown = np.linalg.norm(d, axis=1)
print("worst cols", np.argsort(col)[-8:], col[np.argsort(col)[-8:]])
print("worst rows", np.argsort(rown)[-8:], rown[np.argsort(rown)[-8:]])
i, j = np.unravel_index(np.argmax(np.abs(d)), d.shape)
print("max elem", i, j, gg[k][i, j], g32[k][i, j], g64[k][i, j])
# dh1 / losses
print("losses gpu", res["gpu"][0], "o64", res["o64"][0])
