"""k_fwd16p (the act16 forward levels on an LDS-DMA ring) against k_fwd16 (register-staged
slabs), bit for bit.

Both kernels accumulate every output element over K in the same order (64-deep slabs in
increasing k, two 16x16x32 bf16 MFMAs per slab and fragment, the same lane <-> operand
mapping), zero the same k >= K elements and share the FwdEpi epilogue, so a whole update
(losses, parameters, gradients, Adam state) must come out bit-identical with either one on
the forward levels.  The k_fwd16 run goes in a child process with SACMI_NO_FWD16P=1 (the
launcher reads the switch once per process).  Shapes: BASELINE configs[4] per GPU (NAO
S661 A23 H512, batch 4096, bf16): K = 685 / 662 (a partial last slab) on L1 / L3 / L7 and
K = 512 on L2 / L4 / L8; 256x128 tiles on L1 / L2, 128x128 on L3 / L4 / L7 / L8.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle.sac_step import SacConfig, init_params, synthetic_rows

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FWD_SITES = ("gemm_L1_fc1", "gemm_L2_fc2", "gemm_L3_tgt_fc1", "gemm_L4_tgt_fc2",
             "gemm_L7_act_fc1", "gemm_L8_act_fc2")


def run_updates(out_path, n_hidden=2):
    """Two updates at the config-5 shapes on fixed minibatches and noise; writes the
    losses, every tensor of every net (param / grad / Adam m, v) and the forward levels'
    kernel names (one instrumented multi-update graph) to out_path (.npz)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import ctx_grads, ctx_state, load_params, make_ctx
    cfg = SacConfig(661, 23, 512, n_hidden=n_hidden)
    B = 4096
    params = init_params(cfg, 91, bias_scale=0.05)
    rows = synthetic_rows(cfg, 6000, 92, state_scale=0.5)
    rng = np.random.default_rng(93)
    ctx = make_ctx(cfg, max_batch=B, capacity=6000, compute_dtype="bf16")
    load_params(ctx, params)
    ctx.push(*rows)
    assert ctx.act16(B)
    out = {}
    for t in range(2):
        idx = rng.choice(6000, B, replace=False)
        e1 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
        e2 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
        out[f"loss{t}"] = np.asarray(ctx.step(B, idx=idx, eps1=e1, eps2=e2), np.float64)
    for k, v in ctx_state(ctx, cfg).items():
        out["p." + k] = v
    for k, v in ctx_grads(ctx, cfg).items():
        out["g." + k] = v
    ks, _ = ctx.profile_timeline(B, 2)
    kern = {k["site"]: (k["kernel"], k["grid"]) for k in ks if k["site"] in FWD_SITES}
    out["kernels"] = np.frombuffer(json.dumps(kern).encode(), np.uint8)
    np.savez(out_path, **out)


@pytest.mark.parametrize("n_hidden", [2, 3])
def test_fwd16p_bitexact_vs_fwd16(tmp_path, n_hidden):
    new = tmp_path / "fwd16p.npz"
    old = tmp_path / "fwd16.npz"
    run_updates(str(new), n_hidden)
    env = dict(os.environ, SACMI_NO_FWD16P="1")
    paths = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "humanoid-walking-with-sac_amd")]
    code = (f"import sys; sys.path[:0] = {paths!r}; "
            f"import test_gpu_fwd16p as t; t.run_updates({str(old)!r}, {n_hidden})")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    a, b = np.load(new), np.load(old)
    ka = json.loads(bytes(a["kernels"]).decode())
    kb = json.loads(bytes(b["kernels"]).decode())
    assert set(ka) >= {"gemm_L1_fc1", "gemm_L2_fc2", "gemm_L3_tgt_fc1", "gemm_L7_act_fc1"}
    assert all(v[0] == "k_fwd16p" for v in ka.values()), ka
    assert all(v[0] == "k_fwd16" for v in kb.values()), kb
    assert ka["gemm_L1_fc1"][1] == 256 and ka["gemm_L3_tgt_fc1"][1] == 256   # one tile per CU
    keys = [k for k in a.files if k != "kernels"]
    assert keys == [k for k in b.files if k != "kernels"]
    for k in keys:
        assert np.array_equal(a[k], b[k]), k
