"""Kernel-variant switches of the act16 (batch-4096, bf16) update, each bit for bit against
the form it replaces.

k_axk16p (the act16 dh levels on an LDS-DMA ring) against k_axk16 (register-staged slabs).

Both kernels accumulate every output element over K in the same order (64-deep slabs in
increasing k, two 16x16x32 bf16 MFMAs per slab and fragment with the same lane <-> operand
mapping), form the same bf16 A operand (u = [h2 > 0] bf16(w3) on the row-prologue levels,
the fp32 gradient rounded to bf16 on the plain ones), share the row prologue and the
coefficient / ReLU-mask epilogue, and store the same fp32 u rows for the weight gradient —
so whole updates (losses, parameters, gradients, Adam state) come out bit-identical with
either one.  The ring kernel is opt-in (SACMI_AXK16P=1, read per enqueue; measured slower,
DESIGN.md §12f).  Shapes: BASELINE
configs[4] per GPU (NAO S661 A23 H512, batch 4096, bf16): L5 / L9 (row prologue, 128x128
tiles, two critics: 256 workgroups), L12 (plain, one net: 64x128 tiles), and with three
hidden layers the plain two-critic levels (128x128).  A level that hosts a ride (L12 of an
update that gathers the next batch) stays on k_axk16.

The layer-L weight gradient forming its operand u = [h > 0] w_head from the bf16 activation
(opt-in, SACMI_DW_U_TRANSFORM=1: L5 stores no u rows; measured slower) against the u rows L5
stores (the default): the same fp32 values times the same coefficients, so the same bits.

k_dw_fin_p (the split-K weight gradients' fixed-order sum + Adam + Polyak on a looping grid,
the next block's loads issued before this block's stores; opt-in, SACMI_DWFIN_P=1, measured
slower) against k_dw_fin (one group per thread): the same per-group arithmetic, so the same
bits.
"""
import os

import numpy as np
import pytest

from oracle.sac_step import SacConfig, init_params, synthetic_rows
from test_gpu_parity import ctx_grads, ctx_state, load_params, make_ctx

pytestmark = pytest.mark.gpu

DH_SITES = ("gemm_L5_critic_dh1", "gemm_L9_act_dh1", "gemm_L12_pi_dhp1")


def run_updates(n_hidden, env):
    """Two injected updates and a 3-update launch at the config-5 shapes under the switches
    `env`; the losses, every tensor of every net (param / grad / Adam m, v) and the levels'
    kernels ({site: {(kernel, grid)}})."""
    os.environ.update(env)
    try:
        cfg = SacConfig(661, 23, 512, n_hidden=n_hidden)
        B = 4096
        params = init_params(cfg, 191, bias_scale=0.05)
        rows = synthetic_rows(cfg, 6000, 192, state_scale=0.5)
        rng = np.random.default_rng(193)
        ctx = make_ctx(cfg, max_batch=B, capacity=6000, compute_dtype="bf16", seed=7)
        load_params(ctx, params)
        ctx.push(*rows)
        assert ctx.act16(B)
        out = {}
        for t in range(2):
            idx = rng.choice(6000, B, replace=False)
            e1 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
            e2 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
            out[f"loss{t}"] = np.asarray(ctx.step(B, idx=idx, eps1=e1, eps2=e2), np.float64)
        ctx.step_many_async(B, 3)
        out["many"] = ctx.fetch_losses(3).ravel()
        for k, v in ctx_state(ctx, cfg).items():
            out["p." + k] = v
        for k, v in ctx_grads(ctx, cfg).items():
            out["g." + k] = v
        for n in ("policy", "q1", "q2"):
            for slot in ("m", "v"):
                for k, v in ctx.get_net(n, slot).items():
                    out[f"{slot}.{n}.{k}"] = v
        ks, _ = ctx.profile_timeline(B, 2)
        kern = {}
        for k in ks:
            if k["site"].startswith("gemm_L"):
                kern.setdefault(k["site"], set()).add((k["kernel"], k["grid"]))
        ctx.close()
        return out, kern
    finally:
        for k in env:
            os.environ.pop(k, None)


def assert_same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("n_hidden", [2, 3])
def test_axk16p_bitexact_vs_axk16(n_hidden):
    a, ka = run_updates(n_hidden, {"SACMI_AXK16P": "1"})
    b, kb = run_updates(n_hidden, {})
    ka = {s: {v for v in ks if v[0].startswith("k_axk16")} for s, ks in ka.items()}
    kb = {s: {v for v in ks if v[0].startswith("k_axk16")} for s, ks in kb.items()}
    # the ring kernel ran the two-critic row-prologue levels on one tile per CU ...
    for site in ("gemm_L5_critic_dh1", "gemm_L9_act_dh1"):
        assert ("k_axk16p", 256) in ka[site], (site, ka[site])
    # ... and L12 where no ride sits on it; the switch really switched
    assert any(kn == "k_axk16p" for kn, _ in ka["gemm_L12_pi_dhp1"]), ka["gemm_L12_pi_dhp1"]
    assert all(kn == "k_axk16" for v in kb.values() for kn, _ in v), kb
    if n_hidden == 3:
        assert sum(kn == "k_axk16p" for v in ka.values() for kn, _ in v) > 3, ka
    assert_same(a, b)


@pytest.mark.parametrize("n_hidden", [2, 3])
def test_dw_fin_p_bitexact_vs_dw_fin(n_hidden):
    a, ka = run_updates(n_hidden, {"SACMI_DWFIN_P": "1"})
    b, kb = run_updates(n_hidden, {})
    for site in ("gemm_L6_critic_dW_adam", "gemm_L13_pi_dW_adam"):
        assert {kn for kn, _ in ka[site]} >= {"k_dw_part16", "k_dw_fin_p"}, (site, ka[site])
        assert {kn for kn, _ in kb[site]} >= {"k_dw_part16", "k_dw_fin"}, (site, kb[site])
        assert "k_dw_fin_p" not in {kn for kn, _ in kb[site]}
    assert_same(a, b)


@pytest.mark.parametrize("n_hidden", [2, 3])
def test_dw_u_transform_bitexact_vs_u_rows(n_hidden):
    a, _ = run_updates(n_hidden, {"SACMI_DW_U_TRANSFORM": "1"})
    b, _ = run_updates(n_hidden, {})
    assert_same(a, b)
