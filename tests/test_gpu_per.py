"""PER on the GPU vs the reference's PrioritizedReplayBuffer fixtures (tests/golden/per.npz).

Bit-exact: sampled indices, numpy MT19937 stream advance, update_priorities (last
duplicate wins), push-time max priority.  IS weights: within 4 ulp (the reference's
float32 ``**`` runs through numpy's SIMD pow, which is up to 1 ulp from powf —
SURVEY §0 C6)."""
import os

import numpy as np
import pytest

from oracle import per as P
from oracle.pyrandom import MT19937

pytestmark = pytest.mark.gpu


def _ctx(cap, batch=4096):
    from sacmi import Config, Context
    return Context(Config(1, 1, 4, max_batch=batch, capacity=cap, replay="per"), 0)


def _push(ctx, n):
    ctx.push(np.arange(n, dtype=np.float32).reshape(n, 1), np.zeros((n, 1), np.float32),
             np.zeros(n, np.float32), np.zeros((n, 1), np.float32), np.zeros(n, np.uint8))


@pytest.mark.parametrize("case", range(4))
def test_per_sample_matches_reference(golden_dir, case):
    z = np.load(os.path.join(golden_dir, "per.npz"))
    seed, n, batch, cap = (int(x) for x in z["cases"][case])
    ctx = _ctx(cap)
    _push(ctx, n)
    ctx.per_set_priorities(z[f"c{case}.prio_before"])
    from sacmi import _lib as L
    ctx.set_scalar(L.S_PER_FRAME, int(z[f"c{case}.frame"]))
    ctx.set_mt(1, z[f"c{case}.np_key"], int(z[f"c{case}.np_pos"]))
    idx, w = ctx.per_sample(batch)
    assert np.array_equal(idx, z[f"c{case}.idx"])
    ref_w = z[f"c{case}.weights"]
    ulp = np.spacing(np.maximum(np.abs(ref_w), np.float32(1e-30)))
    assert np.all(np.abs(w - ref_w) <= 4 * ulp), np.max(np.abs(w - ref_w) / ulp)
    key, pos = ctx.get_mt(1)
    assert pos == int(z[f"c{case}.np_post_pos"])
    assert np.array_equal(key, z[f"c{case}.np_post_key"])
    assert int(ctx.get_scalar(L.S_PER_FRAME)) == int(z[f"c{case}.frame"]) + 1
    # rows gathered by slot carry their push order (wrapped ring for case 2)
    s, *_ = ctx.get_slots(idx)
    assert np.array_equal(s[:, 0], z[f"c{case}.states"])
    # update_priorities: sequential, last duplicate wins
    vals = (z[f"c{case}.upd_prio"].astype(np.float64) + 1e-6).astype(np.float32)
    ctx.per_update(idx, vals)
    assert np.array_equal(ctx.per_priorities(), z[f"c{case}.prio_after"])
    # next push gets max(priorities) over the whole array
    _push(ctx, 1)
    assert np.array_equal(ctx.per_priorities(), z[f"c{case}.prio_after_push"])


def test_per_small_probabilities_fallback_exact():
    """Probabilities below 2^-29 take the sequential float64 cumsum path: indices
    still equal numpy's np.random.choice."""
    n = 3000
    ctx = _ctx(4096)
    _push(ctx, n)
    rng = np.random.default_rng(1)
    prio = rng.uniform(0, 1, 4096).astype(np.float32)
    prio[:n:7] = np.float32(1e-30)
    prio[5] = np.float32(1e6)
    ctx.per_set_priorities(prio)
    np.random.seed(3)
    st = np.random.get_state()
    ctx.set_mt(1, st[1], st[2])
    idx, w = ctx.per_sample(512)
    probs = P.probs_from(prio, n)
    ridx, _ = P.sample_from_probs(probs, 512, MT19937.from_npstate(st), P.beta_at(1))
    assert np.array_equal(idx, ridx)


def test_per_driven_update_runs_and_uses_slots():
    from oracle.sac_step import NETS, OracleSAC, SacConfig, init_params, synthetic_rows
    import torch
    from sacmi import Config, Context
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 81, bias_scale=0.05)
    rows = synthetic_rows(cfg, 300, 82, state_scale=0.5)
    ctxs = []
    for _ in range(2):
        c = Context(Config(24, 4, 64, max_batch=64, capacity=256, replay="per"), 0)
        for n in NETS:
            c.set_net(n, params[n])
        c.push(*rows)                                # wraps: 300 rows into 256 slots
        c.per_update(np.arange(256), np.linspace(0.1, 3, 256).astype(np.float32))
        c.set_mt(1, np.arange(624, dtype=np.uint32), 624)
        ctxs.append(c)
    idx, _ = ctxs[0].per_sample(64)                  # the indices the update will draw
    ctxs[1].step(64, eps1=np.zeros((64, 4), np.float32), eps2=np.zeros((64, 4), np.float32))
    # oracle on the slot rows
    s, a, r, s2, d = ctxs[0].get_slots(idx)
    o = OracleSAC(cfg, params, torch.float64)
    L = o.step(s, a, r, s2, d, np.zeros((64, 4), np.float32), np.zeros((64, 4), np.float32))
    st = ctxs[1].get_net("q1")
    assert np.isfinite(st["fc1.weight"]).all()
    got = ctxs[1].step(64, idx=None, eps1=np.zeros((64, 4), np.float32),
                       eps2=np.zeros((64, 4), np.float32))
    assert np.all(np.isfinite(got))
    # losses of the first update: recompute on a fresh pair for an exact comparison
    c = Context(Config(24, 4, 64, max_batch=64, capacity=256, replay="per"), 0)
    for n in NETS:
        c.set_net(n, params[n])
    c.push(*rows)
    c.per_update(np.arange(256), np.linspace(0.1, 3, 256).astype(np.float32))
    c.set_mt(1, np.arange(624, dtype=np.uint32), 624)
    lg = c.step(64, eps1=np.zeros((64, 4), np.float32), eps2=np.zeros((64, 4), np.float32))
    want = np.array([L["q1_loss"], L["q2_loss"], L["policy_loss"]])
    np.testing.assert_allclose(lg, want, rtol=1e-5)


@pytest.mark.parametrize("n,batch,bad", [(300_001, 4096, False), (70_000, 1000, True)])
def test_per_many_blocks_vs_oracle(n, batch, bad):
    """The fused 3-launch PER path over many 8192-row chunks and 1024-row scan blocks
    (block-total scan in LDS over >256 blocks, ragged last chunk and block): indices
    bit-exact vs the numpy-semantics oracle; the sequential-cumsum fallback too."""
    ctx = _ctx(n + 5, batch)
    _push(ctx, n)
    rng = np.random.default_rng(11)
    prio = rng.uniform(0.01, 2.0, n + 5).astype(np.float32)
    if bad:
        prio[::13] = np.float32(1e-25)
    ctx.per_set_priorities(prio)
    np.random.seed(5)
    st = np.random.get_state()
    ctx.set_mt(1, st[1], st[2])
    idx, w = ctx.per_sample(batch)
    probs = P.probs_from(prio, n)
    ridx, rw = P.sample_from_probs(probs, batch, MT19937.from_npstate(st), P.beta_at(1))
    assert np.array_equal(idx, ridx)
    ulp = np.spacing(np.maximum(np.abs(rw), np.float32(1e-30)))
    assert np.all(np.abs(w - rw) <= 4 * ulp)


def test_per_filling_buffer_one_graph_and_eager_identical():
    """A push-then-update loop on a PER context that is still filling (trainer.py:194-205
    with the prioritized buffer): the fused PER sampler reads the fill on the device, so
    ONE captured update graph serves every fill level (graph count constant), and the
    results are bit-identical to the eager (SACMI_NO_GRAPH=1) updates."""
    import torch  # noqa: F401
    from oracle.sac_step import NETS, SacConfig, init_params, synthetic_rows
    from sacmi import Config, Context
    from sacmi import _lib as L
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 91, bias_scale=0.05)
    rows = synthetic_rows(cfg, 1200, 92, state_scale=0.5)
    out = []
    for ng in ("0", "1"):
        os.environ["SACMI_NO_GRAPH"] = ng
        try:
            c = Context(Config(24, 4, 64, max_batch=64, capacity=20000, replay="per", seed=5), 0)
        finally:
            os.environ.pop("SACMI_NO_GRAPH", None)
        for n in NETS:
            c.set_net(n, params[n])
        c.push(*[x[:200] for x in rows])
        c.set_mt(1, np.arange(624, dtype=np.uint32) * 7 + 1, 624)
        counts, losses = [], []
        for i in range(50):
            lo = 200 + 20 * i
            c.push(*[x[lo:lo + 20] for x in rows])
            c.step_async(64)
            counts.append(int(c.get_scalar(L.S_GRAPH_COUNT)))
        losses = c.fetch_losses(50)
        out.append((counts, losses, {n: c.get_net(n) for n in NETS}, c.per_priorities(1200),
                    c.get_mt(1)))
        c.close()
    counts, losses, nets, prio, mt = out[0]
    assert len(c0 := set(counts)) == 1 and c0 == {1}, counts
    assert set(out[1][0]) == {0}                       # eager context: no graphs
    assert losses.shape == (50, 3) and np.all(np.isfinite(losses))
    assert np.array_equal(losses, out[1][1])
    for n in NETS:
        for k in nets[n]:
            assert np.array_equal(nets[n][k], out[1][2][n][k]), (n, k)
    assert np.array_equal(prio, out[1][3])
    assert np.array_equal(mt[0], out[1][4][0]) and mt[1] == out[1][4][1]
