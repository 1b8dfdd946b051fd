"""Pin the CPU oracle to the reference's own outputs (tests/golden/*.npz, produced by
tools/make_golden.py running the reference in the build container)."""
import os

import numpy as np
import pytest
import torch

from oracle import per as P
from oracle.pyrandom import MT19937, random_samples, sample_indices, sample_setsize
from oracle.sac_step import NETS, OracleSAC, SacConfig, init_params, synthetic_rows


def _z(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_uniform_indices_bitexact(golden_dir):
    z = _z(golden_dir, "idx_uniform.npz")
    for c, (seed, n, k) in enumerate(z["cases"]):
        mt = MT19937(z[f"c{c}.key"], int(z[f"c{c}.pos"]))
        idx = sample_indices(mt, int(n), int(k))
        assert np.array_equal(idx, z[f"c{c}.idx"]), (seed, n, k)
        assert mt.pos == int(z[f"c{c}.post_pos"])
        assert np.array_equal(mt.key, z[f"c{c}.post_key"])


def test_sample_errors_like_reference():
    mt = MT19937(np.arange(624, dtype=np.uint32), 624)
    with pytest.raises(ValueError, match="Sample larger than population"):
        sample_indices(mt, 10, 11)
    assert sample_setsize(256) == 1045 and sample_setsize(4096) == 16405


def test_numpy_random_sample_bridge():
    np.random.seed(5)
    st = np.random.get_state()
    ref = np.random.random_sample(9)
    mt = MT19937.from_npstate(st)
    assert np.array_equal(random_samples(mt, 9), ref)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 127, 128, 129, 1000, 8191, 8192, 8193, 70001])
def test_pairwise_sum_matches_numpy(n):
    a = (np.random.default_rng(n).uniform(0, 2, n).astype(np.float32)) ** np.float32(0.6)
    assert P.pairwise_sum_f32(a) == a.sum()


def test_per_oracle_bitexact(golden_dir):
    z = _z(golden_dir, "per.npz")
    for c, (seed, n, batch, cap) in enumerate(z["cases"]):
        L = min(int(n), int(cap))
        probs = P.probs_from(z[f"c{c}.prio_before"], L)
        assert np.array_equal(probs, z[f"c{c}.probs"])
        mt = MT19937(z[f"c{c}.np_key"], int(z[f"c{c}.np_pos"]))
        idx, w = P.sample_from_probs(probs, int(batch), mt, P.beta_at(int(z[f"c{c}.frame"])))
        assert np.array_equal(idx, z[f"c{c}.idx"])
        assert np.array_equal(w, z[f"c{c}.weights"])
        assert mt.pos == int(z[f"c{c}.np_post_pos"])
        up = P.update_priorities(z[f"c{c}.prio_before"], idx, z[f"c{c}.upd_prio"])
        assert np.array_equal(up, z[f"c{c}.prio_after"])
        pushed, pos, _ = P.push_priority(up, L, (int(n)) % int(cap), int(cap))
        assert np.array_equal(pushed, z[f"c{c}.prio_after_push"])
        assert pos == int(z[f"c{c}.pos_after_push"])


def _golden_params(z, cfg):
    from oracle.sac_step import param_shapes
    return {n: {k: z[f"in.{n}.{k}"] for k in param_shapes(cfg)[n]} for n in NETS}


@pytest.mark.parametrize("fixture", ["step_small.npz", "step_model2.npz"])
def test_oracle_fp32_bitexact_small(golden_dir, fixture):
    """step_model2.npz: networks_model2 (3 hidden layers) swapped into the reference SAC."""
    z = _z(golden_dir, fixture)
    S, A, H, B, N = (int(x) for x in z["cfg"][:5])
    cfg = SacConfig(S, A, H, n_hidden=int(z["cfg"][5]) if z["cfg"].size > 5 else 2)
    orc = OracleSAC(cfg, _golden_params(z, cfg), dtype=torch.float32)
    rows = [z[f"rows.{k}"] for k in ("s", "a", "r", "s2", "d")]
    for t in range(2):
        mt = MT19937(z[f"step{t}.mt_key"], int(z[f"step{t}.mt_pos"]))
        idx = sample_indices(mt, N, B)
        assert np.array_equal(idx, z[f"step{t}.idx"])
        L = orc.step(*[x[idx] for x in rows], z[f"step{t}.eps1"], z[f"step{t}.eps2"])
        assert np.array_equal([L["q1_loss"], L["q2_loss"], L["policy_loss"]], z[f"step{t}.losses"])
        st = orc.state()
        for k in z.files:
            if k.startswith(f"step{t}.out."):
                assert np.array_equal(st[k[len(f"step{t}.out."):]], z[k]), k


def test_oracle_fp32_bitexact_humanoid(golden_dir):
    z = _z(golden_dir, "step_humanoid.npz")
    S, A, H, B, N = (int(x) for x in z["cfg"])
    cfg = SacConfig(S, A, H)
    ps, rs = (int(x) for x in z["seeds"])
    params = init_params(cfg, ps, float(z["bias_scale"]))
    rows = synthetic_rows(cfg, N, rs, float(z["state_scale"]))
    orc = OracleSAC(cfg, params, dtype=torch.float32)
    stride = int(z["stride"])
    for t in range(2):
        idx = z[f"step{t}.idx"]
        L = orc.step(*[x[idx] for x in rows], z[f"step{t}.eps1"], z[f"step{t}.eps2"])
        assert np.array_equal([L["q1_loss"], L["q2_loss"], L["policy_loss"]], z[f"step{t}.losses"])
        st = orc.state()
        for k in z.files:
            pre = f"step{t}.sample."
            if k.startswith(pre):
                assert np.array_equal(st[k[len(pre):]].reshape(-1)[::stride], z[k]), k


@pytest.mark.parametrize("dims", [(24, 4, 64), (376, 17, 256)])
def test_dropin_networks_init_equals_reference(golden_dir, dims):
    """networks_model1 drop-in modules, built in SAC.__init__ order under the same torch
    seed, reproduce the reference's initial weights bit for bit (init_seed3.npz)."""
    from networks_model1 import GaussianPolicy, QNetwork
    z = np.load(os.path.join(golden_dir, "init_seed3.npz"))
    S, A, H = dims
    torch.manual_seed(3)
    mods = {"policy": GaussianPolicy(S, A, H)}
    for n in ("q1", "q2", "q1_target", "q2_target"):
        mods[n] = QNetwork(S, A, H)
    mods["q1_target"].load_state_dict(mods["q1"].state_dict())
    mods["q2_target"].load_state_dict(mods["q2"].state_dict())
    for n, m in mods.items():
        for k, v in m.state_dict().items():
            assert np.array_equal(v.numpy(), z[f"{S}_{A}_{H}.{n}.{k}"]), (n, k)


def test_dropin_networks_model2_init_equals_reference(golden_dir):
    """networks_model2 drop-in (orthogonal policy init, 3 hidden layers) reproduces the
    reference's initial weights under the same torch seed (init_seed3.npz, m2_ keys)."""
    from networks_model2 import GaussianPolicy, QNetwork
    z = np.load(os.path.join(golden_dir, "init_seed3.npz"))
    S, A, H = 24, 4, 64
    torch.manual_seed(3)
    mods = {"policy": GaussianPolicy(S, A, H)}
    for n in ("q1", "q2", "q1_target", "q2_target"):
        mods[n] = QNetwork(S, A, H)
    mods["q1_target"].load_state_dict(mods["q1"].state_dict())
    mods["q2_target"].load_state_dict(mods["q2"].state_dict())
    for n, m in mods.items():
        for k, v in m.state_dict().items():
            assert np.array_equal(v.numpy(), z[f"m2_{S}_{A}_{H}.{n}.{k}"]), (n, k)


def test_model2_key_layout():
    from sacmi.core import net_keys
    from oracle.sac_step import param_shapes
    cfg = SacConfig(24, 4, 64, n_hidden=3)
    for net in ("policy", "q1"):
        assert [k for k, _l, _p in net_keys(net, 3)] == list(param_shapes(cfg)[net])
    cfg2 = SacConfig(24, 4, 64)
    for net in ("policy", "q1"):
        assert [k for k, _l, _p in net_keys(net, 2)] == list(param_shapes(cfg2)[net])


def test_reference_checkpoint_fixture_matches_dropin_layout():
    """The reference's shipped best_model.pt files (Humanoid H=256 S=376 A=17, BipedalWalker
    S=24 A=4; fixture from tools/make_ckpt_fixture.py, weights_only loader): key sets, file
    order and shapes are exactly the drop-in networks' state_dict layout, and the rebuilt
    dicts load strictly into them with the reference's values at every sampled position."""
    import ckpt_fixture as cf
    from sacmi.networks import GaussianPolicy, QNetwork
    z, keys = cf.load_fixture()
    for tag in ("humanoid", "bipedal"):
        d = keys[tag]["dims"]
        ck = cf.rebuild(tag)
        mods = {"policy": GaussianPolicy(d["S"], d["A"], d["H"])}
        for n in ("q1", "q2", "q1_target", "q2_target"):
            mods[n] = QNetwork(d["S"], d["A"], d["H"])
        for n, m in mods.items():
            sd = ck[f"{n}_state_dict"]
            assert list(sd) == list(m.state_dict()), (tag, n)
            m.load_state_dict(sd)            # strict: same keys, same shapes
            for k, v in m.state_dict().items():
                p = f"{tag}.{n}.{k}"
                assert np.array_equal(v.numpy().reshape(-1)[z[p + ".idx"]], z[p + ".val"]), p
        assert torch.is_tensor(ck["alpha"]) and ck["alpha"].requires_grad


def test_forced_relu_masks_reproduce_the_unmasked_step():
    """OracleSAC.step(masks=...) evaluates the update under given ReLU decisions (the GPU's,
    in tests/test_gpu_parity.py).  Given the oracle's OWN decisions, it is the unmasked step
    bit for bit; one flipped decision moves the critic loss and the gradients."""
    import torch
    from oracle.sac_step import OracleSAC, SacConfig, init_params, synthetic_rows
    cfg = SacConfig(6, 2, 16)
    params = init_params(cfg, 3, bias_scale=0.1)
    s, a, r, s2, d = synthetic_rows(cfg, 8, 4, state_scale=0.5)
    rng = np.random.default_rng(5)
    e1, e2 = (rng.standard_normal((8, 2)).astype(np.float32) for _ in range(2))
    q1 = params["q1"]
    x = np.concatenate([s, a], 1).astype(np.float64)
    pre = x @ q1["fc1.weight"].T.astype(np.float64) + q1["fc1.bias"]
    own = {("q1", 0): (pre > 0).astype(np.float32)}
    ref = OracleSAC(cfg, params, torch.float64)
    l_ref = ref.step(s, a, r, s2, d, e1, e2)
    m = OracleSAC(cfg, params, torch.float64)
    l_m = m.step(s, a, r, s2, d, e1, e2, masks=own)
    assert l_ref == l_m
    for k, v in ref.grads_flat().items():
        assert np.array_equal(v, m.grads_flat()[k]), k
    flipped = {("q1", 0): own[("q1", 0)].copy()}
    i, j = np.argwhere(own[("q1", 0)] > 0)[0]
    flipped[("q1", 0)][i, j] = 0.0
    f = OracleSAC(cfg, params, torch.float64)
    l_f = f.step(s, a, r, s2, d, e1, e2, masks=flipped)
    assert l_f["q1_loss"] != l_ref["q1_loss"] and l_f["q2_loss"] == l_ref["q2_loss"]
    g_f, g_r = f.grads_flat()["q1.fc1.weight"], ref.grads_flat()["q1.fc1.weight"]
    assert not np.array_equal(g_f, g_r)
