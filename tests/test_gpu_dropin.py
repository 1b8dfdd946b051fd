"""The drop-in modules (sac_imp / replay_buffer / networks_model1 names) on the GPU,
driven the way the reference's trainer.py drives them (trainer.py:182-209)."""
import random

import numpy as np
import pytest
import torch

from oracle.pyrandom import MT19937, sample_indices

pytestmark = pytest.mark.gpu

S, A, H = 24, 4, 64


def _agent(**kw):
    from sac_imp import SAC
    torch.manual_seed(0)
    kw.setdefault("capacity", 5000)
    return SAC(S, A, hidden_dim=H, device="cuda", max_batch=256, **kw)


def _fill(agent, n, seed=0):
    rng = np.random.default_rng(seed)
    for _ in range(n):    # the trainer pushes one transition per env step
        agent.replay_buffer.push(rng.standard_normal(S), rng.uniform(-0.4, 0.4, A).astype(np.float32),
                                 float(rng.standard_normal()), rng.standard_normal(S),
                                 bool(rng.random() < 0.02))


def test_trainer_loop_contract():
    agent = _agent()
    _fill(agent, 300)
    assert len(agent.replay_buffer) == 300
    hist = []
    for _ in range(5):
        if len(agent.replay_buffer) > 64:               # trainer.py:202 gate (strict)
            hist.append(agent.update_parameters(64))
    assert len(hist) == 5
    for h in hist:
        assert set(h) == {"q1_loss", "q2_loss", "policy_loss"}
        assert all(isinstance(v, float) and np.isfinite(v) for v in h.values())
    # alpha becomes exp(log_alpha) (a tensor) after the first update (sac_imp.py:135)
    assert torch.is_tensor(agent.alpha)
    np.testing.assert_allclose(float(agent.alpha), float(agent.log_alpha.exp()), rtol=1e-6)


def test_state_dicts_match_reference_layout_and_init():
    agent = _agent()
    sd = agent.policy.state_dict()
    assert list(sd) == ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "mean.weight",
                        "mean.bias", "log_std.weight", "log_std.bias"]
    assert tuple(agent.q1.state_dict()["fc1.weight"].shape) == (H, S + A)
    # targets start as copies (sac_imp.py:35-36)
    for k, v in agent.q1.state_dict().items():
        assert torch.equal(v, agent.q1_target.state_dict()[k])
    # device holds exactly the mirrors' values
    live = agent._ctx.get_net("policy")
    for k, v in sd.items():
        assert np.array_equal(live[k].reshape(v.shape), v.numpy())


def test_select_action_shapes_and_bounds():
    agent = _agent()
    a = agent.select_action(np.zeros(S))
    assert a.shape == (A,) and np.all(np.abs(a) <= 0.4)
    st = np.random.default_rng(1).standard_normal(S).astype(np.float32)
    det = agent.select_action(st, evaluate=True)
    with torch.no_grad():   # evaluate: tanh(mean)*scale+bias on the CPU mirror
        mean, _ = agent.policy(torch.from_numpy(st).unsqueeze(0))
        ref = (torch.tanh(mean) * 0.4).numpy()[0]
    np.testing.assert_allclose(det, ref, rtol=1e-5, atol=1e-5)
    b = agent.select_action(np.zeros((7, S)))
    assert b.shape == (7, A)


def test_sync_python_random_consumes_like_reference():
    agent = _agent(sync_python_random=True)
    _fill(agent, 2000)
    random.seed(123)
    pre = random.getstate()
    agent.update_parameters(256)
    mt = MT19937.from_pystate(pre)
    sample_indices(mt, 2000, 256)
    assert random.getstate() == mt.to_pystate()

    def device_state():
        key, pos = agent._ctx.get_mt(0)
        return tuple(int(x) for x in key) + (pos,)
    # the device sampler drew from the same state as Python's random.sample (the drop-in
    # runs the latter on the host while the GPU runs the update): the streams stay equal
    # through pushes, batch sizes on both sample branches, and the caller drawing from
    # `random` between updates (adopted by the next update)
    assert device_state() == random.getstate()[1]
    rng = np.random.default_rng(4)
    for t in range(6):
        agent.replay_buffer.push(rng.standard_normal(S), rng.uniform(-0.4, 0.4, A).astype(np.float32),
                                 0.5, rng.standard_normal(S), False)
        if t == 3:
            random.random()
        b = (256, 64, 8)[t % 3]
        pre = random.getstate()
        agent.update_parameters(b)
        mt = MT19937.from_pystate(pre)
        sample_indices(mt, len(agent.replay_buffer), b)
        assert random.getstate() == mt.to_pystate(), t
        assert device_state() == random.getstate()[1], t


def test_checkpoint_roundtrip(tmp_path):
    agent = _agent()
    _fill(agent, 400)
    for _ in range(3):
        agent.update_parameters(64)
    path = str(tmp_path / "ck.pt")
    agent.save_checkpoint(path, episode=7, total_steps=123)
    ck = torch.load(path, weights_only=True)
    for k in ("policy_state_dict", "q1_state_dict", "q1_optimizer_state_dict", "log_alpha",
              "alpha_optimizer_state_dict", "replay_buffer"):
        assert k in ck
    assert float(ck["q1_optimizer_state_dict"]["state"][0]["step"]) == 3.0
    other = _agent()
    ep, ts = other.load_checkpoint(path)
    assert (ep, ts) == (7, 123)
    assert len(other.replay_buffer) == 400
    for n in ("policy", "q1", "q2", "q1_target", "q2_target"):
        a, b = agent._ctx.get_net(n), other._ctx.get_net(n)
        for k in a:
            assert np.array_equal(a[k], b[k]), (n, k)
    for n in ("policy", "q1"):
        assert np.array_equal(agent._ctx.get_net(n, "m")["fc1.weight"],
                              other._ctx.get_net(n, "m")["fc1.weight"])
    # both continue identically from the same state and the same sampling stream
    key, pos = agent._ctx.get_mt(0)
    other._ctx.set_mt(0, key, pos)
    from sacmi import _lib as L
    other._ctx.set_scalar(L.S_NOISE_COUNTER, agent._ctx.get_scalar(L.S_NOISE_COUNTER))
    assert agent.update_parameters(64) == other.update_parameters(64)


def test_standalone_replay_buffer_is_random_sample():
    from replay_buffer import ReplayBuffer
    rb = ReplayBuffer(capacity=500)
    for i in range(700):
        rb.push(np.array([float(i), 0.5]), np.zeros(2, np.float32), float(i), np.zeros(2), False)
    assert len(rb) == 500
    random.seed(5)
    pre = random.getstate()
    s, a, r, s2, d = rb.sample(32)
    mt = MT19937.from_pystate(pre)
    want = sample_indices(mt, 500, 32) + 200          # deque position -> pushed id
    assert np.array_equal(s[:, 0], want.astype(np.float64))
    assert random.getstate() == mt.to_pystate()
    with pytest.raises(ValueError, match="Sample larger than population"):
        rb.sample(501)


def test_model2_dropin_checkpoint_and_update(tmp_path, golden_dir):
    """SAC(networks="model2"): the networks_model2 swap (sac_imp.py:4 import edited) —
    init equals the reference's under the same torch seed, fc1..fc4 / fc1..fc3+heads
    state dicts round-trip through the device, updates run."""
    import os
    from sac_imp import SAC
    z = np.load(os.path.join(golden_dir, "init_seed3.npz"))
    torch.manual_seed(3)
    agent = SAC(24, 4, hidden_dim=64, device="cuda", capacity=5000, max_batch=256,
                networks="model2")
    for n in ("policy", "q1", "q2", "q1_target", "q2_target"):
        live = agent._ctx.get_net(n)
        for k, v in getattr(agent, n).state_dict().items():
            # orthogonal_ runs a LAPACK QR: bitwise on the build host, ULP-level elsewhere
            np.testing.assert_allclose(v.numpy(), z[f"m2_24_4_64.{n}.{k}"], rtol=1e-5, atol=1e-5)
            assert np.array_equal(live[k].reshape(v.shape), v.numpy()), (n, k)
    assert list(agent.q1.state_dict())[-2:] == ["fc4.weight", "fc4.bias"]
    _fill(agent, 300)
    h = agent.update_parameters(64)
    assert all(np.isfinite(v) for v in h.values())
    p = str(tmp_path / "m2.pt")
    agent.save_checkpoint(p, 1, 300)
    torch.manual_seed(4)
    b = SAC(24, 4, hidden_dim=64, device="cuda", capacity=5000, max_batch=256, networks="model2")
    b.load_checkpoint(p)
    for n in ("policy", "q1_target"):
        for k, v in getattr(agent, n).state_dict().items():
            assert torch.equal(v, getattr(b, n).state_dict()[k]), (n, k)
    assert np.isfinite(b.update_parameters(64)["q1_loss"])


def test_select_action_graph_replays_track_state():
    """select_action replays one captured graph per (rows, evaluate): every call draws
    fresh noise (device-side counter), and the replay reads the live weights (after an
    update the deterministic action follows the new policy, == the CPU mirror)."""
    agent = _agent()
    _fill(agent, 300)
    st = np.random.default_rng(2).standard_normal(S).astype(np.float32)
    a1, a2 = agent.select_action(st), agent.select_action(st)
    assert not np.array_equal(a1, a2)
    d1 = agent.select_action(st, evaluate=True)
    assert np.array_equal(d1, agent.select_action(st, evaluate=True))
    for _ in range(3):
        agent.update_parameters(64)
    d2 = agent.select_action(st, evaluate=True)
    assert not np.array_equal(d1, d2)
    with torch.no_grad():
        mean, _ = agent.policy(torch.from_numpy(st).unsqueeze(0))
        ref = (torch.tanh(mean) * 0.4).numpy()[0]
    np.testing.assert_allclose(d2, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tag", ["humanoid", "bipedal"])
def test_loads_reference_checkpoint_fixture(tmp_path, tag):
    """The reference's own best_model.pt layouts (tests/golden/ckpt_reference.npz, from the
    shipped results/*/best_model.pt via a weights-only loader): the rebuilt dict, saved
    with torch.save, loads through SAC.load (sac_imp.py:165-173); every device tensor is
    the file's tensor bit for bit, alpha is the saved one, and the deterministic action of
    the loaded policy equals the CPU forward of the same weights."""
    import ckpt_fixture as cf
    from sac_imp import SAC
    from oracle.sac_step import _policy_forward
    z, keys = cf.load_fixture()
    d = keys[tag]["dims"]
    ck = cf.rebuild(tag)
    p = str(tmp_path / "best_model.pt")
    torch.save(ck, p)
    torch.manual_seed(1)
    agent = SAC(d["S"], d["A"], hidden_dim=d["H"], device="cuda", capacity=1000, max_batch=64)
    agent.load(p)
    for n in cf.NETS:
        live = agent._ctx.get_net(n)
        for k, v in ck[f"{n}_state_dict"].items():
            assert np.array_equal(live[k].reshape(v.shape), v.numpy()), (tag, n, k)
            idx = z[f"{tag}.{n}.{k}.idx"]
            assert np.array_equal(live[k].reshape(-1)[idx], z[f"{tag}.{n}.{k}.val"])
    assert float(agent.alpha) == float(z[f"{tag}.alpha"][0])
    st = np.random.default_rng(5).standard_normal((8, d["S"])).astype(np.float32)
    got = agent.select_action(st, evaluate=True)
    pol = {k: v.double() for k, v in ck["policy_state_dict"].items()}
    with torch.no_grad():
        mean, _ = _policy_forward(pol, torch.from_numpy(st).double())
        want = (torch.tanh(mean) * 0.4).numpy()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)


def test_checkpoint_restores_reference_list_buffer(tmp_path):
    """The replay restore branch of load_checkpoint (sac_imp.py:229-230): a buffer saved as
    the reference's list of (state, action, reward, next_state, done) tuples of numpy
    values (PrioritizedReplayBuffer.buffer, replay_buffer.py:28) is restored in order,
    bit for bit, and REPLACES a non-empty replay as the reference's assignment does; rows
    that do not fit the agent raise before anything of it is overwritten."""
    rng = np.random.default_rng(8)
    rows = [(rng.standard_normal(S), rng.uniform(-0.4, 0.4, A).astype(np.float32),
             float(rng.standard_normal()), rng.standard_normal(S), bool(rng.random() < 0.2))
            for _ in range(150)]
    src = _agent()
    p = str(tmp_path / "ck.pt")
    src.save_checkpoint(p, episode=3, total_steps=150, replay_buffer=False)
    ck = torch.load(p, weights_only=True)
    ck["replay_buffer"] = rows
    torch.save(ck, p)
    dst = _agent()
    assert dst.load_checkpoint(p) == (3, 150)
    assert len(dst.replay_buffer) == 150
    s, a, r, s2, d = dst.replay_buffer._rows_at(np.arange(150))
    for i, (si, ai, ri, s2i, di) in enumerate(rows):
        assert np.array_equal(s[i], si.astype(np.float32)) and np.array_equal(a[i], ai)
        assert r[i] == np.float32(ri) and np.array_equal(s2[i], s2i.astype(np.float32))
        assert bool(d[i]) == di
    full = _agent()
    _fill(full, 300)                     # 300 rows (some still staged on the host) ...
    full.load_checkpoint(p)              # ... replaced by the checkpoint's 150
    assert len(full.replay_buffer) == 150
    s3, a3, r3, s23, d3 = full.replay_buffer._rows_at(np.arange(150))
    assert np.array_equal(s3, s) and np.array_equal(a3, a) and np.array_equal(r3, r)
    assert np.array_equal(s23, s2) and np.array_equal(d3, d)
    _fill(full, 5, seed=9)               # pushes continue after the restored rows
    assert len(full.replay_buffer) == 155
    # a checkpoint whose rows do not fit: nothing of the agent is overwritten
    bad = dict(ck)
    bad["replay_buffer"] = [(np.zeros(S + 1), np.zeros(A, np.float32), 0.0, np.zeros(S + 1), False)]
    torch.save(bad, p)
    other = _agent()
    _fill(other, 100, seed=4)
    before = other._ctx.get_net("policy")
    with torch.no_grad():
        for prm in src.policy.parameters():
            prm.add_(1.0)
    bad["policy_state_dict"] = src.policy.state_dict()
    torch.save(bad, p)
    with pytest.raises(ValueError, match="do not fit"):
        other.load_checkpoint(p)
    after = other._ctx.get_net("policy")
    assert all(np.array_equal(before[k], after[k]) for k in before)
    assert len(other.replay_buffer) == 100


def test_select_action_stochastic_vs_oracle():
    """select_action(state, evaluate=False) (sac_imp.py:54-72 -> networks_model1.py:78-99)
    with the Normal noise injected: the action equals the oracle's policy sample
    tanh(mean + eps * std) * scale + bias on the same weights and eps within 1e-5."""
    from oracle.sac_step import SacConfig, _policy_sample, init_params
    cfg = SacConfig(376, 17, 512)
    params = init_params(cfg, 17, bias_scale=0.05)
    from sacmi import Config, Context
    ctx = Context(Config(376, 17, 512, max_batch=256, capacity=1000), 0)
    for n in ("policy", "q1", "q2", "q1_target", "q2_target"):
        ctx.set_net(n, params[n])
    rng = np.random.default_rng(18)
    for n in (1, 7, 64, 200):      # env-rate (pinned zero-copy) and batched (copy) paths
        st = (rng.standard_normal((n, 376)) * 0.5).astype(np.float32)
        eps = rng.standard_normal((n, 17)).astype(np.float32)
        got = ctx.act(st, deterministic=False, eps=eps)
        pol = {k: torch.tensor(v, dtype=torch.float64) for k, v in params["policy"].items()}
        with torch.no_grad():
            want, _ = _policy_sample(pol, torch.from_numpy(st).double(),
                                     torch.from_numpy(eps).double(), 0.4, 0.0)
        np.testing.assert_allclose(got, want.numpy(), rtol=1e-5, atol=1e-6, err_msg=f"n={n}")
    ctx.close()


def test_push_paths_store_identical_rows():
    """sacmi_push_packed (the drop-in's staged rows: mapped staging read by the scatter
    kernel for chunks of <= 16 rows, the copy path beyond) and sacmi_push store the same
    rows with the same deque(maxlen) positions — single rows, small and large chunks, across
    the ring's wrap (replay_memory.py push / deque semantics)."""
    from collections import deque

    from sacmi import Config, Context
    cap = 700
    ref = deque(maxlen=cap)
    rng = np.random.default_rng(5)
    ctx = Context(Config(S, A, hidden_dim=16, max_batch=64, capacity=cap), 0)
    w = 2 * S + A + 2
    for n, packed in [(1, True), (300, False), (5, True), (1, True), (40, True), (16, True),
                      (17, True), (250, False), (1, True), (123, True)]:
        s = rng.standard_normal((n, S)).astype(np.float32)
        a = rng.standard_normal((n, A)).astype(np.float32)
        r = rng.standard_normal(n).astype(np.float32)
        s2 = rng.standard_normal((n, S)).astype(np.float32)
        d = rng.random(n) < 0.3
        if packed:
            p = np.concatenate([s, a, r[:, None], s2, d[:, None].astype(np.float32)], axis=1)
            assert p.shape == (n, w)
            ctx.push_packed(np.ascontiguousarray(p), n)
        else:
            ctx.push(s, a, r, s2, d)
        for i in range(n):
            ref.append((s[i], a[i], r[i], s2[i], d[i]))
    assert len(ctx) == len(ref) == cap
    got = ctx.get_rows(np.arange(cap, dtype=np.int64))
    for k, col in enumerate(zip(*ref)):
        want = np.stack(col).astype(np.float32).reshape(got[k].shape)
        assert np.array_equal(got[k], want), k


def test_push_mailbox_updates_match_scatter_path():
    """The trainer's row per env step waits in the push mailbox and is stored by the next
    synchronous update's sampler kernel (sacmi.hip PushMailbox): the same updates as when
    every row goes through the scatter kernel first (here forced by a replay read before
    each update), bit for bit — across the ring's wrap (deque(maxlen)), with done flags,
    and with two rows between updates."""
    agents = []
    for _ in range(2):
        a = _agent(capacity=400)
        _fill(a, 380, seed=9)
        agents.append(a)
    rng = np.random.default_rng(10)
    for t in range(40):
        rows = [(rng.standard_normal(S), rng.uniform(-0.4, 0.4, A).astype(np.float32),
                 float(rng.standard_normal()), rng.standard_normal(S), bool(rng.random() < 0.2))
                for _ in range(1 if t % 5 else 2)]
        losses = []
        for k, a in enumerate(agents):
            for row in rows:
                a.replay_buffer.push(*row)
            if k == 1:                                   # the scatter path
                a.replay_buffer._flush()
                a._ctx.get_rows(np.zeros(1, np.int64))
            losses.append(a.update_parameters(64))
        assert losses[0] == losses[1], t
    for n in ("policy", "q1", "q2", "q1_target", "q2_target"):
        sa, sb = agents[0]._ctx.get_net(n), agents[1]._ctx.get_net(n)
        for k in sa:
            assert np.array_equal(sa[k], sb[k]), (n, k)
    n = len(agents[0].replay_buffer)
    ra = agents[0]._ctx.get_rows(np.arange(n, dtype=np.int64))
    rb = agents[1]._ctx.get_rows(np.arange(n, dtype=np.int64))
    for x, y in zip(ra, rb):
        assert np.array_equal(x, y)
