"""GPU parity: the HIP path (through the C ABI) against the oracle and the goldens.

Bars:
* replay indices, RNG state after sampling, Polyak (given our own online params):
  bit-exact;
* losses: relative error vs the fp64 oracle <= 1e-5;
* gradients (per tensor, normwise) vs the fp64 oracle <= 5e-5 — on well-conditioned
  inputs (states ~ N(0, 0.1^2) at Humanoid size, 0.5 at the small size);
* parameter deltas (per tensor) vs the fp64 oracle: within 4x (+ 1e-4 abs floor) of
  the deviation the reference's own fp32 step shows against the same fp64 truth
  (Adam's first steps are ~lr*sign(g): an fp32 re-association flips signs of
  near-zero gradient entries, so an elementwise 1e-5 bar is unattainable even by the
  reference itself — SURVEY §0 C5).
"""
import os

import numpy as np
import pytest
import torch

from oracle.pyrandom import MT19937, sample_indices
from oracle.sac_step import NETS, OracleSAC, SacConfig, init_params, param_shapes, synthetic_rows

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-5
# gradients, per tensor normwise vs fp64: 1e-5 at batch <= 1024 on
# well-conditioned inputs, or 4x the reference's own fp32 deviation where that is larger;
# the achieved errors are printed (and appended to $SACMI_GRAD_TABLE as JSON lines)
GRAD_TOL = 1e-5
# batch 4096 (allow_flips): 5e-5 against plain fp64, else explained by ReLU flips alone
GRAD_TOL_B4096 = 5e-5
# batch 4096: a few of the ~2-4 M ReLU pre-activations land within fp32 rounding of zero,
# and WHICH ones flip against fp64 depends on the fp32 summation order; a flipped mask
# bit in a deep layer perturbs every shallower layer's gradient through the chain (the
# reference's own fp32 step, on the same inputs, measured up to 1.2e-4 from fp64 on the
# GPU box's CPU torch).  A tensor over the bar passes only if the flips are the whole
# story: within MASKED_GRAD_TOL of fp64 evaluated under the GPU's own masks, with every
# flipped decision at an fp64 pre-activation within FLIP_Z_TOL of its layer's largest
# |pre-activation| (flip_evidence)
FLIP_Z_TOL = 1e-5


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / max(nb, 1e-30))


def make_ctx(cfg: SacConfig, max_batch, capacity, **kw):
    from sacmi import Config, Context
    c = Config(cfg.state_dim, cfg.action_dim, cfg.hidden_dim, max_batch=max_batch,
               gamma=cfg.gamma, tau=cfg.tau, lr=cfg.lr, alpha=cfg.alpha,
               automatic_entropy_tuning=cfg.automatic_entropy_tuning, capacity=capacity,
               n_hidden=cfg.n_hidden, **kw)
    ctx = Context(c, 0)
    from sacmi import _lib as L
    ctx.set_scalar(L.S_KEEP_GRADS, 1)     # the tests compare gradients too
    return ctx


@pytest.fixture(scope="module")
def nccl_world1():
    """One 1-rank RCCL process group for the module's data-parallel tests (initialised once,
    destroyed after the last of them): no process-group teardown / re-init between tests."""
    import socket
    import torch.distributed as dist
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    torch.cuda.synchronize()
    dist.destroy_process_group()


def load_params(ctx, params):
    for n in NETS:
        ctx.set_net(n, params[n])


def ctx_state(ctx, cfg):
    from sacmi import _lib as L
    shapes = param_shapes(cfg)
    out = {}
    for n in NETS:
        for k, v in ctx.get_net(n, "param", shapes[n]).items():
            out[f"{n}.{k}"] = v
    out["log_alpha"] = np.array([ctx.get_scalar(L.S_LOG_ALPHA)], np.float32)
    return out


def ctx_grads(ctx, cfg):
    from sacmi import _lib as L
    shapes = param_shapes(cfg)
    out = {}
    for n in ("policy", "q1", "q2"):
        for k, v in ctx.get_net(n, "grad", shapes[n]).items():
            out[f"{n}.{k}"] = v
    out["log_alpha"] = np.array([ctx.get_scalar(L.S_GRAD_LOG_ALPHA)], np.float32)
    return out


def ctx_alpha_state(ctx):
    """log_alpha, its Adam moments and every optimizer's step count (sac_imp.py:128-135)."""
    from sacmi import _lib as L
    g = ctx.get_scalar
    return {"log_alpha": g(L.S_LOG_ALPHA), "adam.log_alpha.m": g(L.S_ADAM_M_LOG_ALPHA),
            "adam.log_alpha.v": g(L.S_ADAM_V_LOG_ALPHA), "alpha": g(L.S_ALPHA),
            "steps": [g(L.S_STEP_POLICY), g(L.S_STEP_Q1), g(L.S_STEP_Q2), g(L.S_STEP_ALPHA)]}


def oracle_from_ctx(ctx, cfg, dtype):
    """An oracle agent holding EXACTLY the GPU context's current training state (params,
    targets, Adam moments and steps, log_alpha and its Adam state, alpha): the next update
    of both starts from identical inputs, so its losses can be held to LOSS_TOL."""
    shapes = param_shapes(cfg)
    params = {n: ctx.get_net(n, "param", shapes[n]) for n in NETS}
    o = OracleSAC(cfg, params, dtype)
    al = ctx_alpha_state(ctx)
    steps = dict(zip(("policy", "q1", "q2"), al["steps"][:3]))
    for n in ("policy", "q1", "q2"):
        if steps[n] == 0:
            continue
        m, v = ctx.get_net(n, "m", shapes[n]), ctx.get_net(n, "v", shapes[n])
        for k, t in o.nets[n].items():
            o.opt[n].state[t] = {"step": torch.tensor(float(steps[n])),
                                 "exp_avg": torch.tensor(m[k], dtype=dtype),
                                 "exp_avg_sq": torch.tensor(v[k], dtype=dtype)}
    with torch.no_grad():
        o.log_alpha.fill_(float(np.float32(al["log_alpha"])))
    if al["steps"][3] > 0:
        o.opt["alpha"].state[o.log_alpha] = {
            "step": torch.tensor(float(al["steps"][3])),
            "exp_avg": torch.tensor([al["adam.log_alpha.m"]], dtype=dtype),
            "exp_avg_sq": torch.tensor([al["adam.log_alpha.v"]], dtype=dtype)}
        o.alpha = torch.tensor([al["alpha"]], dtype=dtype)   # the GPU's fp32 exp(log_alpha)
    return o


def run_case(cfg, params, rows, B, steps, seed, with_idx=True):
    """Returns per-step (losses, state, grads) for gpu / oracle fp32 / oracle fp64.  From
    the second update on, both oracles are re-anchored on the GPU's state (oracle_from_ctx)
    so that every update is compared on identical inputs."""
    ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]))
    load_params(ctx, params)
    ctx.push(*rows)
    o32 = OracleSAC(cfg, params, torch.float32)
    o64 = OracleSAC(cfg, params, torch.float64)
    rng = np.random.default_rng(seed)
    out = []
    for t in range(steps):
        if t:
            o32, o64 = oracle_from_ctx(ctx, cfg, torch.float32), oracle_from_ctx(ctx, cfg, torch.float64)
        idx = rng.choice(len(rows[2]), B, replace=False)
        e1 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
        e2 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
        lg = ctx.step(B, idx=idx, eps1=e1, eps2=e2)
        batch = [x[idx] for x in rows]
        l32 = o32.step(*batch, e1, e2)
        l64 = o64.step(*batch, e1, e2)
        out.append(dict(gpu=(lg, ctx_state(ctx, cfg), ctx_grads(ctx, cfg)), alpha=ctx_alpha_state(ctx),
                        o32=(l32, o32.state(), o32.grads_flat()),
                        o64=(l64, o64.state(), o64.grads_flat())))
    return ctx, out


def split_flips(d, ref):
    """(normwise error, flip count) of a parameter delta against a reference delta, with
    flip-like elements set aside: an element whose delta differs by more than a quarter of
    the tensor's largest reference delta took an Adam step of the other sign (a gradient
    within fp32 summation noise of zero), which any fp32 evaluation order
    may do.  The rest must agree closely."""
    d = np.asarray(d, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    flips = np.abs(d - ref) > 0.25 * max(np.abs(ref).max(), 1e-30)
    return rel(d[~flips], ref[~flips]), int(flips.sum())


def check_delta_vs_reference(d_gpu, d_o64, ref, what):
    """GPU delta vs the reference's fp32 delta, graded against the fp64 truth's distance
    from that same reference delta: no more flip-like elements than max(2, 4x the truth's,
    0.2 %), and on the others within 4x the truth's error (+1e-4)."""
    e_g, f_g = split_flips(d_gpu, ref)
    e_o, f_o = split_flips(d_o64, ref)
    assert f_g <= max(2, 4 * f_o, int(0.002 * np.size(ref))), (what, "flips", f_g, f_o)
    assert e_g <= 4 * e_o + 1e-4, (what, "delta", e_g, e_o)


def report_grad_errors(name, tol, table, second="fp32_ref", strict=False):
    """Print the achieved per-tensor gradient errors (GPU vs fp64, and the reference's own
    fp32 vs fp64 — or `second`) and append them to $SACMI_GRAD_TABLE when set.  strict: the
    bar is `tol` alone (no 4x-reference escape)."""
    print(f"\n[grad errors] {name} (bar {tol:g}{'' if strict else ' or 4x fp32 ref'})")
    for k, (e, e_ref) in sorted(table.items()):
        ok = e <= (tol if strict else max(tol, 4 * e_ref))
        print(f"  {k:28s} gpu {e:9.3e}  {second} {e_ref:9.3e}  {'ok' if ok else 'OVER'}")
    path = os.environ.get("SACMI_GRAD_TABLE")
    if path:
        import json
        with open(path, "a") as f:
            f.write(json.dumps({"case": name, "bar": tol, "second": second,
                                "tensors": {k: {"gpu": e, second: r} for k, (e, r) in table.items()}}) + "\n")


def check_step(res, prev, name, allow_flips=False, masked=None):
    lg, sg, gg = res["gpu"]
    l32, s32, g32 = res["o32"]
    l64, s64, g64 = res["o64"]
    for i, k in enumerate(("q1_loss", "q2_loss", "policy_loss")):
        assert abs(lg[i] - l64[k]) <= LOSS_TOL * max(abs(l64[k]), 1e-3), (name, k, lg[i], l64[k])
    bad = {}
    tol = GRAD_TOL_B4096 if allow_flips else GRAD_TOL
    table = {}
    for k, v in g64.items():
        # the bar, or 4x the reference's own fp32 deviation where that is larger
        e, e_ref = rel(gg[k], v), rel(g32[k], v)
        table[k] = (e, e_ref)
        if e > max(tol, 4 * e_ref):
            if allow_flips and masked is not None and rel(gg[k], masked[k]) <= MASKED_GRAD_TOL:
                continue
            bad[k] = (e, e_ref)
    report_grad_errors(name, tol, table)
    assert not bad, (name, "grad", bad)
    for k in sg:
        p0 = prev.get(k, np.zeros(1))            # log_alpha starts at 0 (sac_imp.py:49)
        d_gpu = sg[k].astype(np.float64) - p0
        d_64 = s64[k].astype(np.float64) - p0
        d_32 = s32[k].astype(np.float64) - p0
        e_gpu, e_ref = rel(d_gpu, d_64), rel(d_32, d_64)
        if allow_flips and e_gpu > 4 * e_ref + 1e-4:
            # Adam's first step is lr*g/(|g|+eps) ~ lr*sign(g): one flip-perturbed
            # near-zero gradient entry moves a 512-entry bias delta by ~9 %.  The update
            # is checked against the HIP path's OWN gradient instead (fp64 Adam step /
            # Polyak of the online delta): that isolates the optimizer kernels
            net, key = k.split(".", 1)
            if net.endswith("_target"):
                # Polyak with the reference's three separately rounded fp32 ops: bit-exact
                src = net[:-len("_target")]
                tau = np.float32(0.005)
                t_old = prev[k].astype(np.float32)
                want32 = t_old * (np.float32(1) - tau) + sg[f"{src}.{key}"] * tau
                assert np.array_equal(sg[k], want32), (name, "polyak", k)
                continue
            else:
                g = gg[k].astype(np.float64)
                want = -3e-4 * g / (np.abs(g) + 1e-8)
            e_own = rel(d_gpu, want)
            assert e_own <= 1e-4, (name, "delta vs own gradient", k, e_own)
            continue
        assert e_gpu <= 4 * e_ref + 1e-4, (name, "delta", k, e_gpu, e_ref)
    if "alpha" in res:                          # the alpha optimizer (sac_imp.py:128-135)
        al = res["alpha"]
        for key in ("adam.log_alpha.m", "adam.log_alpha.v"):
            want = float(np.asarray(s64[key]).reshape(-1)[0])
            assert abs(al[key] - want) <= GRAD_TOL_B4096 * abs(want) + 1e-12, (name, key, al[key], want)
        a64 = float(s64["alpha"])
        assert abs(al["alpha"] - a64) <= LOSS_TOL * a64, (name, "alpha", al["alpha"], a64)
        st64 = float(np.asarray(s64["adam.policy.step"]))
        assert al["steps"] == [st64] * 4, (name, "optimizer steps", al["steps"], st64)


def flat_params(params):
    return {f"{n}.{k}": np.asarray(v, np.float64) for n in params for k, v in params[n].items()}


def test_step_small_vs_oracle():
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 31, bias_scale=0.05)
    rows = synthetic_rows(cfg, 500, 32, state_scale=0.5)
    _, out = run_case(cfg, params, rows, B=32, steps=3, seed=33)
    prev = flat_params(params)
    for t, res in enumerate(out):   # every update, each on the GPU's state before it
        check_step(res, prev, f"small step {t}")
        prev = {k: v.astype(np.float64) for k, v in res["gpu"][1].items()}


def test_step_bipedal_config1_vs_oracle():
    """BASELINE configs[0] shapes (BipedalWalker-v3: obs 24, act 4, hidden 256, batch 256)."""
    cfg = SacConfig(24, 4, 256)
    params = init_params(cfg, 81, bias_scale=0.05)
    rows = synthetic_rows(cfg, 2000, 82, state_scale=0.5)
    _, out = run_case(cfg, params, rows, B=256, steps=1, seed=83)
    check_step(out[0], flat_params(params), "bipedal config 1 step 0")


def test_step_humanoid_vs_oracle():
    cfg = SacConfig(376, 17, 512)
    params = init_params(cfg, 41, bias_scale=0.02)
    rows = synthetic_rows(cfg, 3000, 42, state_scale=0.1)
    _, out = run_case(cfg, params, rows, B=256, steps=1, seed=43)
    check_step(out[0], flat_params(params), "humanoid step 0")   # (step 2: the re-anchored test)


def test_step_humanoid_second_step_reanchored():
    """The second update (alpha is now exp(log_alpha), Adam past its first step) held to
    the same bars as the first (losses 1e-5 vs fp64, gradients 5e-5, deltas, alpha state):
    the oracles start from exactly the GPU's state after update 1 (oracle_from_ctx), so
    only update 2's arithmetic is compared."""
    cfg = SacConfig(376, 17, 512)
    params = init_params(cfg, 41, bias_scale=0.02)
    rows = synthetic_rows(cfg, 3000, 42, state_scale=0.1)
    ctx, out = run_case(cfg, params, rows, B=256, steps=1, seed=43)
    check_step(out[0], flat_params(params), "humanoid step 0")
    prev = {k: v.astype(np.float64) for k, v in out[0]["gpu"][1].items()}
    o32, o64 = oracle_from_ctx(ctx, cfg, torch.float32), oracle_from_ctx(ctx, cfg, torch.float64)
    rng = np.random.default_rng(44)
    idx = rng.choice(len(rows[2]), 256, replace=False)
    e1 = rng.standard_normal((256, cfg.action_dim)).astype(np.float32)
    e2 = rng.standard_normal((256, cfg.action_dim)).astype(np.float32)
    lg = ctx.step(256, idx=idx, eps1=e1, eps2=e2)
    batch = [x[idx] for x in rows]
    l32, l64 = o32.step(*batch, e1, e2), o64.step(*batch, e1, e2)
    res = dict(gpu=(lg, ctx_state(ctx, cfg), ctx_grads(ctx, cfg)), alpha=ctx_alpha_state(ctx),
               o32=(l32, o32.state(), o32.grads_flat()), o64=(l64, o64.state(), o64.grads_flat()))
    check_step(res, prev, "humanoid step 1 (re-anchored)")


@pytest.mark.parametrize("n_hidden", [2, 3])
def test_step_humanoid_b4096_vs_oracle(n_hidden):
    """Batch 4096 (BASELINE configs[2] shapes): the batch-4096-class level kernels against
    plain fp64 at 5e-5 per gradient tensor; a tensor over that bar must be explained by
    ReLU flips alone (flip_evidence: within 1e-5 of fp64 under the GPU's own masks, every
    flipped decision at a pre-activation within FLIP_Z_TOL of zero, relative to its layer)."""
    cfg = SacConfig(376, 17, 512, n_hidden=n_hidden)
    params = init_params(cfg, 101, bias_scale=0.02)
    rows = synthetic_rows(cfg, 6000, 102, state_scale=0.1)
    B = 4096
    ctx, out = run_case(cfg, params, rows, B=B, steps=1, seed=103)
    rng = np.random.default_rng(103)                       # run_case's draws for its update
    idx = rng.choice(len(rows[2]), B, replace=False)
    e1 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
    e2 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
    masks = gpu_relu_masks(ctx, cfg, B)
    gm, _, zmax = flip_evidence(cfg, params, [x[idx] for x in rows], e1, e2, masks)
    assert zmax <= FLIP_Z_TOL, ("a flipped ReLU decision away from zero", zmax)
    check_step(out[0], flat_params(params), f"humanoid B4096 n_hidden {n_hidden}", allow_flips=True,
               masked=gm)
    ctx.close()


@pytest.mark.parametrize("fixture", ["step_small.npz", "step_model2.npz"])
def test_golden_small_two_steps_device_sampling(golden_dir, fixture):
    """Indices drawn ON THE GPU from the reference's MT state reproduce the
    reference's update (losses vs the reference's own fp32 outputs); step_model2.npz is
    the reference SAC with networks_model2 (3 hidden layers)."""
    z = np.load(os.path.join(golden_dir, fixture))
    S, A, H, B, N = (int(x) for x in z["cfg"][:5])
    cfg = SacConfig(S, A, H, n_hidden=int(z["cfg"][5]) if z["cfg"].size > 5 else 2)
    params = {n: {k: z[f"in.{n}.{k}"] for k in param_shapes(cfg)[n]} for n in NETS}
    ctx = make_ctx(cfg, max_batch=B, capacity=N)
    load_params(ctx, params)
    ctx.push(*[z[f"rows.{k}"] for k in ("s", "a", "r", "s2", "d")])
    ctx.set_mt(0, z["step0.mt_key"], int(z["step0.mt_pos"]))
    for t in range(2):
        lg = ctx.step(B, idx=None, eps1=z[f"step{t}.eps1"], eps2=z[f"step{t}.eps2"])
        ref = z[f"step{t}.losses"]
        np.testing.assert_allclose(lg, ref, rtol=2e-5, atol=1e-7)
        # the generator advanced exactly as CPython's did
        if t == 0:
            key, pos = ctx.get_mt(0)
            mt = MT19937(z["step0.mt_key"], int(z["step0.mt_pos"]))
            sample_indices(mt, N, B)
            assert pos == mt.pos and np.array_equal(key, mt.key)
    st = ctx_state(ctx, cfg)
    # the fp64 truth on the same minibatches and noise: the two-update parameter deltas
    # must sit within 4x its own distance from the reference's fp32 deltas
    o64 = OracleSAC(cfg, params, torch.float64)
    rows = [z[f"rows.{k}"] for k in ("s", "a", "r", "s2", "d")]
    for t in range(2):
        i = z[f"step{t}.idx"]
        o64.step(*[x[i] for x in rows], z[f"step{t}.eps1"], z[f"step{t}.eps2"])
    so = o64.state()
    for n in NETS:
        for k in param_shapes(cfg)[n]:
            ref = z[f"step1.out.{n}.{k}"].astype(np.float64) - params[n][k]
            check_delta_vs_reference(st[f"{n}.{k}"] - params[n][k], so[f"{n}.{k}"] - params[n][k],
                                     ref, (fixture, n, k))
    np.testing.assert_allclose(st["log_alpha"], z["step1.out.log_alpha"], rtol=1e-5, atol=1e-9)
    assert abs(ctx.get_scalar(1) - float(z["step1.out.alpha"])) < 1e-6


def test_step_model2_vs_oracle():
    """networks_model2 (3 hidden layers, networks_model2.py:18-99): the extra hidden
    GEMM levels (forward, critic / actor-pass dh, policy dh) against the fp64 oracle."""
    cfg = SacConfig(24, 4, 64, n_hidden=3)
    params = init_params(cfg, 51, bias_scale=0.05)
    rows = synthetic_rows(cfg, 500, 52, state_scale=0.5)
    _, out = run_case(cfg, params, rows, B=32, steps=1, seed=53)
    check_step(out[0], flat_params(params), "model2 small step 0")


def test_step_model2_humanoid_vs_oracle():
    cfg = SacConfig(376, 17, 512, n_hidden=3)
    params = init_params(cfg, 61, bias_scale=0.02)
    rows = synthetic_rows(cfg, 2000, 62, state_scale=0.1)
    _, out = run_case(cfg, params, rows, B=256, steps=1, seed=63)
    check_step(out[0], flat_params(params), "model2 humanoid step 0")


def test_golden_humanoid_losses(golden_dir):
    z = np.load(os.path.join(golden_dir, "step_humanoid.npz"))
    S, A, H, B, N = (int(x) for x in z["cfg"])
    cfg = SacConfig(S, A, H)
    ps, rs = (int(x) for x in z["seeds"])
    params = init_params(cfg, ps, float(z["bias_scale"]))
    rows = synthetic_rows(cfg, N, rs, float(z["state_scale"]))
    ctx = make_ctx(cfg, max_batch=B, capacity=N)
    load_params(ctx, params)
    ctx.push(*rows)
    ctx.set_mt(0, z["step0.mt_key"], int(z["step0.mt_pos"]))
    stride = int(z["stride"])
    o64 = OracleSAC(cfg, params, torch.float64)
    prev_g = prev_o = flat_params(params)
    for t in range(2):
        lg = ctx.step(B, eps1=z[f"step{t}.eps1"], eps2=z[f"step{t}.eps2"])
        # the reference's own fp32 losses (sac_imp.py:140-144), same minibatch and noise
        np.testing.assert_allclose(lg, z[f"step{t}.losses"], rtol=LOSS_TOL, atol=1e-7)
        idx = z[f"step{t}.idx"]
        o64.step(*[x[idx] for x in rows], z[f"step{t}.eps1"], z[f"step{t}.eps2"])
        sg, so = ctx_state(ctx, cfg), o64.state()
        # parameter deltas against the REFERENCE's (strided samples + per-tensor norms of
        # its delta): within 4x the fp64 truth's own distance from the reference's fp32
        # step (Adam's ~lr*sign(g) first steps flip on near-zero gradients)
        for k in prev_g:
            ref_s = z[f"step{t}.sample.{k}"].astype(np.float64)
            ref_d = ref_s - prev_r[k] if t else ref_s - prev_g[k].reshape(-1)[::stride]
            d_g = (sg[k].astype(np.float64) - prev_g[k]).reshape(-1)
            d_o = (so[k].astype(np.float64) - prev_o[k]).reshape(-1)
            check_delta_vs_reference(d_g[::stride], d_o[::stride], ref_d, (t, k, "delta samples"))
            dn = float(z[f"step{t}.dnorm.{k}"])
            if dn > 0:
                n_g, n_o = abs(np.linalg.norm(d_g) - dn) / dn, abs(np.linalg.norm(d_o) - dn) / dn
                assert n_g <= 4 * n_o + 1e-4, (t, k, "delta norm", n_g, n_o)
        prev_r = {k: z[f"step{t}.sample.{k}"].astype(np.float64) for k in prev_g}
        prev_g = {k: sg[k].astype(np.float64) for k in prev_g}
        prev_o = {k: so[k].astype(np.float64) for k in prev_g}


@pytest.mark.parametrize("case", range(12))
def test_device_random_sample_bitexact(golden_dir, case):
    z = np.load(os.path.join(golden_dir, "idx_uniform.npz"))
    seed, n, k = (int(x) for x in z["cases"][case])
    cfg = SacConfig(1, 1, 16)
    ctx = make_ctx(cfg, max_batch=max(k, 1), capacity=n)
    ctx.push(np.arange(n, dtype=np.float32).reshape(n, 1), np.zeros((n, 1), np.float32),
             np.zeros(n, np.float32), np.zeros((n, 1), np.float32), np.zeros(n, np.uint8))
    ctx.set_mt(0, z[f"c{case}.key"], int(z[f"c{case}.pos"]))
    idx = ctx.sample_indices(k)
    assert np.array_equal(idx, z[f"c{case}.idx"])
    key, pos = ctx.get_mt(0)
    assert pos == int(z[f"c{case}.post_pos"])
    assert np.array_equal(key, z[f"c{case}.post_key"])


def test_device_random_sample_after_wraparound():
    """Deque positions map through the ring head once the buffer is full."""
    cfg = SacConfig(2, 1, 16)
    cap, n = 300, 770
    ctx = make_ctx(cfg, max_batch=64, capacity=cap)
    s = np.stack([np.arange(n), -np.arange(n)], 1).astype(np.float32)
    ctx.push(s, np.zeros((n, 1)), np.arange(n, dtype=np.float32), s, np.zeros(n, np.uint8))
    assert len(ctx) == cap
    rows_s, _, rows_r, _, _ = ctx.get_rows(np.arange(cap))
    assert np.array_equal(rows_r, np.arange(n - cap, n, dtype=np.float32))
    assert np.array_equal(rows_s[:, 0], np.arange(n - cap, n, dtype=np.float32))


@pytest.mark.parametrize("replay", ["uniform", "per"])
def test_push_chunks_and_wrap_exact(replay):
    """Ingest through the pinned staging slots (1024-row chunks, two slots in flight):
    pushes of 1, 1023, 1500 and 3000 rows into a 2500-row ring — chunk edges, ring wrap
    inside a chunk, a push larger than the ring (deque(maxlen) keeps the last rows) —
    land bit for bit in deque order; the device fill the sampler reads matches len."""
    S, A = 37, 5
    cfg = SacConfig(S, A, 16)
    cap = 2500
    ctx = make_ctx(cfg, max_batch=64, capacity=cap, replay=replay)
    rng = np.random.default_rng(5)
    hist = []
    for n in (1, 1023, 1500, 3000, 7):
        rows = (rng.standard_normal((n, S)).astype(np.float32),
                rng.standard_normal((n, A)).astype(np.float32),
                rng.standard_normal(n).astype(np.float32),
                rng.standard_normal((n, S)).astype(np.float32),
                rng.random(n) < 0.3)
        ctx.push(*rows)
        hist.append(rows)
        want = [np.concatenate([h[j] for h in hist])[-cap:] for j in range(5)]
        L = min(cap, len(want[2]))
        assert len(ctx) == L
        got = ctx.get_rows(np.arange(L))
        for j in range(5):
            assert np.array_equal(got[j], want[j]), (n, j)
    if replay == "uniform":
        idx = ctx.sample_indices(64)
        assert idx.min() >= 0 and idx.max() < cap and len(set(idx.tolist())) == 64
    else:
        assert ctx.per_priorities(cap).max() == 1.0


def test_polyak_bitexact_and_determinism():
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 51, bias_scale=0.05)
    rows = synthetic_rows(cfg, 400, 52, state_scale=0.5)
    outs = []
    from sacmi import _lib as L
    for keep in (1, 0):          # gradient export on/off: same bits, targets included
        ctx = make_ctx(cfg, max_batch=64, capacity=400)
        ctx.set_scalar(L.S_KEEP_GRADS, keep)
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, (np.arange(624, dtype=np.uint64) * 2654435761 % (2**32)).astype(np.uint32), 624)
        for _ in range(3):
            before_t = {n: ctx.get_net(n) for n in ("q1_target", "q2_target")}
            ctx.step(64)                           # device indices + device noise
        after = {n: ctx.get_net(n) for n in NETS}
        tau = np.float32(0.005)
        omt = np.float32(1.0 - 0.005)
        for tn, on in (("q1_target", "q1"), ("q2_target", "q2")):
            for k in after[tn]:
                exp = (before_t[tn][k] * omt + after[on][k] * tau).astype(np.float32)
                assert np.array_equal(after[tn][k], exp), (tn, k)
        outs.append(after)
    for n in NETS:
        for k in outs[0][n]:
            assert np.array_equal(outs[0][n][k], outs[1][n][k]), (n, k)


@pytest.mark.parametrize("shape", ["small", "nao_b4096_bf16", "nao_b4096_bf16_set", "nao_b4096_bf16_m2",
                                   "per_b4096"])
def test_many_updates_per_launch_identical(shape):
    """sacmi_step_many_async(n) (trainer.py:203-204 loop in one launch) == n single
    launches, bit for bit, losses included — also at the config-5 shapes (batch 4096,
    bf16: the LDS-staged level kernels, split-K dW with its XCD placement, device
    sampling of 4096 rows — the pool branch at 6,000 rows, the set branch at 20,000; the
    next update's sampler forked beside L6 and its gather beside L12 on the side stream) and
    with prioritized replay at batch 4096 (config 3: the PER sampler on the side stream)."""
    from sacmi import _lib as L
    replay = "uniform"
    if shape == "small":
        cfg, B, nrows, dt = SacConfig(24, 4, 64), 64, 500, "fp32"
    elif shape == "per_b4096":
        cfg, B, nrows, dt, replay = SacConfig(376, 17, 512), 4096, 9000, "fp32", "per"
    else:
        cfg, B, nrows, dt = SacConfig(661, 23, 512), 4096, 6000, "bf16"
        if shape.endswith("_set"):
            nrows = 20000
        if shape.endswith("_m2"):                  # networks_model2: L2b / L5b / L9b / L11
            cfg, nrows = SacConfig(661, 23, 512, n_hidden=3), 20000
    params = init_params(cfg, 61, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 62, state_scale=0.5)
    prio = np.random.default_rng(64).uniform(0.1, 2.0, nrows).astype(np.float32)
    res = []
    for many in (True, False):
        ctx = make_ctx(cfg, max_batch=B, capacity=nrows, compute_dtype=dt, replay=replay)
        load_params(ctx, params)
        ctx.push(*rows)
        if replay == "per":
            ctx.per_set_priorities(prio)
            ctx.set_mt(1, (np.arange(624, dtype=np.uint64) * 69069 % (2**32)).astype(np.uint32), 624)
        ctx.set_mt(0, (np.arange(624, dtype=np.uint64) * 40503 % (2**32)).astype(np.uint32), 624)
        if many:
            ctx.step_many_async(B, 5)
            ctx.step_many_async(B, 2)
        else:
            for _ in range(7):
                ctx.step_async(B)
        res.append((ctx.fetch_losses(7), {n: ctx.get_net(n) for n in NETS},
                    ctx.get_mt(0 if replay == "uniform" else 1), ctx.get_scalar(L.S_PER_FRAME)))
        ctx.close()
    assert np.array_equal(res[0][0], res[1][0]) and res[0][0].shape == (7, 3)
    for n in NETS:
        for k in res[0][1][n]:
            assert np.array_equal(res[0][1][n][k], res[1][1][n][k]), (n, k)
    assert np.array_equal(res[0][2][0], res[1][2][0]) and res[0][2][1] == res[1][2][1]
    assert res[0][3] == res[1][3]


def test_bf16_shadows_stay_current():
    """bf16 mode keeps bf16 shadows of the weights for the batch-4096 level kernels, written
    by every Adam / Polyak store.  A context whose shadows are re-derived from its own
    parameters between updates (set_net -> refresh) must update exactly like one that
    relies on the in-kernel shadow writes: a stale shadow would change the next update."""
    cfg = SacConfig(661, 23, 512)
    B, nrows = 4096, 6000
    params = init_params(cfg, 81, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 82, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 40503 % (2**32)).astype(np.uint32)
    ctxs = []
    for _ in range(2):
        ctx = make_ctx(cfg, max_batch=B, capacity=nrows, compute_dtype="bf16")
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, key, 624)
        ctxs.append(ctx)
    a, b = ctxs
    for _ in range(2):
        a.step_async(B)
        b.step_async(B)
    for n in NETS:                          # b: shadows re-derived from its own weights
        b.set_net(n, b.get_net(n))
    a.step_async(B)
    b.step_async(B)
    assert np.array_equal(a.fetch_losses(3), b.fetch_losses(3))
    for n in NETS:
        pa, pb = a.get_net(n), b.get_net(n)
        for k in pa:
            assert np.array_equal(pa[k], pb[k]), (n, k)


def test_batch_larger_than_buffer_raises():
    cfg = SacConfig(3, 2, 16)
    ctx = make_ctx(cfg, max_batch=32, capacity=100)
    ctx.push(np.zeros((10, 3)), np.zeros((10, 2)), np.zeros(10), np.zeros((10, 3)), np.zeros(10))
    with pytest.raises(ValueError, match="Sample larger than population"):
        ctx.step(11)


def test_graph_and_eager_identical():
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 61, bias_scale=0.05)
    rows = synthetic_rows(cfg, 400, 62, state_scale=0.5)
    res = []
    for ng in ("0", "1"):
        os.environ["SACMI_NO_GRAPH"] = ng
        try:
            ctx = make_ctx(cfg, max_batch=64, capacity=400, seed=7)
        finally:
            os.environ.pop("SACMI_NO_GRAPH", None)
        load_params(ctx, params)
        ctx.push(*rows)
        ls = [ctx.step(64) for _ in range(3)]
        res.append((np.array(ls), {n: ctx.get_net(n) for n in NETS}))
    assert np.array_equal(res[0][0], res[1][0])
    for n in NETS:
        for k in res[0][1][n]:
            assert np.array_equal(res[0][1][n][k], res[1][1][n][k])


def test_rng_seed_device_rekeys_noise():
    """sacmi_rng_seed_device: a context re-keyed to (seed, 0) updates exactly like one
    created with that seed; re-keying after the update graphs were captured takes effect
    (a new key changes the next update, the same key and counter change nothing)."""
    from sacmi import _lib as L
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 71, bias_scale=0.05)
    rows = synthetic_rows(cfg, 400, 72, state_scale=0.5)

    def fresh(seed):
        ctx = make_ctx(cfg, max_batch=64, capacity=400, seed=seed)
        load_params(ctx, params)
        ctx.push(*rows)
        return ctx

    a, f = fresh(11), fresh(99)
    f.rng_seed_device(11, 0)
    for _ in range(2):
        assert np.array_equal(a.step(64), f.step(64))
    for n in NETS:
        pa, pf = a.get_net(n), f.get_net(n)
        for k in pa:
            assert np.array_equal(pa[k], pf[k])
    b, c, d = fresh(99), fresh(99), fresh(99)
    l1 = [x.step(64) for x in (b, c, d)]               # graphs captured under key 99
    assert np.array_equal(l1[0], l1[1]) and np.array_equal(l1[0], l1[2])
    b.rng_seed_device(11, 1)
    c.rng_seed_device(99, 1)
    assert b.get_scalar(L.S_NOISE_COUNTER) == 1
    lb, lc, ld = b.step(64), c.step(64), d.step(64)
    assert np.array_equal(lc, ld)
    assert not np.array_equal(lb, ld)


@pytest.mark.parametrize("n_hidden,dtype,B", [(2, "fp32", 64), (3, "fp32", 64), (2, "bf16", 64),
                                              (2, "bf16", 2048), (3, "bf16", 2048)])
def test_dp_phase_path_matches_fused_step_world1(n_hidden, dtype, B, nccl_world1):
    """sacmi.dp over a 1-rank RCCL group (phases + in-place all-reduce on the adopted
    torch gradient arena) == the fused single-graph update, bit for bit (also for
    networks_model2 and the bf16 compute dtype)."""
    from sacmi.dp import DataParallelUpdate, GpuBackend
    ctxs, upd = [], None
    try:
        cfg = SacConfig(24, 4, 64, n_hidden=n_hidden)
        params = init_params(cfg, 71, bias_scale=0.05)
        rows = synthetic_rows(cfg, max(400, B + 300), 72, state_scale=0.5)
        key = (np.arange(624, dtype=np.uint64) * 40503 % (2**32)).astype(np.uint32)
        ctxs = []
        for _ in range(2):
            ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]), seed=3, compute_dtype=dtype)
            load_params(ctx, params)
            ctx.push(*rows)
            ctx.set_mt(0, key, 624)
            ctxs.append(ctx)
        upd = DataParallelUpdate(GpuBackend(ctxs[0], torch.device("cuda", 0)))
        for _ in range(3):
            upd(B)
            ctxs[1].step(B)
        upd.flush()
        torch.cuda.synchronize()
        for n in NETS:
            a, b = ctxs[0].get_net(n), ctxs[1].get_net(n)
            for k in a:
                assert np.array_equal(a[k], b[k]), (n, k)
        assert ctxs[0].get_scalar(0) == ctxs[1].get_scalar(0)
    finally:
        # every context closed (and the updater holding the adopted torch gradient arena
        # dropped) before the next test, on a drained device
        torch.cuda.synchronize()
        del upd
        for c in ctxs:
            c.close()


BF16_EMU_LOSS_TOL = 1e-4   # relative, vs the oracle emulating the bf16 operands
BF16_EMU_GRAD_TOL = 2e-2   # per-tensor normwise, vs that emulation (rounding flips of
                           # fp32-order-dependent operands, amplified by batch cancellation)
BF16_TRUTH_GRAD_TOL = 0.15  # vs the exact fp64 oracle (cosine >= ~0.99)


def _check_bf16_update(cfg, lb, gb, emu, exact, l_emu):
    """One bf16 update against the fp64 oracle with the HIP path's bf16 operand roundings
    (emu, after its step) and the exact fp64 oracle (exact, after its step)."""
    g_emu = emu.grads_flat()
    g64 = exact.grads_flat()
    for i, k in enumerate(("q1_loss", "q2_loss", "policy_loss")):
        assert abs(lb[i] - l_emu[k]) <= BF16_EMU_LOSS_TOL * max(abs(l_emu[k]), 1e-2), (k, lb[i], l_emu[k])
    keys = [k for k in g64 if k != "log_alpha"]
    e_emu = {k: rel(gb[k], g_emu[k]) for k in keys}
    e_true = {k: rel(gb[k], g64[k]) for k in keys}
    print("bf16 grad error vs emulation", {k: f"{e:.2e}" for k, e in e_emu.items()})
    print("bf16 grad error vs exact", {k: f"{e:.2e}" for k, e in e_true.items()})
    assert max(e_emu.values()) <= BF16_EMU_GRAD_TOL, e_emu
    # where bf16 moves a gradient most, the emulation accounts for most of the move
    worst = max(keys, key=lambda k: e_true[k])
    assert e_emu[worst] <= 0.25 * e_true[worst], (worst, e_emu[worst], e_true[worst])
    assert max(e_true.values()) <= BF16_TRUTH_GRAD_TOL, e_true
    # the bf16 operands really were used: the fp32 path is ~1e-6 from the truth
    assert max(e_true.values()) > 1e-3, e_true


@pytest.mark.parametrize("S,A,n_hidden,B", [(376, 17, 2, 256), (376, 17, 3, 256), (376, 17, 2, 4096),
                                           (376, 17, 3, 4096), (661, 23, 2, 4096)])
def test_bf16_compute_vs_emulation(S, A, n_hidden, B):
    """compute_dtype bf16 (BASELINE configs[4]; (661, 23, 512, B=4096): configs[4]'s own
    NAO shapes): bf16 MFMA operands, fp32 accumulation, fp32 master weights / Adam / losses.
    No reference counterpart: checked against the fp64 oracle with the same operands
    rounded to bf16 where the HIP path rounds them (oracle/sac_step.py _EmuLinear) — the
    deviation from exact arithmetic is bf16's own (fc1 dW ~7 %: strong cancellation over the
    batch), the kernel's extra error is accumulation-order level.  A second update is held
    to the same bars on oracles re-anchored on the GPU's state after the first
    (oracle_from_ctx: Adam past its first step, alpha = exp(log_alpha), sac_imp.py:135)."""
    cfg = SacConfig(S, A, 512, n_hidden=n_hidden)
    params = init_params(cfg, 71, bias_scale=0.02)
    rows = synthetic_rows(cfg, max(2000, B + 1000), 72, state_scale=0.1)
    rng = np.random.default_rng(73)
    draws = []
    for _ in range(2):
        draws.append((rng.choice(len(rows[2]), B, replace=False),
                      rng.standard_normal((B, cfg.action_dim)).astype(np.float32),
                      rng.standard_normal((B, cfg.action_dim)).astype(np.float32)))
    idx, e1, e2 = draws[0]
    res = {}
    act16 = None
    ctx_b = None
    for dt in ("fp32", "bf16"):
        ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]), compute_dtype=dt)
        load_params(ctx, params)
        ctx.push(*rows)
        if dt == "bf16":
            act16 = ctx.act16(B)
            assert act16 == (B >= 4096)        # bf16-stored activations at the batch-4096 class
        lg = ctx.step(B, idx=idx, eps1=e1, eps2=e2)
        res[dt] = (lg, ctx_grads(ctx, cfg))
        # one update = one step of each optimizer (the actor-pass row prologue advances
        # them exactly once, whichever kernel runs it) and alpha = exp(log_alpha)
        from sacmi import _lib as L
        for which in (L.S_STEP_POLICY, L.S_STEP_Q1, L.S_STEP_Q2, L.S_STEP_ALPHA):
            assert ctx.get_scalar(which) == 1.0, (dt, which)
        la = ctx.get_scalar(L.S_LOG_ALPHA)
        assert abs(ctx.get_scalar(L.S_ALPHA) - np.exp(np.float32(la))) <= 1e-6
        if dt == "bf16":
            ctx_b = ctx
        else:
            ctx.close()
    batch = [x[idx] for x in rows]
    emu = OracleSAC(cfg, params, torch.float64)
    l_emu = emu.step(*batch, e1, e2, bf16_operands=True, bf16_act=act16)
    exact = OracleSAC(cfg, params, torch.float64)
    exact.step(*batch, e1, e2)
    lb, gb = res["bf16"]
    _check_bf16_update(cfg, lb, gb, emu, exact, l_emu)
    assert not np.array_equal(res["fp32"][0], lb)
    # update 2 on re-anchored oracles
    emu2 = oracle_from_ctx(ctx_b, cfg, torch.float64)
    exact2 = oracle_from_ctx(ctx_b, cfg, torch.float64)
    assert abs(float(emu2.alpha.reshape(-1)[0]) - float(np.exp(np.float32(ctx_b.get_scalar(L.S_LOG_ALPHA))))) <= 1e-6
    idx, e1, e2 = draws[1]
    lb2 = ctx_b.step(B, idx=idx, eps1=e1, eps2=e2)
    gb2 = ctx_grads(ctx_b, cfg)
    batch = [x[idx] for x in rows]
    l_emu2 = emu2.step(*batch, e1, e2, bf16_operands=True, bf16_act=act16)
    exact2.step(*batch, e1, e2)
    _check_bf16_update(cfg, lb2, gb2, emu2, exact2, l_emu2)
    for which in (L.S_STEP_POLICY, L.S_STEP_Q1, L.S_STEP_Q2, L.S_STEP_ALPHA):
        assert ctx_b.get_scalar(which) == 2.0, which
    ctx_b.close()


@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("n_hidden", [2, 3])
def test_native_dp_world1_matches_fused(n_hidden, sharded):
    """sacmi_step_dp: the library's own RCCL data-parallel sequence (phases + in-place
    all-reduces, one captured graph per (batch, n), ride-along sampling) over a 1-rank
    communicator == the same number of fused single-GPU updates, bit for bit.
    sharded: the ZeRO-1 form through real RCCL calls — the error flags' all-reduce, the
    in-place reduce-scatter into chunk r and the in-place all-gather (at one rank the whole
    range is the chunk) inside the captured graph."""
    from sacmi import Context
    cfg = SacConfig(24, 4, 64, n_hidden=n_hidden)
    params = init_params(cfg, 91, bias_scale=0.05)
    rows = synthetic_rows(cfg, 400, 92, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 69069 % (2**32)).astype(np.uint32)
    ctxs = []
    for _ in range(2):
        ctx = make_ctx(cfg, max_batch=64, capacity=400, seed=5)
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, key, 624)
        ctxs.append(ctx)
    uid = Context.allreduce_unique_id()
    assert len(uid) == 128
    ctxs[0].allreduce_init(uid, 0, 1)
    ctxs[0].dp_set_sharded(sharded)   # (dp_sharded() reads 0 at one rank: the fused path's)
    ctxs[0].step_dp(64, 5)
    ctxs[0].step_dp(64, 1)
    for _ in range(6):
        ctxs[1].step(64)
    ctxs[0].synchronize()
    for n in NETS:
        a, b = ctxs[0].get_net(n), ctxs[1].get_net(n)
        for k in a:
            assert np.array_equal(a[k], b[k]), (n, k)
    from sacmi import _lib as L
    assert ctxs[0].get_scalar(L.S_LOG_ALPHA) == ctxs[1].get_scalar(L.S_LOG_ALPHA)
    hist = ctxs[0].fetch_losses(6)
    assert hist.shape == (6, 3) and np.all(np.isfinite(hist))
    with pytest.raises(Exception):
        ctxs[1].step_dp(64, 1)            # no communicator on this context


@pytest.mark.parametrize("sharded", [False, True])
def test_native_dp_world1_matches_fused_act16(sharded):
    """The same at config 5's per-GPU shape (NAO S661 A23 H512, batch 4096, bf16): the
    phase-split levels store bf16 activations exactly as the fused ones (act16), the
    split-K weight gradients go through the same k_dw_part16 / k_dw_fin path (plain store
    + k_adam instead of the fused Adam epilogue): bit for bit after three updates (sharded:
    the bf16 shadows re-derived after the in-place all-gather)."""
    from sacmi import Context
    cfg = SacConfig(661, 23, 512)
    B = 4096
    params = init_params(cfg, 93, bias_scale=0.05)
    rows = synthetic_rows(cfg, 20000, 94, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 40503 % (2**32)).astype(np.uint32)
    ctxs = []
    for _ in range(2):
        ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]), seed=5, compute_dtype="bf16")
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, key, 624)
        ctxs.append(ctx)
    assert ctxs[0].act16(B)
    ctxs[0].allreduce_init(Context.allreduce_unique_id(), 0, 1)
    ctxs[0].dp_set_sharded(sharded)
    ctxs[0].step_dp(B, 3)
    fused = np.stack([ctxs[1].step(B) for _ in range(3)])
    ctxs[0].synchronize()
    for n in NETS:
        a, b = ctxs[0].get_net(n), ctxs[1].get_net(n)
        for k in a:
            assert np.array_equal(a[k], b[k]), (n, k)
    # the loss ring of the data-parallel updates against the losses step() returns
    hist = ctxs[0].fetch_losses(3)
    assert hist.shape == (3, 3)
    np.testing.assert_allclose(hist, fused, rtol=1e-6, atol=1e-7)


def _config4_ctxs(k, cfg, params, rows, prio, key, B):
    ctxs = []
    for _ in range(k):
        ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]), seed=9, replay="per")
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.per_set_priorities(prio)
        ctx.set_mt(1, key, 624)                   # the rank's numpy stream (PER uniforms)
        ctxs.append(ctx)
    return ctxs


def _assert_same_agent(a, b, what):
    from sacmi import _lib as L
    for n in NETS:
        x, y = a.get_net(n), b.get_net(n)
        for k in x:
            assert np.array_equal(x[k], y[k]), (what, n, k)
    for s in (L.S_LOG_ALPHA, L.S_ADAM_M_LOG_ALPHA, L.S_ADAM_V_LOG_ALPHA, L.S_PER_FRAME,
              L.S_STEP_POLICY, L.S_STEP_Q1):
        assert a.get_scalar(s) == b.get_scalar(s), (what, s)
    assert np.array_equal(a.get_mt(1)[0], b.get_mt(1)[0]), (what, "numpy MT stream")


def test_dp_config4_per_shard_world1_matches_fused(nccl_world1):
    """BASELINE configs[3] per-GPU work (Humanoid S376 A17 H512, fp32, batch 4096, this
    rank's PRIORITIZED replay shard sampled on the device inside phase 0): the data-parallel
    update over a 1-rank RCCL group — eager torch.distributed driver and the library's own
    sacmi_step_dp — equals the fused
    single-GPU update bit for bit (parameters, alpha state, PER frame, numpy MT stream)."""
    from sacmi.dp import DataParallelUpdate, GpuBackend
    from sacmi import Context
    ctxs, upd = [], None
    try:
        B = 4096
        cfg = SacConfig(376, 17, 512)
        params = init_params(cfg, 111, bias_scale=0.02)
        rows = synthetic_rows(cfg, 12000, 112, state_scale=0.3)
        rng = np.random.default_rng(113)
        prio = rng.uniform(0.05, 2.0, 12000).astype(np.float32)
        key = rng.integers(0, 2**32, 624, dtype=np.uint32)
        dev = torch.device("cuda", 0)
        # eager driver: 2 updates vs 2 fused
        a, f = _config4_ctxs(2, cfg, params, rows, prio, key, B)
        ctxs += [a, f]
        upd = DataParallelUpdate(GpuBackend(a, dev))
        for _ in range(2):
            upd(B)
            f.step(B)
        upd.flush()
        torch.cuda.synchronize()
        _assert_same_agent(a, f, "eager dp")
        a.close(); f.close()
        # the library-issued collectives
        n, f = _config4_ctxs(2, cfg, params, rows, prio, key, B)
        ctxs += [n, f]
        n.allreduce_init(Context.allreduce_unique_id(), 0, 1)
        n.step_dp(B, 2)
        n.step_dp(B, 1)
        for _ in range(3):
            f.step(B)
        n.synchronize()
        _assert_same_agent(n, f, "native dp")
    finally:
        torch.cuda.synchronize()
        del upd
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("B,H", [(256, 512), (1024, 512), (1024, 768)])
def test_dlda_fold_matches_unfolded(B, H):
    """dL/da folded into the dha1 level's epilogue (per-32-column partials, summed by the
    sample-backward tail) vs the standalone dL/da GEMM (SACMI_NO_DLDA_FOLD=1): the same
    update up to fp32 summation order — every gradient within 1e-5 normwise, losses equal
    (they are computed before the actor backward).  Batch 1024 with hidden 768 has more
    32x64 tiles than the one-wave-group form takes: the fold steps aside (no error)."""
    cfg = SacConfig(376, 17, H)
    params = init_params(cfg, 141, bias_scale=0.02)
    rows = synthetic_rows(cfg, max(3000, B + 500), 142, state_scale=0.1)
    rng = np.random.default_rng(143)
    idx = rng.choice(len(rows[2]), B, replace=False)
    e1 = rng.standard_normal((B, 17)).astype(np.float32)
    e2 = rng.standard_normal((B, 17)).astype(np.float32)
    res = []
    for fold in (True, False):
        if not fold:
            os.environ["SACMI_NO_DLDA_FOLD"] = "1"
        try:
            ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]))
            load_params(ctx, params)
            ctx.push(*rows)
            lg = ctx.step(B, idx=idx, eps1=e1, eps2=e2)
            res.append((lg, ctx_grads(ctx, cfg)))
            ctx.close()
        finally:
            os.environ.pop("SACMI_NO_DLDA_FOLD", None)
    (la, ga), (lb, gb) = res
    assert np.array_equal(la[:2], lb[:2])
    assert abs(la[2] - lb[2]) <= 1e-6 * abs(lb[2]) + 1e-9
    for k in gb:
        assert rel(ga[k], gb[k]) <= 1e-5, (k, rel(ga[k], gb[k]))


@pytest.mark.parametrize("sharded", [True, False])
@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("shape", ["config2", "config5_act16"])
def test_native_dp_loopback_world_k_bitexact(world, shape, sharded):
    """The library's data-parallel sequence (sacmi_step_dp, sacmi.hip enqueue_dp) with
    world > 1 arithmetic on one GPU: each all-reduce becomes an in-place x world over the
    same range (what `world` ranks with identical shards produce) and Adam applies 1/world.
    Both scalings are exact for a power-of-two world, so the result equals the fused
    updates BIT FOR BIT only if every gradient element — dL/dlog_alpha included — lies
    inside [q_begin, q_end) or [pi_begin, total) and 1/world is applied exactly once
    (global batch = the ranks' batches concatenated).
    sharded: the ZeRO-1 form (reduce-scatter -> Adam on each rank's chunk -> all-gather),
    every rank's chunk run in turn: the chunks must tile both ranges exactly, and the
    alpha / loss bookkeeping must happen once."""
    from sacmi import _lib as L
    if shape == "config2":
        cfg, B, dt, nrows, n = SacConfig(376, 17, 512), 256, "fp32", 4000, 4
    else:
        cfg, B, dt, nrows, n = SacConfig(661, 23, 512), 4096, "bf16", 20000, 2
    params = init_params(cfg, 95, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 96, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 1812433 % (2**32)).astype(np.uint32)
    ctxs = []
    for _ in range(2):
        ctx = make_ctx(cfg, max_batch=B, capacity=nrows, seed=5, compute_dtype=dt)
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, key, 624)
        ctxs.append(ctx)
    ctxs[0].dp_loopback_init(world)
    ctxs[0].dp_set_sharded(sharded)
    ctxs[0].step_dp(B, n)
    fused = np.stack([ctxs[1].step(B) for _ in range(n)])
    ctxs[0].synchronize()
    for nm in NETS:
        a, b = ctxs[0].get_net(nm), ctxs[1].get_net(nm)
        for k in a:
            assert np.array_equal(a[k], b[k]), (world, shape, nm, k)
        if nm in ("policy", "q1", "q2"):
            for slot in ("m", "v"):
                a, b = ctxs[0].get_net(nm, slot), ctxs[1].get_net(nm, slot)
                for k in a:
                    assert np.array_equal(a[k], b[k]), (world, shape, nm, slot, k)
    for sid in (L.S_LOG_ALPHA, L.S_ADAM_M_LOG_ALPHA, L.S_ADAM_V_LOG_ALPHA, L.S_ALPHA):
        assert ctxs[0].get_scalar(sid) == ctxs[1].get_scalar(sid), sid
    hist = ctxs[0].fetch_losses(n)
    assert np.array_equal(hist, fused)
    for c in ctxs:
        c.close()


def test_single_updates_drawn_ahead_identical():
    """A device-sampled update launch draws the NEXT launch's first batch ahead (its
    random.sample + gather ride in L12 / L13 into the other batch set, the MT state saved);
    the next launch of the same batch size takes it (single or multi-update), any other call
    but a read restores the MT state.
    Against a context with the draw-ahead off (SACMI_NO_PREFETCH at creation), over a call
    sequence that consumes, drops and re-arms it — sync, async and launch / wait updates,
    a push (mailbox) between updates, a host random.sample, a batch-size change, a query
    of the MT state, select_action of 100 / 7 / 1 states between updates — every loss, every parameter, the MT stream and the indices of the
    host sample must be identical, bit for bit."""
    cfg, B, nrows = SacConfig(24, 4, 64), 64, 500
    params = init_params(cfg, 91, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows + 40, 92, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 40503 % (2**32)).astype(np.uint32)
    res = []
    for ahead in (True, False):
        if not ahead:
            os.environ["SACMI_NO_PREFETCH"] = "1"
        try:
            ctx = make_ctx(cfg, max_batch=B, capacity=nrows + 40)
        finally:
            os.environ.pop("SACMI_NO_PREFETCH", None)
        load_params(ctx, params)
        ctx.push(*[x[:nrows] for x in rows])
        ctx.set_mt(0, key, 624)
        out = []
        for _ in range(3):
            out.append(ctx.step(B))                   # consumed by the next
        ctx.step_async(B); ctx.step_async(B)
        out.append(ctx.fetch_losses(2).ravel())    # (a read: the one drawn ahead stays)
        ctx.step_many_async(B, 3)                  # takes it, draws the next launch's ahead
        ctx.step_many_async(B, 2)
        ctx.step_async(B)
        out.append(ctx.fetch_losses(6).ravel())
        out.append(ctx.step(B))
        ctx.push(*[x[nrows:nrows + 1] for x in rows])   # between updates: dropped
        out.append(ctx.step(B))
        out.append(ctx.step(B))
        out.append(ctx.step(B))
        idx = ctx.sample_indices(B)                 # a host random.sample in between
        ctx.step_many_async(B, 4)
        out.append(ctx.fetch_losses(4).ravel())
        out.append(ctx.step(B))
        out.append(ctx.step(B))
        out.append(ctx.step(B // 2))                # another batch size
        ctx.step_launch(B // 2)
        out.append(ctx.step_wait())
        ctx.step_launch(B // 2)
        out.append(ctx.step_wait())
        mt_mid = ctx.get_mt(0)
        out.append(ctx.step(B))
        out.append(ctx.step(B))
        # select_action between single updates: n > 64 states go through batch set 0's
        # x2 rows (the non-zero-copy path), n <= 64 write their actions there, one state
        # takes the GEMVs (writes no batch set) — a batch drawn ahead must not be clobbered
        st = np.asarray(rows[0][:100], np.float32)
        for n_act in (100, 7, 1, 100):
            out.append(ctx.act(st[:n_act], deterministic=True).ravel())
            out.append(ctx.step(B))
        res.append((out, idx, mt_mid, ctx.get_mt(0), {n: ctx.get_net(n) for n in NETS}))
        ctx.close()
    (o1, i1, m1, e1, p1), (o2, i2, m2, e2, p2) = res
    assert len(o1) == len(o2)
    for a, b in zip(o1, o2):
        assert np.array_equal(a, b)
    assert np.array_equal(i1, i2)
    for m, n in ((m1, m2), (e1, e2)):
        assert np.array_equal(m[0], n[0]) and m[1] == n[1]
    for n in NETS:
        for k in p1[n]:
            assert np.array_equal(p1[n][k], p2[n][k]), (n, k)


@pytest.mark.parametrize("world", [3, 5, 6])
def test_native_dp_loopback_sharded_equals_allreduce_nonpow2(world):
    """Non-power-of-two worlds (the chunk tiling of the sharded form: chunks of 64-float
    multiples that do not divide the ranges, the last one reaching into the gap past the
    critic range / the arena's tail slack): x world then x 1/world is not exact in fp32 there,
    so the update is not the fused one — but the sharded form (reduce-scatter -> Adam on each
    rank's chunk -> all-gather, every rank's chunk run in turn) and the all-reduce form apply
    the same two scalings to every element, and must agree BIT FOR BIT: parameters, Adam
    moments, log_alpha state, losses."""
    from sacmi import _lib as L
    cfg, B, nrows, n = SacConfig(376, 17, 512), 256, 4000, 3
    params = init_params(cfg, 97, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 98, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 1812433 % (2**32)).astype(np.uint32)
    ctxs = []
    for sharded in (True, False):
        ctx = make_ctx(cfg, max_batch=B, capacity=nrows, seed=5)
        load_params(ctx, params)
        ctx.push(*rows)
        ctx.set_mt(0, key, 624)
        ctx.dp_loopback_init(world)
        ctx.dp_set_sharded(sharded)
        assert ctx.dp_sharded() == sharded
        ctx.step_dp(B, n)
        ctx.synchronize()
        ctxs.append(ctx)
    a, b = ctxs
    for nm in NETS:
        for slot in (("param", "m", "v") if nm in ("policy", "q1", "q2") else ("param",)):
            x, y = a.get_net(nm, slot), b.get_net(nm, slot)
            for k in x:
                assert np.array_equal(x[k], y[k]), (world, nm, slot, k)
    for sid in (L.S_LOG_ALPHA, L.S_ADAM_M_LOG_ALPHA, L.S_ADAM_V_LOG_ALPHA, L.S_ALPHA, L.S_STEP_POLICY):
        assert a.get_scalar(sid) == b.get_scalar(sid), sid
    assert np.array_equal(a.fetch_losses(n), b.fetch_losses(n))
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("world", [3, 8])
def test_dp_sharded_one_rank_chunks(world):
    """The sharded step's chunk arithmetic (the range's chunks of 64-float multiples, Adam's
    layer segments clipped to rank 0's chunk): the loopback's one-rank mode steps rank 0's
    chunk of each range only, and each range must have some but not all of its elements
    stepped.
    * Critic range: every element holds its fused-update value (inside the chunk) or its
      value before the update (outside), bit for bit at any world (the one-rank mode's
      collectives return the rank's own gradient, and Adam applies no 1/world).
    * Actor range: its gradient comes from the PARTLY stepped critics (sac_imp.py:116-125
      reads the critics after their step).  Reference: the oracle's actor block
      (OracleSAC.actor_step, sac_imp.py:116-135) in fp64 and fp32 on those same critics (read
      back), the update's own minibatch and noise (sacmi_read_batch); the stepped policy
      elements are graded as every parameter delta is (check_delta_vs_reference)."""
    cfg, B, nrows = SacConfig(376, 17, 512), 256, 4000
    params = init_params(cfg, 131, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 132, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 1812433 % (2**32)).astype(np.uint32)
    res = []
    for one in (True, False):
        if one:
            os.environ["SACMI_DP_LOOPBACK_ONE_RANK"] = "1"
        try:
            ctx = make_ctx(cfg, max_batch=B, capacity=nrows, seed=5)
            load_params(ctx, params)
            ctx.push(*rows)
            ctx.set_mt(0, key, 624)
            if one:
                ctx.dp_loopback_init(world)
                ctx.dp_set_sharded(True)
                ctx.step_dp(B, 1)
            else:
                ctx.step(B)                       # the fused update (the same minibatch and noise)
            ctx.synchronize()
            res.append(({n: ctx.get_net(n) for n in ("policy", "q1", "q2")}, ctx.read_batch(B)))
            ctx.close()
        finally:
            os.environ.pop("SACMI_DP_LOOPBACK_ONE_RANK", None)
    (one, (idx, eps)), (fused, (idx_f, eps_f)) = res
    assert np.array_equal(idx, idx_f) and np.array_equal(eps, eps_f)
    init = {n: {k: np.asarray(params[n][k], np.float32).reshape(v.shape) for k, v in one[n].items()}
            for n in one}
    # the critic range
    n_stepped = total = 0
    for net in ("q1", "q2"):
        for k, v in one[net].items():
            stepped = v != init[net][k]
            n_stepped += int(stepped.sum())
            total += v.size
            if stepped.any():
                assert np.array_equal(v[stepped], fused[net][k][stepped]), (net, k)
    assert 0 < n_stepped < total, ("critics", n_stepped, total)
    # the actor range, against the oracle's actor block on the same partly stepped critics
    shapes = param_shapes(cfg)
    start = {n: ({k: one[n][k].reshape(shapes[n][k]) for k in one[n]} if n in ("q1", "q2") else params[n])
             for n in NETS}
    ref = {}
    for dt in (torch.float32, torch.float64):
        o = OracleSAC(cfg, start, dt)
        o.actor_step(rows[0][idx], eps[B:])
        ref[dt] = {k: t.detach().numpy().reshape(one["policy"][k].shape) for k, t in o.nets["policy"].items()}
    n_stepped = total = 0
    for k, v in one["policy"].items():
        stepped = v != init["policy"][k]
        n_stepped += int(stepped.sum())
        total += v.size
        if not stepped.any():
            continue
        p0 = init["policy"][k][stepped].astype(np.float64)
        check_delta_vs_reference(v[stepped] - p0, ref[torch.float64][k][stepped] - p0,
                                 ref[torch.float32][k][stepped] - p0, ("policy", k, world))
    assert 0 < n_stepped < total, ("policy", n_stepped, total)


def test_dp_sharded_moments_read_guard():
    """After a sharded optimizer step that leaves other ranks' chunks of the Adam moments
    unstepped on this GPU (the loopback's one-rank timing mode steps rank 0's chunk only),
    reading the moments (tensors, the log_alpha moment scalars, hence checkpoints) raises
    instead of returning stale values, and neither leaving the sharded form nor
    sacmi_dp_sync_state lifts that (no collective can repair it); parameters stay readable,
    and the timing context may go on stepping (the bench's other optimizer form).  A loopback
    run that stepped every chunk leaves the moments whole: nothing raises after leaving the
    sharded form."""
    from sacmi import _lib as L
    cfg, B = SacConfig(24, 4, 64), 64
    params = init_params(cfg, 99, bias_scale=0.05)
    rows = synthetic_rows(cfg, 400, 100, state_scale=0.5)
    ctx = make_ctx(cfg, max_batch=B, capacity=400, seed=5)
    load_params(ctx, params)
    ctx.push(*rows)
    ctx.dp_loopback_init(4)
    ctx.dp_set_sharded(True)
    os.environ["SACMI_DP_LOOPBACK_ONE_RANK"] = "1"
    try:
        ctx.step_dp(B, 2)
    finally:
        os.environ.pop("SACMI_DP_LOOPBACK_ONE_RANK", None)
    ctx.synchronize()
    assert all(np.all(np.isfinite(v)) for v in ctx.get_net("q1").values())
    with pytest.raises(RuntimeError, match="one-rank"):
        ctx.get_net("q1", "m")
    with pytest.raises(RuntimeError, match="one-rank"):
        ctx.get_scalar(L.S_ADAM_V_LOG_ALPHA)
    ctx.dp_set_sharded(False)
    ctx.dp_sync_state()
    with pytest.raises(RuntimeError, match="one-rank"):
        ctx.get_net("q1", "m")
    ctx.step_dp(B, 1)                                        # (the all-reduce form: timing)
    ctx.synchronize()
    ctx.close()
    # every chunk stepped (the loopback's default): whole moments, a fused update runs after
    ctx = make_ctx(cfg, max_batch=B, capacity=400, seed=5)
    load_params(ctx, params)
    ctx.push(*rows)
    ctx.dp_loopback_init(4)
    ctx.dp_set_sharded(True)
    ctx.step_dp(B, 2)
    ctx.dp_set_sharded(False)
    assert all(np.all(np.isfinite(v)) for v in ctx.get_net("q1", "m").values())
    ctx.step(B)
    ctx.close()


def test_dp_sharded_entry_order_same_sequence():
    """The sharded form entered at creation (SACMI_DP_SHARD=1, read by sacmi_dp_loopback_init)
    and entered from the all-reduce default through sacmi_dp_set_sharded(1) run the same
    per-update sequence: the same launch sites, kernels and grids in the same order — the
    collective sites included — and the same bits.  (Round 5's bench put the two forms'
    lines 42 % apart by position: its two legs ran under different loopback modes, all chunks
    vs rank 0's chunk; bench.py now sets the one-rank mode for every simulated-world leg.)"""
    cfg, B, world, nrows = SacConfig(376, 17, 512), 256, 8, 4000
    params = init_params(cfg, 141, bias_scale=0.05)
    rows = synthetic_rows(cfg, nrows, 142, state_scale=0.5)
    key = (np.arange(624, dtype=np.uint64) * 1812433 % (2**32)).astype(np.uint32)
    seqs, states = [], []
    os.environ["SACMI_DP_LOOPBACK_ONE_RANK"] = "1"          # the bench's simulated-world mode
    try:
        for entry in ("creation", "switch"):
            if entry == "creation":
                os.environ["SACMI_DP_SHARD"] = "1"
            try:
                ctx = make_ctx(cfg, max_batch=B, capacity=nrows, seed=5)
                load_params(ctx, params)
                ctx.push(*rows)
                ctx.set_mt(0, key, 624)
                ctx.dp_loopback_init(world)
            finally:
                os.environ.pop("SACMI_DP_SHARD", None)
            if entry == "switch":
                assert not ctx.dp_sharded()
                ctx.dp_set_sharded(True)
            assert ctx.dp_sharded()
            ctx.step_dp(B, 2)
            kernels, _ = ctx.profile_timeline(B, 2, data_parallel=True)
            seqs.append([(k["site"], k["site_idx"], k["kernel"], k["grid"]) for k in kernels])
            ctx.synchronize()
            states.append({n: ctx.get_net(n) for n in ("policy", "q1", "q2")})
            ctx.close()
    finally:
        os.environ.pop("SACMI_DP_LOOPBACK_ONE_RANK", None)
    # (site_idx counts every launch site in order, the collective sites included — in the
    # loopback their stand-ins stamp no timeline: they show as the gaps, >= 5 per update:
    # the flags, two reduce-scatters, two gathers / shard Adams)
    assert seqs[0] == seqs[1]
    idx = {i for _, i, _, _ in seqs[0]}
    assert len(set(range(max(idx) + 1)) - idx) >= 5 * 2, sorted(idx)
    for n in states[0]:
        for k in states[0][n]:
            assert np.array_equal(states[0][n][k], states[1][n][k]), (n, k)


MASKED_GRAD_TOL = 1e-5   # normwise per tensor, vs fp64 evaluated under the GPU's ReLU masks


def flip_evidence(cfg, params, batch, e1, e2, masks):
    """fp64 under the GPU's own ReLU masks: (its gradients, {(pass, layer): flipped decisions},
    the largest |fp64 pre-activation| of a flipped decision relative to its layer's largest
    |pre-activation|).  The pre-activations are the fp64 ones downstream of the GPU's
    decisions, so a flip that only fp32 rounding explains sits near 0 on this scale."""
    om = OracleSAC(cfg, params, torch.float64)
    flips, zrel = {}, [0.0]
    import oracle.sac_step as osm
    orig = osm._relu
    def spy(x, tag, i):
        if tag and (tag, i) in masks:
            z = x.detach().numpy()
            f = (z > 0) != (masks[(tag, i)] > 0)
            flips[(tag, i)] = int(f.sum())
            if f.any():
                zrel[0] = max(zrel[0], float(np.abs(z[f]).max() / max(np.abs(z).max(), 1e-30)))
        return orig(x, tag, i)
    osm._relu = spy
    try:
        om.step(*batch, e1, e2, masks=masks)
    finally:
        osm._relu = orig
    print("ReLU decisions the GPU took differently from fp64:", {f"{t}.{i}": n for (t, i), n in flips.items() if n},
          f"largest |z| of a flip / layer max: {zrel[0]:.2e}")
    return om.grads_flat(), flips, zrel[0]


def gpu_relu_masks(ctx, cfg, B):
    """{(tag, layer): 0/1 mask} of every ReLU of the last update, from the activations it left
    in HBM (sacmi_read_activation; OracleSAC.step(masks=...) tags)."""
    masks = {}
    for layer in range(cfg.n_hidden):
        for p, tags in ((0, ("q1", "q2")), (1, ("q1t", "q2t")), (2, ("q1a", "q2a"))):
            h = ctx.read_activation(p, layer, B)
            for i, t in enumerate(tags):
                masks[(t, layer)] = (h[i] > 0).astype(np.float32)
        h = ctx.read_activation(3, layer, B)
        masks[("pi_s2", layer)] = (h[:B] > 0).astype(np.float32)
        masks[("pi_s", layer)] = (h[B:] > 0).astype(np.float32)
    return masks


@pytest.mark.parametrize("n_hidden,B", [(2, 4096), (3, 4096), (2, 3000)])
def test_step_humanoid_b4096_under_gpu_masks(n_hidden, B):
    """Batch 4096 (BASELINE configs[2] shapes) at the 1e-5 gradient bar — and batch 3000, whose
    row counts are no multiple of the x6 kernels' 128-row tiles (k_fwd_x6's clamped rows, the
    split-K ranges of k_dw_part_x6; the dh levels fall back to k_gemm): the fp64 truth is
    recomputed under the GPU's OWN ReLU masks (read back from the activations the update left
    in HBM).  Where test_step_humanoid_b4096_vs_oracle needs its ReLU-flip allowances
    (q1.fc1.weight 2.9e-4 against plain fp64), the flips are the whole story if every gradient
    tensor sits within 1e-5 of this masked truth; the number of flipped decisions per pass is
    printed with the per-tensor table."""
    cfg = SacConfig(376, 17, 512, n_hidden=n_hidden)
    params = init_params(cfg, 101, bias_scale=0.02)
    rows = synthetic_rows(cfg, 6000, 102, state_scale=0.1)
    ctx = make_ctx(cfg, max_batch=B, capacity=len(rows[2]))
    load_params(ctx, params)
    ctx.push(*rows)
    rng = np.random.default_rng(103)
    idx = rng.choice(len(rows[2]), B, replace=False)
    e1 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
    e2 = rng.standard_normal((B, cfg.action_dim)).astype(np.float32)
    lg = ctx.step(B, idx=idx, eps1=e1, eps2=e2)
    gg = ctx_grads(ctx, cfg)
    masks = gpu_relu_masks(ctx, cfg, B)
    batch = [x[idx] for x in rows]
    om = OracleSAC(cfg, params, torch.float64)
    lm = om.step(*batch, e1, e2, masks=masks)
    o64 = OracleSAC(cfg, params, torch.float64)
    o64.step(*batch, e1, e2)
    g64 = o64.grads_flat()
    # the decisions the GPU took differently from plain fp64, per pass and layer, and how far
    # from zero their fp64 pre-activations sit
    gm, _, zmax = flip_evidence(cfg, params, batch, e1, e2, masks)
    assert zmax <= FLIP_Z_TOL, ("a flipped ReLU decision away from zero", zmax)
    for i, k in enumerate(("q1_loss", "q2_loss", "policy_loss")):
        assert abs(lg[i] - lm[k]) <= LOSS_TOL * max(abs(lm[k]), 1e-3), (k, lg[i], lm[k])
    table = {k: (rel(gg[k], v), rel(gg[k], g64[k])) for k, v in gm.items()}
    report_grad_errors(f"humanoid B{B} n_hidden {n_hidden} under the GPU's ReLU masks", MASKED_GRAD_TOL, table,
                       second="gpu_vs_plain_fp64", strict=True)
    bad = {k: e for k, (e, _) in table.items() if e > MASKED_GRAD_TOL}
    assert not bad, bad
    ctx.close()
