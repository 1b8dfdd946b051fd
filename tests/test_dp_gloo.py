"""World-size-2 data-parallel update on CPU (gloo): the production DataParallelUpdate
driver over the oracle backend must equal one single-process update on the
concatenated batch, and both replicas must stay identical."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from oracle.sac_step import NETS, OracleSAC, SacConfig, init_params, synthetic_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_equals_global_batch(tmp_path):
    import dp_oracle
    cfg = SacConfig(6, 2, 16)
    params = init_params(cfg, 5, bias_scale=0.05)
    world, B, steps = 2, 8, 3
    shards = [synthetic_rows(cfg, 40, 100 + r, state_scale=0.5) for r in range(world)]
    rng = np.random.default_rng(9)
    idx = [[rng.choice(40, B, replace=False) for _ in range(world)] for _ in range(steps)]
    eps1 = [[rng.standard_normal((B, 2)).astype(np.float32) for _ in range(world)] for _ in range(steps)]
    eps2 = [[rng.standard_normal((B, 2)).astype(np.float32) for _ in range(world)] for _ in range(steps)]
    mp.start_processes(dp_oracle.worker,
                       args=(world, _free_port(), cfg, params, shards, idx, eps1, eps2,
                             str(tmp_path), steps),
                       nprocs=world, join=True, start_method="spawn")
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    # replicas bitwise identical
    for k in r0.files:
        assert np.array_equal(r0[k], r1[k]), k
    # == one update on the concatenated global batch
    ref = OracleSAC(cfg, params, dtype=torch.float64)
    for t in range(steps):
        batch = [np.concatenate([shards[r][j][idx[t][r]] for r in range(world)]) for j in range(5)]
        ref.step(*batch, np.concatenate(eps1[t]), np.concatenate(eps2[t]))
    st = ref.state()
    for n in NETS:
        for k in init_params(cfg, 5)[n]:
            key = f"{n}.{k}"
            np.testing.assert_allclose(r0[key], st[key], rtol=1e-9, atol=1e-12, err_msg=key)
    np.testing.assert_allclose(r0["log_alpha"], st["log_alpha"], rtol=1e-9, atol=1e-12)


def test_dp_two_ranks_per_shards_equals_global_batch(tmp_path):
    """BASELINE configs[3] on CPU: two ranks, each with its OWN prioritized replay shard
    (non-uniform priorities, its own numpy MT stream and frame counter) — the production
    DataParallelUpdate driver over gloo equals one update on the concatenation of the two
    shards' prioritized draws, and the replicas stay identical."""
    import dp_oracle
    cfg = SacConfig(6, 2, 16)
    params = init_params(cfg, 15, bias_scale=0.05)
    world, B, steps, n = 2, 8, 3, 50
    shards = [synthetic_rows(cfg, n, 200 + r, state_scale=0.5) for r in range(world)]
    rng = np.random.default_rng(19)
    prios = [rng.uniform(0.05, 3.0, n).astype(np.float32) for _ in range(world)]
    keys = [rng.integers(0, 2**32, 624, dtype=np.uint32) for _ in range(world)]
    eps1 = [[rng.standard_normal((B, 2)).astype(np.float32) for _ in range(world)] for _ in range(steps)]
    eps2 = [[rng.standard_normal((B, 2)).astype(np.float32) for _ in range(world)] for _ in range(steps)]
    mp.start_processes(dp_oracle.worker_per,
                       args=(world, _free_port(), cfg, params, shards, prios, keys, eps1, eps2,
                             str(tmp_path), steps, B),
                       nprocs=world, join=True, start_method="spawn")
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    for k in r0.files:
        if not k.startswith("idx"):
            assert np.array_equal(r0[k], r1[k]), k
    # each rank drew from its own shard's prioritized distribution
    draws = [dp_oracle.per_shard_indices(prios[r], n, B, keys[r], steps) for r in range(world)]
    for t in range(steps):
        assert np.array_equal(r0[f"idx{t}"], draws[0][t][0])
        assert np.array_equal(r1[f"idx{t}"], draws[1][t][0])
    assert not all(np.array_equal(draws[0][t][0], draws[1][t][0]) for t in range(steps))
    ref = OracleSAC(cfg, params, dtype=torch.float64)
    for t in range(steps):
        batch = [np.concatenate([shards[r][j][draws[r][t][0]] for r in range(world)]) for j in range(5)]
        ref.step(*batch, np.concatenate(eps1[t]), np.concatenate(eps2[t]))
    st = ref.state()
    for nn_ in NETS:
        for k in init_params(cfg, 15)[nn_]:
            key = f"{nn_}.{k}"
            np.testing.assert_allclose(r0[key], st[key], rtol=1e-9, atol=1e-12, err_msg=key)
    np.testing.assert_allclose(r0["log_alpha"], st["log_alpha"], rtol=1e-9, atol=1e-12)
