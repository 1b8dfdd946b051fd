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
