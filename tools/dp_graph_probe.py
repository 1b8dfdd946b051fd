#!/usr/bin/env python3
"""Can a data-parallel update (library phases + RCCL all_reduce) be captured into one
torch.cuda.CUDAGraph?  World-1 probe: captured updates must equal eager ones bit for bit.
Run under torch.distributed.run --nproc-per-node 1."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-walking-with-sac_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench as B  # noqa: E402
from sacmi import Config, Context  # noqa: E402
from sacmi.dp import DataParallelUpdate, GpuBackend  # noqa: E402


def make(device, fill=50_000):
    ctx = Context(Config(B.S_DIM, B.A_DIM, B.HIDDEN, max_batch=256, capacity=fill, seed=3), 0)
    B.init_agent(ctx, 0)
    ctx.push(*B.synth(fill, 11))
    ctx.set_mt(0, np.arange(624, dtype=np.uint32) * 7 + 1, 624)
    return ctx


def main():
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    n = int(os.environ.get("PROBE_N", "10"))
    # eager reference
    ce = make(device)
    ue = DataParallelUpdate(GpuBackend(ce, device))
    for _ in range(2 * n):
        ue(256)
    ue.flush()
    torch.cuda.synchronize()
    # captured
    cg = make(device)
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        be = GpuBackend(cg, device)
    cg.set_stream(s.cuda_stream)
    ug = DataParallelUpdate(be)
    with torch.cuda.stream(s):
        ug(256)                      # warm: builds nothing inside capture
        ug.flush()
    torch.cuda.synchronize()
    # redo from scratch so both runs see identical state
    cg2 = make(device)
    with torch.cuda.stream(s):
        be2 = GpuBackend(cg2, device)
    cg2.set_stream(s.cuda_stream)
    ug2 = DataParallelUpdate(be2)
    g = torch.cuda.CUDAGraph()
    t0 = time.perf_counter()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            ug2(256)
        ug2.flush()
    print("captured", n, "updates in", round(time.perf_counter() - t0, 3), "s", flush=True)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    same = True
    for net in ("policy", "q1", "q2", "q1_target", "q2_target"):
        a, b = ce.get_net(net), cg2.get_net(net)
        for k in a:
            if not np.array_equal(a[k], b[k]):
                same = False
                print("DIFF", net, k, float(np.abs(a[k] - b[k]).max()))
    print("bitwise_equal", same, flush=True)
    # timing: replay vs eager
    reps = 20
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / (reps * n)
    t0 = time.perf_counter()
    for _ in range(reps * n):
        ue(256)
    ue.flush()
    torch.cuda.synchronize()
    te = (time.perf_counter() - t0) / (reps * n)
    print(f"graph {1e6 * tg:.1f} us/update  eager {1e6 * te:.1f} us/update", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
