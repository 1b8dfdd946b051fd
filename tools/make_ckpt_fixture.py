#!/usr/bin/env python3
"""Fixture of the reference's OWN checkpoints, for tests/golden/.

Reads the two `best_model.pt` files the reference ships (written by its
``SAC.save``, sac_imp.py:154-163) with ``torch.load(weights_only=True)`` only — nothing in
them is executed — and writes, per checkpoint:

  keys            the top-level keys and, per state dict, its keys in file order
  <ck>.<net>.<key>.shape    the tensor's shape
  <ck>.<net>.<key>.idx      a strided sample of flat element positions (every STRIDE-th,
                            plus the last element)
  <ck>.<net>.<key>.val      the reference's values at those positions (float32, bit copies)
  <ck>.<net>.<key>.sum      float64 sum and sum of squares of the whole tensor (checksum)
  <ck>.alpha                the saved alpha ([1] float32 tensor with requires_grad)

The GPU test (tests/test_gpu_dropin.py) rebuilds a full-shape dict from this (sampled
positions hold the reference's values, the rest a seeded fill), saves it with torch.save,
loads it through the drop-in ``SAC.load`` and checks every device tensor bit for bit.

Runs only in the build container (needs /root/reference).
Usage:  python tools/make_ckpt_fixture.py [--out tests/golden/ckpt_reference.npz]
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np
import torch

REF = "/root/reference/results"
CKPTS = {
    "humanoid": ("sac_Humanoid-v5_1734629000/best_model.pt", dict(S=376, A=17, H=256)),
    "bipedal": ("sac_BipedalWalker-v3_1737453113/best_model.pt", dict(S=24, A=4, H=256)),
}
NETS = ("policy", "q1", "q2", "q1_target", "q2_target")
STRIDE = 97


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tests", "golden", "ckpt_reference.npz"))
    args = ap.parse_args()
    out = {}
    keys = {}
    for tag, (rel, dims) in CKPTS.items():
        ck = torch.load(os.path.join(REF, rel), weights_only=True, map_location="cpu")
        keys[tag] = {"top": list(ck.keys()), "dims": dims,
                     "nets": {n: list(ck[f"{n}_state_dict"].keys()) for n in NETS}}
        for n in NETS:
            for k, t in ck[f"{n}_state_dict"].items():
                a = t.detach().cpu().numpy().astype(np.float32, copy=False)
                flat = a.reshape(-1)
                idx = np.unique(np.concatenate([np.arange(0, flat.size, STRIDE), [flat.size - 1]]))
                p = f"{tag}.{n}.{k}"
                out[p + ".shape"] = np.array(a.shape, np.int64)
                out[p + ".idx"] = idx.astype(np.int64)
                out[p + ".val"] = flat[idx].copy()
                f64 = flat.astype(np.float64)
                out[p + ".sum"] = np.array([f64.sum(), (f64 * f64).sum()])
        al = ck["alpha"]
        out[f"{tag}.alpha"] = np.asarray(al.detach().cpu().numpy() if torch.is_tensor(al) else al,
                                         np.float32).reshape(-1)
        out[f"{tag}.alpha_is_tensor"] = np.array(int(torch.is_tensor(al)))
    out["keys"] = np.array(json.dumps(keys))
    np.savez_compressed(args.out, **out)
    print("wrote", args.out, os.path.getsize(args.out), "bytes")


if __name__ == "__main__":
    main()
