"""Rebuild full-shape checkpoints from tests/golden/ckpt_reference.npz (the reference's own
best_model.pt files, tools/make_ckpt_fixture.py): every tensor has the reference's key,
shape and file order; the strided sample positions hold the reference's values, the other
elements a seeded fill (the fixture keeps samples + checksums, not whole tensors)."""
import json
import os

import numpy as np
import torch

NETS = ("policy", "q1", "q2", "q1_target", "q2_target")
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt_reference.npz")


def load_fixture():
    z = np.load(FIXTURE)
    return z, json.loads(str(z["keys"]))


def rebuild(tag: str, seed: int = 0) -> dict:
    """The checkpoint dict of `tag` ("humanoid" | "bipedal") in the reference's format
    (sac_imp.py:154-163: five state dicts + alpha)."""
    z, keys = load_fixture()
    rng = np.random.default_rng(seed)
    ck = {}
    for n in NETS:
        sd = {}
        for k in keys[tag]["nets"][n]:
            p = f"{tag}.{n}.{k}"
            shape = tuple(int(x) for x in z[p + ".shape"])
            flat = (rng.standard_normal(int(np.prod(shape))) * 0.05).astype(np.float32)
            flat[z[p + ".idx"]] = z[p + ".val"]
            sd[k] = torch.from_numpy(flat.reshape(shape))
        ck[f"{n}_state_dict"] = sd
    al = torch.from_numpy(z[f"{tag}.alpha"].copy())
    ck["alpha"] = al.requires_grad_(True) if int(z[f"{tag}.alpha_is_tensor"]) else float(al[0])
    assert list(ck) == keys[tag]["top"]
    return ck
