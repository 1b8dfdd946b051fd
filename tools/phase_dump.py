#!/usr/bin/env python3
"""Per-phase medians of the GEMM levels from a diagnostic timeline dump (SACMI_DIAG_DUMP,
a -DSACMI_DIAG_PHASES build).  k_gemm phases (wave 0 of the first 256 workgroups):
0 entry, 1 setup done (before the K loop), 2 wave 0's K loop + MFMAs done, 3 every wave
done (the pre-epilogue barrier; incl. the row prologue), 4 epilogue stores issued, 5 exit;
6 / 7 the last wave's entry and K-loop end (lastin: its entry after wave 0's); 8 / 9 the
desc landed / the tile placed.
usage: tools/phase_dump.py dump.bin"""
import struct
import sys

import numpy as np


SLOW = 0


def main(path):
    raw = open(path, "rb").read()
    sites, per, words, nph = struct.unpack("4q", raw[:32])
    names = [raw[32 + 32 * i:64 + 32 * i].split(b"\0")[0].decode() for i in range(sites)]
    w = np.frombuffer(raw[32 + 32 * sites:], np.uint64).reshape(sites, per, words)
    t0 = min(int(w[s, k, 0]) for s in range(sites) for k in range(per) if w[s, k, 0] != 2**64 - 1)
    acc = {}
    for s in range(sites):
        k = 0
        x = w[s, k]
        if x[0] == 2**64 - 1 or int(x[2]) != 1:      # k_gemm only (TL_GEMM)
            continue
        p0 = words - 256 * nph                        # phase words follow the end slots
        ph = x[p0:p0 + 256 * nph].reshape(256, nph).astype(np.int64)
        live = ph[:, 0] > 0
        ph = ph[live]
        if len(ph) == 0:
            continue
        start = int(x[0])
        d = {
            "start": np.median(ph[:, 0] - start) * 0.01,
            "startmax": np.max(ph[:, 0] - start) * 0.01,
            "setup": np.median(ph[:, 1] - ph[:, 0]) * 0.01,
            "core0": np.median(ph[:, 2] - ph[:, 1]) * 0.01,
            "wait": np.median(ph[:, 3] - ph[:, 2]) * 0.01,
            "epi": np.median(ph[:, 4] - ph[:, 3]) * 0.01,
            "tail": np.median(ph[:, 5] - ph[:, 4]) * 0.01,
            "wg": np.median(ph[:, 5] - ph[:, 0]) * 0.01,
            "wgmax": np.max(ph[:, 5] - ph[:, 0]) * 0.01,
        }
        if nph >= 8 and np.all(ph[:, 6] > 0):   # the last wave's entry / K-loop end
            d["lastin"] = np.median(ph[:, 6] - ph[:, 0]) * 0.01
            d["lastcore"] = np.median(ph[:, 7] - ph[:, 6]) * 0.01
        if nph >= 10 and np.all(ph[:, 8] > 0) and np.all(ph[:, 8] >= ph[:, 1]):
            # staged core: first / last slab barrier
            d["slab0"] = np.median(ph[:, 8] - ph[:, 1]) * 0.01
            d["slabs"] = np.median(ph[:, 9] - ph[:, 8]) * 0.01
            d["lastmma"] = np.median(ph[:, 2] - ph[:, 9]) * 0.01
        elif nph >= 10 and np.all(ph[:, 8] > 0):
            # register-direct core: the setup split — desc round trip, tile placement, the rest
            d["desc"] = np.median(ph[:, 8] - ph[:, 0]) * 0.01
            d["place"] = np.median(ph[:, 9] - ph[:, 8]) * 0.01
            d["pre"] = np.median(ph[:, 1] - ph[:, 9]) * 0.01
        acc.setdefault(names[s], []).append(d)
        if SLOW:   # the slowest workgroups of this site's first launch, phase by phase
            bids = np.nonzero(live)[0]
            tot = ph[:, 5] - ph[:, 0]
            for r in np.argsort(tot)[::-1][:SLOW]:
                seg = np.diff(ph[r]) * 0.01
                print(f"  slow {names[s]:28s} wg {bids[r]:4d} start {(ph[r, 0] - start) * 0.01:6.2f} "
                      f"total {tot[r] * 0.01:6.2f} phases " + " ".join(f"{v:5.2f}" for v in seg))
    keys = ["start", "startmax", "setup", "core0", "wait", "epi", "tail", "wg", "wgmax", "lastin", "lastcore",
            "slab0", "slabs", "lastmma", "desc", "place", "pre"]
    print(f"{'site':32s} " + " ".join(f"{k:>8s}" for k in keys))
    for n, lst in acc.items():
        print(f"{n:32s} " + " ".join(f"{np.median([d.get(k, np.nan) for d in lst]):8.2f}" for k in keys))


if __name__ == "__main__":
    if len(sys.argv) > 2:
        SLOW = int(sys.argv[2])
    main(sys.argv[1])
