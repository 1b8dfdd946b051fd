"""Host-side check of the x6 kernels' LDS layout (no GPU): the XOR chunk swizzle of
k_fwd_x6's planes and k_axk_x6's A planes, read from kernels.hip, is a permutation of each
64-byte row's 16-byte chunks, and it is bank-conflict-free for the two access patterns the
kernels issue — the ds_read_b128 fragment reads (row = lane & 15 of a 16-row block, chunk =
lane >> 4) in the lane groups of MI355X_MICROARCH.md §LDS, and the staging ds_write_b64
stores (8 threads a row, 4 bf16 each) in 16-lane contiguous groups.  The layout is the one
profiles/r06/x6_swizzle_ab measured; the GPU parity tests check the values through it."""
import pathlib
import re

KERNELS = pathlib.Path(__file__).resolve().parents[1] / "humanoid-walking-with-sac_amd" / "csrc" / "kernels.hip"
ROW_BYTES = 64                      # 32 bf16 per row, no pad

# ds_read_b128: four 16-lane groups, one LDS cycle each when conflict-free (64 banks x 4 B)
B128_GROUPS = [
    [*range(0, 4), *range(12, 16), *range(20, 28)],
    [*range(4, 12), *range(16, 20), *range(28, 32)],
    [*range(32, 36), *range(44, 48), *range(52, 60)],
    [*range(36, 44), *range(48, 52), *range(60, 64)],
]


def swizzle_fns():
    src = KERNELS.read_text()
    exprs = re.findall(r"auto cw = \[\]\(int r, int k\) \{ return (.+?); \};", src)
    assert len(exprs) == 2, "k_fwd_x6 and k_axk_x6 each define the chunk swizzle"
    assert exprs[0] == exprs[1], "one layout for both kernels"
    expr = exprs[0]
    assert re.fullmatch(r"[\s\d()<>&^|rk+\-*]+", expr), expr     # plain integer arithmetic
    return expr, eval(f"lambda r, k: {expr}")


def test_swizzle_permutes_each_rows_chunks():
    _, cw = swizzle_fns()
    for r in range(256):
        cols = sorted(cw(r, k) for k in range(32))
        assert cols == list(range(32)), r
        for k in range(0, 32, 8):           # a 16-byte chunk stays whole and aligned
            assert [cw(r, k + i) for i in range(8)] == [cw(r, k) + i for i in range(8)]


def test_fragment_reads_conflict_free():
    _, cw = swizzle_fns()
    for base in range(0, 128, 16):          # every 16-row block a wave reads
        for grp in B128_GROUPS:
            slots = set()
            for lane in grp:
                r, chunk = base + (lane & 15), lane >> 4
                addr = r * ROW_BYTES + cw(r, 8 * chunk) * 2
                slots.add((addr // 16) % 16)     # 4-bank slot of the 256-byte bank row
            assert len(slots) == 16, (base, grp)


def test_staging_stores_conflict_free():
    _, cw = swizzle_fns()
    tpr = 8                                  # threads per row, 4 k (8 bytes) each
    for tid0 in range(0, 512, 16):           # 16-lane contiguous groups of ds_write_b64
        banks = []
        for tid in range(tid0, tid0 + 16):
            r, kq = tid // tpr, 4 * (tid % tpr)
            addr = r * ROW_BYTES + cw(r, kq) * 2
            banks += [(addr // 4) % 32, (addr // 4 + 1) % 32]
        assert sorted(banks) == list(range(32)), tid0


def test_unswizzled_rows_would_conflict():
    """The control: plain 64-byte rows put two lanes of every read group on one slot."""
    def worst(cw):
        w = 0
        for grp in B128_GROUPS:
            slots = {}
            for lane in grp:
                r, chunk = lane & 15, lane >> 4
                s = ((r * ROW_BYTES + cw(r, 8 * chunk) * 2) // 16) % 16
                slots[s] = slots.get(s, 0) + 1
            w = max(w, max(slots.values()))
        return w
    assert worst(lambda r, k: k) == 2
    assert worst(swizzle_fns()[1]) == 1
