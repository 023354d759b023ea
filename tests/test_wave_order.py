"""The GPU's wave reductions (elp_kernels.hip wave_tree / wave_max_f64 /
wave_min_f64) run DPP steps inside 16-lane rows -- quad_perm xor 1, quad_perm
xor 2, row_half_mirror, row_mirror -- then ds_swizzle xor 16 and the halves by
readlane.  The mirrors are not xor patterns; DESIGN.md §4 argues that after a
full quad reduction every lane of a group holds the same value, so lane 0 ends
with the pairwise tree over offsets 1, 2, 4, ..., 32 that the oracle's
wave_dot / art_sum compute.  This checks the claim bit for bit on random data
(Python floats are IEEE doubles, each + rounds once, as on the device)."""
import random

import numpy as np


def dpp_ladder(v):
    v = list(v)
    steps = [lambda l: l ^ 1, lambda l: l ^ 2,
             lambda l: (l & ~7) | (7 - (l & 7)),     # row_half_mirror
             lambda l: (l & ~15) | (15 - (l & 15)),  # row_mirror
             lambda l: l ^ 16]                        # ds_swizzle xor 16 (inside each 32)
    for src in steps:
        v = [v[l] + v[src(l)] for l in range(64)]
    return v[0] + v[32], v


def ascending_tree(v):
    lane = list(v)
    off = 1
    while off < 64:
        for l in range(0, 64 - off, 2 * off):
            lane[l] = lane[l] + lane[l + off]
        off *= 2
    return lane[0]


def test_dpp_ladder_equals_oracle_tree_bitwise():
    rng = random.Random(7)
    for trial in range(300):
        scale = 10.0 ** rng.uniform(-8, 8)
        v = [rng.uniform(-1, 1) * scale * (10.0 ** rng.uniform(-6, 6)) for _ in range(64)]
        got, lanes = dpp_ladder(v)
        assert got == ascending_tree(v), trial
        # each 32-lane half is uniform after the swizzle step (the readlane of lane 0 / 32 is safe)
        assert len(set(lanes[:32])) == 1 and len(set(lanes[32:])) == 1


def test_dpp_ladder_max_min_match_numpy():
    rng = np.random.default_rng(3)
    for _ in range(100):
        v = rng.standard_normal(64) * 10.0 ** rng.uniform(-5, 5)
        mx = list(v)
        mn = list(v)
        for src in [lambda l: l ^ 1, lambda l: l ^ 2, lambda l: (l & ~7) | (7 - (l & 7)),
                    lambda l: (l & ~15) | (15 - (l & 15)), lambda l: l ^ 16]:
            mx = [max(mx[l], mx[src(l)]) for l in range(64)]
            mn = [min(mn[l], mn[src(l)]) for l in range(64)]
        assert max(mx[0], mx[32]) == v.max() and min(mn[0], mn[32]) == v.min()
