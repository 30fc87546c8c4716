"""The rollout's chunk pass sums each head per lane as a pairwise tree (pairs, quads, octets,
16-unit rows, then (S2 + S3) + (S0 + S1); xagents_amd/csrc/mlp_rollout.hip chunk_heads) and
claims that this is bitwise the value xa_wave_sum's DPP butterfly leaves in lane 63
(xa_common.hpp: quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror, then
row_bcast:15 into rows 1 / 3 and row_bcast:31 into rows 2 / 3). This host test emulates both
in float32, lane by lane, on random and adversarial inputs."""
import numpy as np


def _butterfly_lane63(v):
    """xa_wave_sum on 64 f32 lanes; returns lane 63 (the value read back)."""
    v = v.astype(np.float32).copy()
    lanes = np.arange(64)

    def dpp(x, src):  # every lane reads lane src[l] (all lanes active)
        return x[src]

    v = v + dpp(v, lanes ^ 1)  # quad_perm [1,0,3,2]
    v = v + dpp(v, lanes ^ 2)  # quad_perm [2,3,0,1]
    row, pos = lanes // 16, lanes % 16
    v = v + dpp(v, row * 16 + (pos // 8) * 8 + (7 - pos % 8))  # row_half_mirror
    v = v + dpp(v, row * 16 + (15 - pos))  # row_mirror
    # row_bcast:15 (lane 15 of the previous row) into rows 1 and 3; other rows add 0
    b = np.zeros(64, np.float32)
    for r in (1, 3):
        b[r * 16:(r + 1) * 16] = v[(r - 1) * 16 + 15]
    v = v + b
    # row_bcast:31 (lane 31) into rows 2 and 3
    b = np.zeros(64, np.float32)
    b[32:64] = v[31]
    v = v + b
    return v[63]


def _pairwise_tree(p):
    """chunk_heads' per-lane sum of the 64 products p (float32)."""
    p = p.astype(np.float32)
    f = np.float32
    s = []
    for r in range(4):
        o = []
        for oc in range(2):
            q = []
            for qd in range(2):
                j0 = 16 * r + 8 * oc + 4 * qd
                q.append(f(f(p[j0] + p[j0 + 1]) + f(p[j0 + 2] + p[j0 + 3])))
            o.append(f(q[0] + q[1]))
        s.append(f(o[0] + o[1]))
    return f(f(s[2] + s[3]) + f(s[0] + s[1]))


def test_chunk_heads_tree_equals_wave_butterfly():
    rng = np.random.default_rng(7)
    cases = [rng.standard_normal(64).astype(np.float32) for _ in range(2000)]
    # wide dynamic range and cancellation: where a different association would differ
    cases += [(rng.standard_normal(64) * 10.0 ** rng.integers(-8, 8, 64)).astype(np.float32)
              for _ in range(2000)]
    h2 = np.tanh(rng.standard_normal((500, 64))).astype(np.float32)
    w = (rng.standard_normal((500, 64)) * 0.1).astype(np.float32)
    cases += [(a * b).astype(np.float32) for a, b in zip(h2, w)]  # the rollout's h2 * w3 products
    differs_from_sequential = 0
    for p in cases:
        tree, fly = _pairwise_tree(p), _butterfly_lane63(p)
        assert tree.tobytes() == fly.tobytes(), (tree, fly)
        seq = np.float32(0)
        for x in p:
            seq = np.float32(seq + x)
        differs_from_sequential += seq.tobytes() != tree.tobytes()
    # the check has teeth: a plain left-to-right sum differs on many of these inputs
    assert differs_from_sequential > 100
