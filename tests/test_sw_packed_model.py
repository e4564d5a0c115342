"""CPU model of the packed-half Smith-Waterman tile body (hclib_amd/csrc/sw.hip
sw_pk_tile / sw_pk_scores), lane for lane, in numpy float16.

What it pins down without a GPU: the two claims the packed body's exactness
rests on (DESIGN.md §3 `k_sw_dag_pk`):
  * tile-relative values v = G - G(corner), G = H + row + col, stay integers
    in [-2, 2048] for tiles up to 256 x 512 cells, so f16 max / add are exact;
  * no masks are needed: columns outside the tile carry a null code (score 0)
    and the top row reads 0 past the tile, so every row keeps its left value
    before the tile and its right-column value after it.
The model runs the kernel's schedule (lane L: rows 2L, 2L+1 in the low
halves and 128+2L, 129+2L in the high halves, the high band 64 steps
behind, one wave rotation for the cell above, lane 0's top-row / row-127
fix-up, steps padded to whole 64-step chunks) on tiles cut out of a full
reference DP (smith_waterman.cpp:174-229, the global-alignment recurrence of
SURVEY §8a S1), and compares the bottom row, right column and corner with the
DP's, bit for bit."""
import numpy as np
import pytest

# alignment_score_matrix (smith_waterman.cpp:36-43) for codes 0..3 = A C G T
M = np.array([[2, -4, -2, -4], [-4, 2, -4, -2], [-2, -4, 2, -4], [-4, -2, -4, 2]], dtype=np.int64)


def full_dp(s1, s2):
    """H for the whole matrix with the reference's boundary H(0,c) = -c,
    H(r,0) = -r, computed row by row on G = H + r + c (a running max)."""
    n1, n2 = len(s1), len(s2)
    G = np.zeros((n2 + 1, n1 + 1), dtype=np.int64)  # boundary G = 0
    for r in range(1, n2 + 1):
        a = np.maximum(G[r - 1, :-1] + M[s2[r - 1], s1] + 2, G[r - 1, 1:])
        a = np.concatenate(([G[r, 0]], a))
        G[r] = np.maximum.accumulate(a)
    rr = np.arange(n2 + 1)[:, None]
    cc = np.arange(n1 + 1)[None, :]
    return G - rr - cc


def packed_tile(top_h, left_h, corner_h, s1c, s2c):
    """The packed body on one 256-row tile: top_h = H of the row above the tile
    (ncols values), left_h = H of the column left of it (256), corner_h =
    H(R0, C0); s1c / s2c = the tile's codes (0..3). Returns (bottom row H,
    right column H, max |v| seen). Local coordinates: the corner is (0, 0)."""
    f16 = np.float16
    ncols = len(top_h)
    assert len(left_h) == 256 and len(s2c) == 256 and ncols <= 512
    lane = np.arange(64)
    base = corner_h  # G(corner) with local coordinates
    top_v = np.zeros(ncols + 256, dtype=np.int64)
    top_v[:ncols] = top_h + 0 + np.arange(1, ncols + 1) - base
    rows = [1 + 2 * lane, 2 + 2 * lane, 129 + 2 * lane, 130 + 2 * lane]  # lo q0, lo q1, hi q0, hi q1
    lv = [left_h[r - 1] + r - base for r in rows]
    lr0 = np.stack([lv[0], lv[2]], axis=1).astype(f16)  # [:, 0] low half, [:, 1] high half
    lr1 = np.stack([lv[1], lv[3]], axis=1).astype(f16)
    s2q = [s2c[r - 1] for r in rows]

    def up_of(lr1_, topv):
        rot = np.roll(lr1_, 1, axis=0)  # wave_ror:1 — lane L gets lane L-1, lane 0 gets lane 63
        up = rot.copy()
        up[0, 1] = rot[0, 0]            # lane 0 high: lane 63's low row 127
        up[0, 0] = f16(topv)            # lane 0 low: the top row
        return up

    def scores(x, q):
        ok = (x >= 0) & (x < ncols)
        sc = np.where(ok, M[s2q[q], s1c[np.clip(x, 0, ncols - 1)]] + 2, 0)  # null code: 0
        return sc

    upp = up_of(lr1, 0)  # step -1: lane 0's top input is the corner (v = 0)
    nsteps = ncols + 127
    padded = (nsteps + 63) // 64 * 64
    bottom = np.zeros(ncols, dtype=np.int64)
    vmax = 0
    for s in range(padded):
        up = up_of(lr1, top_v[s])
        xlo, xhi = s - lane, s - 64 - lane
        sc0 = np.stack([scores(xlo, 0), scores(xhi, 2)], axis=1).astype(f16)
        sc1 = np.stack([scores(xlo, 1), scores(xhi, 3)], axis=1).astype(f16)
        h0 = np.maximum(np.maximum(lr0, up), (upp + sc0).astype(f16))
        h1 = np.maximum(np.maximum(lr1, h0), (lr0 + sc1).astype(f16))
        upp, lr0, lr1 = up, h0, h1
        vmax = max(vmax, float(np.abs(h0).max()), float(np.abs(h1).max()))
        x = s - 127
        if 0 <= x < ncols:
            bottom[x] = int(h1[63, 1]) + base - 256 - (x + 1)
    right = np.zeros(256, dtype=np.int64)
    for q, (arr, half) in enumerate([(lr0, 0), (lr1, 0), (lr0, 1), (lr1, 1)]):
        right[rows[q] - 1] = arr[:, half].astype(np.int64) + base - rows[q] - ncols
    return bottom, right, vmax


def _tile_case(rng, ncols, R0, C0, all_match=False):
    n1, n2 = C0 + ncols, R0 + 256
    if all_match:
        s1, s2 = np.zeros(n1, dtype=np.int64), np.zeros(n2, dtype=np.int64)
    else:
        s1, s2 = rng.integers(0, 4, n1), rng.integers(0, 4, n2)
    H = full_dp(s1, s2)
    top = H[R0, C0 + 1:C0 + ncols + 1]
    left = H[R0 + 1:R0 + 257, C0]
    return H, top, left, H[R0, C0], s1[C0:], s2[R0:]


@pytest.mark.parametrize("ncols", [1, 30, 63, 64, 65, 100, 256, 300, 511, 512])
def test_packed_tile_model_matches_dp(ncols):
    rng = np.random.default_rng(ncols)
    for R0, C0, all_match in [(0, 0, False), (256, 3 * ncols, False), (0, ncols, True), (256, 0, True)]:
        H, top, left, corner, s1c, s2c = _tile_case(rng, ncols, R0, C0, all_match)
        bottom, right, vmax = packed_tile(top, left, corner, s1c, s2c)
        assert np.array_equal(bottom, H[R0 + 256, C0 + 1:C0 + ncols + 1]), (ncols, R0, C0, all_match)
        assert np.array_equal(right, H[R0 + 1:R0 + 257, C0 + ncols]), (ncols, R0, C0, all_match)
        # the f16-exactness bound (4 per diagonal step from the corner)
        assert vmax <= 4 * max(256, ncols) <= 2048


def test_packed_tile_reaches_the_f16_bound():
    """All-match input, the 256 x 512 tile at rows 512..768: its top row
    already climbs 4 per column (G(512, x) = 4 min(512, x)), so v reaches
    exactly 2048 — the end of the integer run f16 holds — and the outputs are
    still exact."""
    rng = np.random.default_rng(0)
    H, top, left, corner, s1c, s2c = _tile_case(rng, 512, 512, 0, all_match=True)
    bottom, right, vmax = packed_tile(top, left, corner, s1c, s2c)
    assert vmax == 2048
    assert np.array_equal(bottom, H[768, 1:513]) and np.array_equal(right, H[513:769, 512])


def test_model_dp_is_the_oracles():
    """The model's full DP agrees with the oracle's restatement of the
    reference tile program (oracle/sw_oracle.c) on the final score."""
    from oracle import loader as L

    rng = np.random.default_rng(7)
    for n1, n2, tw, th in [(300, 200, 300, 200), (513, 700, 171, 100), (1024, 512, 256, 256)]:
        s1, s2 = rng.integers(0, 4, n1), rng.integers(0, 4, n2)
        H = full_dp(s1[: n1 // tw * tw], s2[: n2 // th * th])
        want = L.sw_score((s1 + 1).astype(np.int8).tobytes(), (s2 + 1).astype(np.int8).tobytes(), tw, th)
        assert H[-1, -1] == want
