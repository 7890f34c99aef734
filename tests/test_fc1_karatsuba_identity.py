"""CPU (float64): FC1 (Beluga.py:43-44; y = W . flatten(conv6 rows), rows t*640 + c as the library
repacks it) equals the block-Karatsuba form the f16x3 library runs (beluga.hip "FC1 as a
block-Karatsuba convolution"): per window, in each of its 4 roles, the sum of its 4 block products
of the D1 / D2 / DD row sequences plus the tail -- computed from the window's own rows alone, and
computed once per group of 4 windows 25 rows apart and shared -- with C channels shrunk to 3 so
the check runs in milliseconds."""
import numpy as np

C = 3                       # conv6 channels (640 in Beluga)
ROWS = 106                  # conv6 rows per window
N = 5                       # FC1 outputs (2003)
SEQ = [3, 2, 3, 1, 0, 1, 3, 2, 3]           # product g: sequence (0 x, 1 D1, 2 D2, 3 DD)
BLK = [0, 1, 1, 2, 3, 3, 2, 3, 3]           #   at block BLK[g] of its group
ROLE = [[0, 1, 3, 4], [1, 2, 4, 5], [3, 4, 6, 7], [4, 5, 7, 8]]
COEF = [[1, 0, 0, 0], [1, 1, 0, 0], [0, -1, 0, 0], [1, 0, 1, 0], [1, 1, 1, 1],
        [0, -1, 0, -1], [0, 0, -1, 0], [0, 0, -1, -1], [0, 0, 0, 1]]


def _sequences(x):
    """D1, D2, DD over the rows of x [R, C] (NaN where a lag row is missing)."""
    R = x.shape[0]
    pad = np.full((75, C), np.nan)
    xp = np.concatenate([x, pad])
    d1 = xp[:R] - xp[25:R + 25]
    d2 = xp[:R] - xp[50:R + 50]
    dd = (xp[:R] - xp[25:R + 25]) - (xp[50:R + 50] - xp[75:R + 75])
    return [x, d1, d2, dd]


def _weights(W):
    """Product weights [9][N, 25*C] and the tail [N, 6*C] from W [N, 106*C] (K = t*C + c)."""
    V = [W[:, 25 * q * C:25 * (q + 1) * C] for q in range(4)]
    return [sum(c * v for c, v in zip(COEF[g], V)) for g in range(9)], W[:, 100 * C:]


def _product(seqs, Wg, g, gstart):
    s = seqs[SEQ[g]]
    a = s[gstart + 25 * BLK[g]:gstart + 25 * BLK[g] + 25].reshape(-1)
    assert not np.isnan(a).any(), "a product read a row outside the window"
    return Wg[g] @ a


def test_every_role_equals_direct_fc1_from_its_own_rows():
    rng = np.random.default_rng(0)
    W = rng.standard_normal((N, ROWS * C))
    Wg, T = _weights(W)
    for role in range(4):
        x = rng.standard_normal((ROWS, C))
        seqs = _sequences(x)            # the window's own rows only: a NaN read would show
        gstart = -25 * role
        # shift into non-negative row coordinates: pad the window's rows in front
        seqs = [np.concatenate([np.full((25 * role, C), np.nan), s]) for s in seqs]
        y = sum(_product(seqs, Wg, g, gstart + 25 * role) for g in ROLE[role])
        y = y + T @ x[100:106].reshape(-1)
        np.testing.assert_allclose(y, W @ x.reshape(-1), rtol=1e-12, atol=1e-12)


def test_shared_group_products_equal_direct_fc1_of_every_window():
    """A pool2-phase block of conv6 rows with 11 windows 25 rows apart (two full groups and a
    partial one): products computed once per group and shared give every window's FC1."""
    rng = np.random.default_rng(1)
    W = rng.standard_normal((N, ROWS * C))
    Wg, T = _weights(W)
    R = 25 * 10 + ROWS
    x = rng.standard_normal((R, C))
    seqs = _sequences(x)
    cache = {}
    for j in range(11):
        off = 25 * j
        role = j % 4
        gstart = off - 25 * role
        y = T @ x[off + 100:off + 106].reshape(-1)
        for g in ROLE[role]:
            if (gstart, g) not in cache:
                cache[(gstart, g)] = _product(seqs, Wg, g, gstart)
            y = y + cache[(gstart, g)]
        np.testing.assert_allclose(y, W @ x[off:off + ROWS].reshape(-1), rtol=1e-12, atol=1e-12)
    # 9 products per full group of 4 windows instead of 16 block products
    assert sum(1 for (gs, _g) in cache if gs == 0) == 9


def test_roles_and_group_starts_from_offsets():
    """The library's role rule on the segment path: role = (conv6 offset / 25) mod 4 with conv6
    offset = bp offset / 16 (pipeline.fc1_role), so 200-bp sweeps alternate pool2 phases and
    same-phase windows 400 bp apart are consecutive roles of one group."""
    from expecto_amd.pipeline import fc1_role, sweep_roles
    assert [fc1_role(o, 41800) for o in (0, 400, 800, 1200, 1600, 2000)] == [0, 1, 2, 3, 0, 1]
    assert [fc1_role(o, 41800) for o in (200, 600, 1000, 1400)] == [0, 1, 2, 3]
    assert fc1_role(0, 41800, rc=True) == fc1_role(39800, 41800)
    r = sweep_roles(list(range(-20000, 20000, 200)))
    assert r.shape == (2, 200) and set(r.ravel().tolist()) == {0, 1, 2, 3}
