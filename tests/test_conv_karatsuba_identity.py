"""CPU (float64): conv3 / conv4 (Beluga.py:29-32, an 8-tap correlation over all input channels)
equals the pair Karatsuba form of the round-5 probe kernel (tools/ck_karatsuba.h beluga_conv_h3k,
measured slower than the direct kernel and kept out of the library): per output
pair (y[2p], y[2p+1]), S + V and S + U with S over the pair sums s[q] = x[2q] + x[2q+1] (4 taps),
V over the odd rows (4 taps) and U over the even rows (5 taps) -- 13 K blocks per pair instead of
16 -- with the weights in the kernel's step order (S, U, V; chunk-major, tap-minor) as ck_weights
built them.  Channels shrunk so the check runs in milliseconds."""
import numpy as np

CIN, COUT, CH = 64, 5, 32          # two 32-channel chunks


def _step_weights(W):
    """W [COUT, CIN, 8] -> [COUT, 13 * CIN] in ck_weights' order: kb = (phase, chunk, tap), k = kb*32 + j."""
    nch = CIN // CH
    w = lambda c, t: W[:, c * CH:(c + 1) * CH, t] if 0 <= t <= 7 else np.zeros((COUT, CH))
    blocks = []
    for c in range(nch):                                  # S: w_2i
        blocks += [w(c, 2 * i) for i in range(4)]
    for c in range(nch):                                  # U: w_2i-1 - w_2i
        blocks += [w(c, 2 * i - 1) - w(c, 2 * i) for i in range(5)]
    for c in range(nch):                                  # V: w_2i+1 - w_2i
        blocks += [w(c, 2 * i + 1) - w(c, 2 * i) for i in range(4)]
    return np.concatenate(blocks, axis=1)


def _karatsuba(x, Wk):
    """y [2P, COUT] from x [2P + 8, CIN] (rows) and the step-order weights."""
    nch = CIN // CH
    P = (x.shape[0] - 8) // 2
    xe, xo = x[0::2], x[1::2]                             # rows 2q, 2q + 1
    s = xe + xo
    acc_e = np.zeros((P, COUT))
    kb = 0
    for seq, taps, phase in ((s, 4, "S"), (xe, 5, "U"), (xo, 4, "V")):
        if phase == "U":
            acc_o = acc_e.copy()                          # the shared S, then U into acc_o
        for c in range(nch):
            for i in range(taps):
                a = seq[i:i + P, c * CH:(c + 1) * CH]
                prod = a @ Wk[:, kb * CH:(kb + 1) * CH].T
                if phase == "U":
                    acc_o += prod
                else:
                    acc_e += prod
                kb += 1
    y = np.empty((2 * P, COUT))
    y[0::2], y[1::2] = acc_e, acc_o
    return y


def test_pair_karatsuba_equals_the_direct_correlation():
    rng = np.random.default_rng(0)
    W = rng.standard_normal((COUT, CIN, 8))
    for P in (1, 7, 20):
        x = rng.standard_normal((2 * P + 8, CIN))
        want = np.stack([np.einsum("oct,tc->o", W, x[t:t + 8]) for t in range(2 * P)])
        got = _karatsuba(x, _step_weights(W))
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-11)


def test_thirteen_k_blocks_per_pair():
    W = np.zeros((COUT, CIN, 8))
    assert _step_weights(W).shape[1] == 13 * CIN             # vs 16 * CIN for two direct outputs
