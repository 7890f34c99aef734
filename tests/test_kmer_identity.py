"""CPU: the k-mer regrouping the library's conv2 gather rests on (DESIGN.md §3 "conv1 + conv2 as
a k-mer table").  With F(x) = relu(conv1) of an 8-mer and W2_j conv2's tap matrices
(Beluga.py:23-26), conv2 at position p equals

    sum_{i<4} T_i(9-mer at p + 2i)       T_i(y) = W2_{2i} F(y_0..7) + W2_{2i+1} F(y_1..8)
    Q_0(11-mer at p) + Q_1(11-mer at p+4)  Q_h(y) = sum_{t<4} W2_{4h+t} F(y_t..t+7)

for every base sequence over A, G, C, T, N (N = the zero one-hot column, chromatin.py:155-160).
Checked in float64 against the direct conv1 -> ReLU -> conv2 (Beluga.py:23-26 written out) on
seeded weights of Beluga's shapes and a sequence with an N run and scattered N."""
import numpy as np


def _onehot(codes):
    """[4, L] float64: channel c for code c < 4 (encodeSeqs' A, G, C, T order), all zero for N."""
    x = np.zeros((4, len(codes)))
    k = codes < 4
    x[codes[k], np.nonzero(k)[0]] = 1.0
    return x


def _direct(w1, b1, w2, codes):
    """conv2 (before its bias) at every position p < L - 14 of one sequence, float64."""
    x = _onehot(codes)                                   # [4, L]
    L = x.shape[1]
    c1 = np.stack([np.einsum("oc,cl->ol", w1[:, :, k], x[:, k:L - 7 + k]) for k in range(8)]).sum(0)
    f = np.maximum(c1 + b1[:, None], 0.0)               # [320, L - 7]
    T = f.shape[1] - 7
    return np.stack([np.einsum("oc,cl->ol", w2[:, :, j], f[:, j:T + j]) for j in range(8)]).sum(0)


def _F(w1, b1, mer):
    s = b1.copy()
    for k, c in enumerate(mer):
        if c < 4:
            s += w1[:, c, k]
    return np.maximum(s, 0.0)


def test_pair_and_quad_tables_equal_the_direct_conv2():
    rng = np.random.default_rng(3)
    w1 = rng.normal(0, 0.5, (320, 4, 8))
    b1 = rng.normal(0, 0.5, 320)
    w2 = rng.normal(0, 0.05, (320, 320, 8))
    codes = rng.integers(0, 4, 160).astype(np.uint8)
    codes[40:52] = 4                                     # an N run
    codes[::23] = 4                                      # scattered N
    want = _direct(w1, b1, w2, codes)                    # [320, 160 - 14]
    pad = np.concatenate([codes, np.full(16, 4, np.uint8)])   # past the end: N
    for p in range(want.shape[1]):
        pair = sum(w2[:, :, 2 * i] @ _F(w1, b1, pad[p + 2 * i:p + 2 * i + 8])
                   + w2[:, :, 2 * i + 1] @ _F(w1, b1, pad[p + 2 * i + 1:p + 2 * i + 9]) for i in range(4))
        quad = sum(sum(w2[:, :, 4 * h + t] @ _F(w1, b1, pad[p + 4 * h + t:p + 4 * h + t + 8]) for t in range(4))
                   for h in range(2))
        np.testing.assert_allclose(pair, want[:, p], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(quad, want[:, p], rtol=1e-12, atol=1e-12)


def test_table_indices_cover_the_kmers():
    """The gather's row indices: a 9-mer is sum_k c_k 5^k (digit k = base k), a quad 11-mer of
    A, G, C, T sum_k c_k 4^k; the pair table's two 8-mers are m9 % 5^8 and m9 // 5 (kmer_pair)."""
    rng = np.random.default_rng(4)
    for _ in range(200):
        c = rng.integers(0, 5, 9)
        m9 = int(sum(int(d) * 5 ** k for k, d in enumerate(c)))
        assert m9 % 5 ** 8 == sum(int(d) * 5 ** k for k, d in enumerate(c[:8]))
        assert m9 // 5 == sum(int(d) * 5 ** k for k, d in enumerate(c[1:]))
    assert 5 ** 9 == 1953125 and 4 ** 11 == 4194304
