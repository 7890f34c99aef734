"""Host-side geometry of the fused conv4 + pool2 epilogue (gemm_kernel.h epilogue_pool_ph02,
beluga.hip run_conv4_pool_fused / seg_delta_pool): the alt windows' ref conv4 rows that the epilogue
keeps unpooled fit the 32-row-per-segment buffer for every SNV position, and the 4-aligned conv3
stride puts every segment's pool groups on 4-aligned rows of conv4's M index space.

Restates seg_delta_table (beluga.hip) for phases {0, 2}; no GPU."""
import numpy as np
import pytest

K_DW4 = 6          # kDW[4]: pooled rows of an alt run per phase
K_W4U = 19         # kW4u: conv4 rows of the alt run
K_SEG_EDGE = 32    # kSegEdge


def floor4(v):
    return v >> 2 if v >= 0 else -((3 - v) >> 2)


def clampi(v, lo, hi):
    return max(lo, min(v, hi))


def seg_dims(L):
    T1 = L - 7
    P1 = (T1 - 7) // 4
    T3 = P1 - 7
    T4 = T3 - 7
    S5 = T4 // 4
    return T1, P1, T3, T4, S5


def edge_range(q, L):
    """[lo, hi) of conv4 rows seg_delta_pool reads for an SNV at q (beluga.hip seg_delta_table)."""
    T1, P1, T3, T4, S5 = seg_dims(L)
    r1 = clampi(q - 7, 0, T1 - 8)
    r2 = clampi(floor4(r1 - 7), 0, P1 - 5)
    r3 = clampi(r2 - 7, 0, T3 - 12)
    r4 = clampi(r3 - 7, 0, T4 - K_W4U)
    t5 = clampi(floor4(r4 - 0), 0, S5 - K_DW4)
    t6 = clampi(floor4(r4 - 2), 0, S5 - K_DW4)
    lo = min(4 * t5, 2 + 4 * t6)
    hi = max(4 * (t5 + K_DW4), 2 + 4 * (t6 + K_DW4))
    return lo, hi, t5, t6


@pytest.mark.parametrize("L", [41_800, 3_600, 10_000])
def test_alt_edge_rows_fit_the_segment_buffer(L):
    for q in range(0, L, 3):
        lo, hi, t5, t6 = edge_range(q, L)
        assert 0 <= lo < hi and hi - lo <= K_SEG_EDGE, (L, q, lo, hi)
        # every row seg_delta_pool reads (phase p, pooled rows tab[5 + i] .. + 6, 4 rows each) is inside
        for p, t in ((0, t5), (2, t6)):
            rows = [p + 4 * (t + g) + j for g in range(K_DW4) for j in range(4)]
            assert lo <= min(rows) and max(rows) < hi


@pytest.mark.parametrize("L", [41_800, 41_804, 41_808, 41_812, 3_600])
def test_segment_rows_start_4_aligned_with_the_padded_conv3_stride(L):
    _, _, T3, T4, _ = seg_dims(L)
    t3p = (T3 + 3) & ~3
    assert t3p % 4 == 0 and T4 <= t3p < T3 + 4
    starts = np.arange(64) * t3p
    assert np.all(starts % 4 == 0)
    # a phase-0 group (rows t .. t+3, t = 0 mod 4 in segment coordinates) is one lane's 4 accumulator
    # rows of a 16-row block; a phase-2 group crosses to the next lane group or block
    for w in range(8):
        for t in range(0, T4 - 3, 4):
            m = w * t3p + t
            assert m % 4 == 0 and (m % 16) // 4 == ((m + 3) % 16) // 4
