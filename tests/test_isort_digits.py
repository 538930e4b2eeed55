"""The MSD index sort's range-proportional digits (csrc/mq_isort.hip: digit_of,
digit_lo, the level policy in msd_index_sort), restated on the host: for a level
over keys x in [0, R) with P digits, M = floor(2^32 P / R) and d(x) = floor(x M / 2^32)
must be monotone and below P; digit d's keys are [lo(d), lo(d + 1)) with
lo(d) = ceil(d 2^32 / M); a child spans at most floor(2^32 / M) + 1 keys (the next
level's R); and the next level's digit of a key relative to its child stays below
that level's P. These are what let the children kernel place ranges without
looking at the data, so they are checked exhaustively on small R and by sampling on
large ones. No GPU."""
import numpy as np
import pytest

TWO32 = 1 << 32


def digit(x, M):
    return (x * M) >> 32


def lo(d, M):
    return -((-(d << 32)) // M)  # ceil(d 2^32 / M)


def check_level(R, P, xs):
    M = (P << 32) // R
    assert M >= 1
    ds = [digit(x, M) for x in xs]
    assert all(0 <= d < P for d in ds), (R, P)
    assert all(a <= b for a, b in zip(ds, ds[1:])), (R, P)  # xs ascending
    Rn = TWO32 // M + 1
    for x, d in zip(xs, ds):
        assert lo(d, M) <= x < lo(d + 1, M), (R, P, x)
        assert min(lo(d + 1, M), R) - lo(d, M) <= Rn, (R, P, d)
    return M, Rn


@pytest.mark.parametrize("R", [2, 3, 7, 255, 256, 257, 1000, 4096, 65537])
@pytest.mark.parametrize("P", [2, 3, 100, 255, 256])
def test_digits_exhaustive_small(R, P):
    check_level(R, P, list(range(R)))


def test_digits_sampled_large():
    rng = np.random.default_rng(3)
    for R in [1 << 32, (1 << 32) - 1, 1_000_000_000, 999_999_937, 1 << 30, 3_908_069, 16_385, 15_266]:
        for P in [2, 7, 86, 255, 256]:
            xs = sorted(set(int(v) for v in rng.integers(0, R, 2000)) | {0, R - 1} |
                        {min(R - 1, lo(d, (P << 32) // R)) for d in range(P)})
            check_level(R, P, xs)


def test_two_levels_of_the_1e9_column():
    """The bench column's keys span 1e9: 256 digits, then 256 more within each child,
    leave 65536 ranges of <= 15 266 keys (<= 2^14: the counting finisher takes them)."""
    R0, P = 1_000_000_000, 256
    M0, R1 = check_level(R0, P, [0, R0 // 3, R0 - 1])
    assert R1 == 3_908_069
    M1, R2 = check_level(R1, P, [0, R1 // 2, R1 - 1])
    assert R2 <= 1 << 14
    # a key relative to its child of level 0 (the next level's digit byte, written by
    # the level-0 scatter) is below R1 and its level-1 digit below 256
    rng = np.random.default_rng(5)
    for x in rng.integers(0, R0, 5000):
        x = int(x)
        d = digit(x, M0)
        y = x - lo(d, M0)
        assert 0 <= y < R1 and digit(y, M1) < P
