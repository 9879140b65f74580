"""csrc/common.h fdiv24: n / d from a float reciprocal plus one correction step is exact for 0 <= n < 2^24.
The GPU's v_cvt_f32_i32 / v_mul_f32 / v_cvt_i32_f32 are IEEE round-to-nearest / truncation, which numpy's
float32 arithmetic reproduces; every divisor a weight-gradient launch can see (HWo, Wo up to 100 x 250 maps)
and n across the whole range, its edges and every multiple boundary of small divisors."""
import numpy as np


def fdiv24(n: np.ndarray, d: int) -> np.ndarray:
    inv = np.float32(1.0) / np.float32(d)
    q = (n.astype(np.float32) * inv).astype(np.int64)  # trunc toward zero, n >= 0
    r = n - q * d
    return q + (r >= d).astype(np.int64) - (r < 0).astype(np.int64)


def test_fdiv24_exact():
    rng = np.random.default_rng(0)
    top = 1 << 24
    divisors = list(range(1, 4097)) + [5 * 11, 9 * 21, 17 * 42, 33 * 83, 47 * 122, 100 * 250, 10007, 65521,
                                       1 << 20, top - 1]
    for d in divisors:
        n = np.concatenate([rng.integers(0, top, 4096), np.arange(0, min(top, 4 * d + 64)),
                            np.arange(top - 4 * d - 64 if top > 4 * d + 64 else 0, top)])
        k = np.arange(1, min(top // d, 2048)) * d
        n = np.concatenate([n, k - 1, k, k + 1])
        n = n[(n >= 0) & (n < top)]
        assert np.array_equal(fdiv24(n, d), n // d), d
