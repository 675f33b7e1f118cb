"""CPU: the arithmetic behind the depth sort's key range (sort.hip KeyRange), restated in numpy.

The depth sort sorts key' = key - kmin over the keys other than 0xFFFFFFFF (Gaussians behind the near plane), those
getting t, the least value past max - kmin whose low byte is (0xFF - kmin) mod 256; pass 0 counts raw low bytes and
reads them rotated by kmin's low byte.  These checks are what makes that the 32-bit stable order (the GPU side:
tests/test_gpu_depth_sort.py):
  * the stable order of key' equals the stable order of the raw keys;
  * pass 0's digit of key' is the raw low byte minus kmin's, mod 256, for every key (0xFFFFFFFF included);
  * t never wraps and its byte count is the working pass count.
"""
import numpy as np
import pytest


def _range(keys):
    valid = keys[keys != 0xFFFFFFFF]
    if valid.size == 0:
        return 0, 0xFF
    kmin, hi = int(valid.min()), int(valid.max())
    r1 = hi - kmin + 1
    return kmin, r1 + ((((0xFF - kmin) & 0xFF) - r1) & 0xFF)


def _keyp(keys, kmin, t):
    k = keys.astype(np.int64)
    return np.where(keys == 0xFFFFFFFF, t, k - kmin)


def _lsd_order(kp, passes):
    """Stable LSD radix order over `passes` bytes of kp (numpy's stable argsort per byte)."""
    order = np.arange(kp.size)
    for p in range(passes):
        d = (kp[order] >> (8 * p)) & 0xFF
        order = order[np.argsort(d, kind="stable")]
    return order


CASES = {
    "span24": lambda r, n: np.float32(1.3) + np.float32(3.4) * r.random(n, dtype=np.float32),
    "wide": lambda r, n: np.exp(r.uniform(np.log(0.21), np.log(5000.0), n)).astype(np.float32),
    "ties": lambda r, n: np.array([0.7, 1.1, 2.5, 9.0], np.float32)[r.integers(0, 4, n)],
    "narrow": lambda r, n: (np.float32(2.0) + np.float32(1e-5) * r.random(n, dtype=np.float32)).astype(np.float32),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("behind", [0.0, 0.1, 1.0])
def test_key_range_order_is_the_32bit_order(case, behind):
    rng = np.random.default_rng(5)
    n = 20_011
    keys = CASES[case](rng, n).astype(np.float32).view(np.uint32).copy()
    keys[rng.random(n) < behind] = 0xFFFFFFFF
    kmin, t = _range(keys)
    assert t <= 0xFFFFFFFF - kmin  # no wrap
    kp = _keyp(keys, kmin, t)
    assert int(kp.max()) == t or not (keys == 0xFFFFFFFF).any()
    assert int(kp[keys != 0xFFFFFFFF].max(initial=-1)) < t  # the 0xFFFFFFFF keys sort last
    passes = max(1, (int(t).bit_length() + 7) // 8)
    assert (kp >> (8 * passes) == 0).all()  # the skipped passes see one digit value: the identity
    # pass 0's rotation: the low byte of key' from the raw low byte
    np.testing.assert_array_equal(kp & 0xFF, (keys.astype(np.int64) - kmin) & 0xFF)
    want = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(_lsd_order(kp, passes), want)
    np.testing.assert_array_equal(_lsd_order(keys.astype(np.int64), 4), want)
