"""Device self-tests of the wave primitives and the sort/scan building blocks (through the C ABI)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _selftest(which, x):
    from gslm import _lib
    out = torch.zeros(64, dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib.gslm_selftest(which, x.data_ptr(), out.data_ptr(), _lib.stream_handle()))
    torch.cuda.synchronize()
    return out.cpu()


def test_transposed_wave_reduction():
    g = torch.Generator().manual_seed(0)
    x = torch.randint(-1000, 1000, (64, 8), generator=g).float()  # integers: exact sums
    got = _selftest(0, x.cuda().contiguous())
    ref = x.sum(dim=0)
    for lane in range(64):
        assert got[lane].item() == ref[(lane >> 3) & 7].item(), lane


def test_dpp_wave_sum():
    g = torch.Generator().manual_seed(1)
    x = torch.randint(-1000, 1000, (64, 8), generator=g).float()
    got = _selftest(1, x.cuda().contiguous())
    assert got[63].item() == x[:, 0].sum().item()


@pytest.mark.parametrize("n", [1, 2047, 2048, 2049, 300_000, 9_000_001])
@pytest.mark.parametrize("force_top", [0, 1])
def test_exclusive_scan_both_forms(n, force_top):
    """the scan's apply pass sums its own prefix of block sums (O(nb^2) loads over the grid) only up to
    4096 blocks of 2048; longer scans (the LM row map at 5M Gaussians / 4K: nb ~ 12k-49k) scan the block sums in a
    launch of their own.  Both forms against torch's cumsum, exact (9M elements: nb = 4395 takes the long form
    unforced)."""
    from gslm import _lib
    g = torch.Generator().manual_seed(n)
    x = torch.randint(0, 64, (n,), generator=g, dtype=torch.int64)
    xin = x.to(torch.int32).cuda()
    out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    tmp = torch.empty((8 * ((n + 2047) // 2048) + 64 + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    tot = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.gslm_selftest_scan(xin.data_ptr(), out.data_ptr(), n, force_top, tmp.data_ptr(), tmp.numel(),
                                           tot.data_ptr(), _lib.stream_handle()))
    torch.cuda.synchronize()
    ref = torch.cumsum(x, 0) - x
    assert torch.equal(out.cpu().to(torch.int64), ref)
    assert int(tot.item()) == int(x.sum())
