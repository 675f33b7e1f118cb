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
