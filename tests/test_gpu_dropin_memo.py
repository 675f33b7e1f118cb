"""The drop-in backward's memo for equal cotangents (diff_gaussian_rasterization/__init__.py, _RasterizeGaussians.backward).

The reference's J^T v (solver_functions.py:101-132) runs two backward calls on one graph, one per half of the [r; r]
pair (loss_image_state.py:93-97); with disable_ssim both halves are the same image (batch_training_loss.py:15-17), so
the two cotangents are equal.  A call whose cotangent equals the previous call's (element for element) returns that
call's gradients.  Checked here through the reference's render() (gslm.train.render: activations in PyTorch, so the
returned gradients pass through autograd nodes and are accumulated into the leaves):
  * equal cotangents (a different tensor with the same values, as the reference's CG vectors are): every leaf's
    accumulated gradient bitwise that of the same two calls with the memo off;
  * a different cotangent on the second call, and a third call after the memo was used: bitwise as with it off
    (the memo is keyed on content and autograd never writes into the returned tensors).
"""
import pytest
import torch

from scenes import make_scene

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grads_of(model, calls, memo, monkeypatch):
    import diff_gaussian_rasterization as dgr
    from gslm.train import PipelineParams, render
    monkeypatch.setattr(dgr, "_BWD_MEMO", memo)
    cam = _grads_of.cam
    model.zero_grad()
    img = render(cam, model, PipelineParams(), torch.zeros(3, device=DEV))["render"]
    r = img - _grads_of.gt
    for k, v in enumerate(calls):
        r.backward(v, retain_graph=k + 1 < len(calls))
    return [None if t.grad is None else t.grad.detach().clone() for t in model.params()]


@pytest.mark.parametrize("pattern", ["equal", "different", "equal_then_different", "three_equal"])
def test_backward_memo_is_bitwise(pattern, monkeypatch):
    model, cams = make_scene("dense_2k_sh3_64x48")
    model = model.to(DEV)
    cam = cams[0].to(DEV)
    g = torch.Generator().manual_seed(11)
    shape = (3, int(cam.image_height), int(cam.image_width))
    _grads_of.cam = cam
    _grads_of.gt = torch.rand(shape, generator=g).to(DEV)
    v = torch.randn(shape, generator=g).to(DEV)
    w = torch.randn(shape, generator=g).to(DEV)
    calls = {"equal": [v, v.clone()],
             "different": [v, w],
             "equal_then_different": [v, v.clone(), w],
             "three_equal": [v, v.clone(), v.clone()]}[pattern]
    on = _grads_of(model, calls, True, monkeypatch)
    off = _grads_of(model, calls, False, monkeypatch)
    assert any(t is not None and t.abs().max() > 0 for t in off)
    for a, b in zip(on, off):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
