"""Host-side helpers of the logits path (no GPU): row padding for vocabularies the
16-B row vectors do not divide (lac_amd.batch.pad_logits / logits_row_multiple)."""
import pytest

torch = pytest.importorskip("torch")


def test_pad_logits_to_the_vector_multiple():
    from lac_amd.batch import logits_row_multiple, pad_logits
    assert logits_row_multiple(torch.bfloat16) == 8 and logits_row_multiple(torch.float32) == 4
    for dt, V, Vp in ((torch.bfloat16, 50257, 50264), (torch.float32, 50257, 50260), (torch.bfloat16, 32000, 32000)):
        x = torch.randn((3, 2, V)).to(dt)
        y = pad_logits(x)
        assert y.shape == (3, 2, Vp) and y.is_contiguous() and y.dtype == dt
        assert torch.equal(y[..., :V], x) and torch.isneginf(y[..., V:].float()).all()
    with pytest.raises(TypeError):
        logits_row_multiple(torch.float16)
