"""Host logic of the bf16 parameter shadow (native_ops.param_shadow): when a
shadow is trusted.  No kernels run; the GPU test is test_param_shadow_gpu.py."""
import pytest
import torch


@pytest.fixture
def ops():
    from pytorch_end2end_speech_recognition_amd import native_ops
    prev = native_ops.compute_dtype()
    native_ops.set_compute_dtype('bf16')
    yield native_ops
    native_ops.set_compute_dtype('bf16' if prev == native_ops.BF16 else 'fp32')


def _model():
    flat = torch.zeros(256)
    params = [torch.nn.Parameter(torch.zeros(8, 4)), torch.nn.Parameter(torch.zeros(8, 4))]
    for p, o in zip(params, (64, 96)):
        p.data = flat[o:o + 32].view(8, 4)
    w = flat[64:128].view(16, 4)          # a layer's combined [fwd; rev] view
    return flat, params, w


def test_shadow_trusted_only_after_the_step_and_until_a_write(ops, monkeypatch):
    monkeypatch.delenv('ASR_PARAM_SHADOW', raising=False)
    flat, params, w = _model()
    sh = ops.param_shadow(flat)
    assert sh is not None and sh.buf.dtype == torch.bfloat16 and sh.buf.numel() == 256
    assert ops._shadow_rows(w, params) is None            # never written
    sh.buf.copy_(torch.arange(256, dtype=torch.bfloat16))
    ops.param_shadow_written(sh, flat, params)
    rows = ops._shadow_rows(w, params)
    assert rows.shape == (16, 4) and rows.data_ptr() == sh.buf[64:].data_ptr()
    assert ops.param_shadow(flat) is sh                   # one shadow per flat buffer
    with torch.no_grad():
        params[1].mul_(2.0)                               # a parameter's own write
    assert ops._shadow_rows(w, params) is None
    ops.param_shadow_written(sh, flat, params)
    assert ops._shadow_rows(w, params) is not None
    flat[0:4].fill_(1.0)                                  # a write through the flat buffer
    assert ops._shadow_rows(w, params) is None


def test_shadow_off_in_fp32_and_by_switch(ops, monkeypatch):
    flat, params, w = _model()
    monkeypatch.setenv('ASR_PARAM_SHADOW', '0')
    assert ops.param_shadow(flat) is None
    monkeypatch.delenv('ASR_PARAM_SHADOW')
    ops.set_compute_dtype('fp32')
    assert ops.param_shadow(flat) is None
    assert ops._shadow_rows(w.clone(), params) is None    # not a view of a flat buffer
