"""Host-side guards that need no GPU."""
import pytest
import torch

import icm as icm_native


def _bare_icm():
    nat = object.__new__(icm_native.NativeIcm)
    nat._bufs, nat._captured = {}, set()

    class _Flat:
        device = torch.device("cpu")
    nat.flat = _Flat()
    return nat


def test_captured_icm_workspace_cannot_grow(monkeypatch):
    """A workspace the collect graph captured (icm.py _buf) raises instead of being
    silently replaced by a larger allocation the replayed graph would not see."""
    nat = _bare_icm()
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    a = nat._buf("ir", (8,))
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    assert nat._buf("ir", (8,)).data_ptr() == a.data_ptr()  # captured at this size
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    assert nat._buf("ir", (4,)).data_ptr() == a.data_ptr()  # smaller views are fine
    with pytest.raises(RuntimeError, match="captured"):
        nat._buf("ir", (16,))
    with pytest.raises(RuntimeError, match="captured"):
        nat._buf("ir", (8,), torch.int32)
    b = nat._buf("mb_phi", (4,))  # uncaptured tags still grow
    assert nat._buf("mb_phi", (64,)).numel() == 64 and b.numel() == 4
