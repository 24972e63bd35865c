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


def _bare_comm(inflight=False, handle=1):
    import native
    c = object.__new__(native.DpComm)
    c.handle, c.world, c.rank, c.inflight = handle, 2, 0, inflight
    return c


def test_dp_comm_refuses_a_second_async_reduction():
    """one asynchronous reduction in flight at a time on the native communicator (a second
    one before the join is refused — csrc/dp.cpp returns the same error); a closed communicator refuses all."""
    import native
    t = torch.zeros(4)
    with pytest.raises(native.NativeError, match="in flight"):
        _bare_comm(inflight=True).all_reduce_(t, wait=False)
    with pytest.raises(native.NativeError, match="closed"):
        _bare_comm(handle=None).all_reduce_(t)
    assert _bare_comm(handle=None).close() == 0  # idempotent


def test_dist_shutdown_closes_the_native_communicator(monkeypatch):
    """dist.shutdown() destroys the process's native communicator (before the process group goes) and forgets
    it; a second call is a no-op."""
    import dist
    closed = []

    class _Comm:
        def close(self):
            closed.append(1)
            return 0
    monkeypatch.setattr(dist, "_dp_comm", _Comm())
    assert dist.shutdown() == 0 and closed == [1] and dist._dp_comm is None
    assert dist.shutdown() is None and closed == [1]
