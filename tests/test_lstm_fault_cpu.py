"""The gconv-LSTM sequence launch's fault reporting on the host side
(ops.lstm_seq_fault over cg_lstm_seq_fault), with the C ABI replaced by a
stand-in: a timed-out pair hand-off (fault word set) raises CGError, an
in-flight launch polled without waiting returns None, a clean one False.  The
kernel side (NaN poisoning, the sticky word, layer() raising) is
tests/test_gpu_lstm.py::test_seq_handoff_timeout_raises_and_poisons."""
import ctypes
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pytest.importorskip("torch")


class FakeLib:
    def __init__(self, state):
        self.state = state  # 0 clean, -1 in flight, 1 fault
        self.calls = []

    def cg_lstm_seq_fault(self, handle, wait, clear, fault_ptr):
        self.calls.append((handle, wait, clear))
        st = self.state if not (wait and self.state == -1) else 0
        ctypes.cast(fault_ptr, ctypes.POINTER(ctypes.c_int32))[0] = st
        return 0 if st <= 0 else 2  # CG_ERR_HIP on a fault

    def cg_last_error(self):
        return b"k_lstm_seq pair hand-off timed out"


class Plan:
    handle = 1234


@pytest.mark.parametrize("state,wait,expect", [(0, True, False), (-1, False, None), (-1, True, False)])
def test_fault_poll_states(monkeypatch, state, wait, expect):
    from cnn_graph_amd import _lib, ops
    fake = FakeLib(state)
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    assert ops.lstm_seq_fault(Plan(), wait=wait) is expect
    assert fake.calls == [(1234, int(wait), 1)]


def test_fault_raises(monkeypatch):
    from cnn_graph_amd import _lib, ops
    monkeypatch.setattr(_lib, "lib", lambda: FakeLib(1))
    with pytest.raises(_lib.CGError, match="hand-off timed out"):
        ops.lstm_seq_fault(Plan(), wait=False)
