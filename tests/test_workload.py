"""The synthetic inputs: the numpy builder the bench uses for
host-staged rounds produces the same Entry rows and Cmd pool as the
reference builder (workload.build_batch), which the GPU generator matches
(tests/test_gpu_parity.py)."""
import ctypes as C

import pytest

from dragonboat_amd import workload as w


@pytest.mark.parametrize("salt", [0, 1, 77, 1 << 20])
def test_build_batch_np_matches_build_batch(salt):
    c, e, p = w.build_batch(257, 1, 0x5EEDD8B0, salt)
    c2, e2, p2 = w.build_batch_np(257, 0x5EEDD8B0, salt)
    assert bytes(C.string_at(C.addressof(e), C.sizeof(e))) == e2.tobytes()
    assert bytes(p) == p2.tobytes()
    assert list(c) == c2.tolist()
