"""The RCCL transport of the PT swap (runtime.hip: bcm3hip_nccl_*), on the one GPU a test box has:
a one-rank communicator sending the boundary records to itself in one grouped round, in the
order SamplerPTDevice posts them (send last -> next, send first -> prev, recv prev, recv next).
The multi-rank exchange logic itself is covered bit for bit by tests/test_ptmh_native_gpu.py
(in-process ranks) and tests/test_pt.py (gloo)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_rccl_self_exchange_round():
    from bcm3_amd import _hip
    L = _hip.lib()
    vp = C.c_void_p
    L.bcm3hip_nccl_get_unique_id.argtypes = [vp]
    L.bcm3hip_nccl_comm_init.argtypes = [vp, C.c_int, C.c_int, C.POINTER(vp)]
    L.bcm3hip_nccl_comm_destroy.argtypes = [vp]
    L.bcm3hip_nccl_exchange.argtypes = [vp, C.c_int, vp, vp, C.c_int, vp, vp, C.c_size_t, vp]
    uid = (C.c_uint8 * 128)()
    assert L.bcm3hip_nccl_get_unique_id(uid) == 0
    comm = vp()
    assert L.bcm3hip_nccl_comm_init(uid, 0, 1, C.byref(comm)) == 0
    try:
        d = 12
        last = torch.arange(d + 4, dtype=torch.float64, device="cuda")
        first = -torch.arange(d + 4, dtype=torch.float64, device="cuda") - 1
        recv_prev = torch.zeros(d + 4, dtype=torch.float64, device="cuda")
        recv_next = torch.zeros(d + 4, dtype=torch.float64, device="cuda")
        sends = (vp * 2)(last.data_ptr(), first.data_ptr())
        recvs = (vp * 2)(recv_prev.data_ptr(), recv_next.data_ptr())
        peers = (C.c_int * 2)(0, 0)
        stream = torch.cuda.current_stream().cuda_stream
        assert L.bcm3hip_nccl_exchange(comm, 2, sends, peers, 2, recvs, peers, d + 4, stream) == 0
        torch.cuda.synchronize()
        # messages between one pair of ranks match in posting order
        assert np.array_equal(recv_prev.cpu().numpy(), last.cpu().numpy())
        assert np.array_equal(recv_next.cpu().numpy(), first.cpu().numpy())
    finally:
        L.bcm3hip_nccl_comm_destroy(comm)
