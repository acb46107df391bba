"""The C-ABI communicator (msat_comm_init / msat_allreduce_sum, include/marlsat_net.h) on one GPU: a
world-1 RCCL communicator through the learner's CapiComm handle.  A SUM over one rank is the identity,
so the buffers must come back bit-identical; the learner's exchange functions run over it unchanged.
Several ranks need one GPU each (RCCL refuses two ranks per device), so N > 1 over this route is
`bench.py` under torchrun with MARLSAT_COLLECTIVES=capi on a multi-GPU node (not run by these tests);
the gloo tests cover the exchange logic with world 2."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from marlsat.learners.collectives import CapiComm

    c = CapiComm(0, 1, CapiComm.unique_id())
    yield c
    c.destroy()


def test_unique_id_size_and_distinct():
    from marlsat import _lib
    from marlsat.learners.collectives import CapiComm

    a, b = CapiComm.unique_id(), CapiComm.unique_id()
    assert len(a) == len(b) == int(_lib.lib.msat_comm_id_bytes()) == 128
    assert a != b


@pytest.mark.parametrize("dtype,n", [(torch.float32, 694803), (torch.float64, 11), (torch.float32, 1)])
def test_world1_allreduce_is_identity(comm, dtype, n):
    g = torch.Generator(device="cuda").manual_seed(n)
    t = torch.randn(n, dtype=dtype, device="cuda", generator=g)
    ref = t.clone()
    comm.all_reduce(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)


def test_world1_allreduce_on_side_stream(comm):
    s = torch.cuda.Stream()
    t = torch.arange(4096, dtype=torch.float32, device="cuda")
    with torch.cuda.stream(s):
        t.mul_(3.0)
        comm.all_reduce(t)  # enqueued behind the multiply on the same stream
        t.add_(1.0)
    s.synchronize()
    assert torch.equal(t, torch.arange(4096, dtype=torch.float32, device="cuda") * 3.0 + 1.0)


def test_learner_exchange_functions_over_capi(comm):
    from marlsat.learners.collectives import allreduce_grads, allreduce_sums, global_moments

    grads = torch.randn(1000, device="cuda")
    ref = grads.clone()
    assert allreduce_grads(grads, comm) == 1.0
    assert torch.equal(grads, ref)
    sums = torch.tensor([3.0, 5.0], dtype=torch.float64, device="cuda")
    assert torch.equal(allreduce_sums(sums.clone(), comm), sums)
    mean, std = global_moments(torch.tensor([2.0, 10.0], dtype=torch.float64, device="cuda"), 4, comm)
    assert mean == 0.5 and abs(std - (10.0 / 4 - 0.25) ** 0.5 - 1e-8) < 1e-15


def test_bad_arguments_are_rejected(comm):
    from marlsat import _lib

    L = _lib.lib
    t = torch.zeros(8, device="cuda")
    assert L.msat_allreduce_sum(comm._comm, t.data_ptr(), 8, 2, _lib.stream_ptr()) == -1
    assert b"dtype" in L.msat_last_error()
    with pytest.raises(ValueError):
        comm.all_reduce(torch.zeros(8, dtype=torch.int32, device="cuda"))
    with pytest.raises(ValueError):
        comm.all_reduce(torch.zeros(8))  # host tensor
    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * 128)()
    assert L.msat_comm_init(uid, 1, 1, ctypes.byref(h)) == -1  # rank outside the world
