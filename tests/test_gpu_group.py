"""The library's own RCCL group (include/phg.h: phg_group_unique_id / phg_create_group /
phg_group_allreduce / phg_ph_exchange; SURVEY 8(b) phg_create_group), the C-ABI multi-GPU path a
reference-side integration with mpi4py would use instead of torch.distributed.

One GPU per box here, so the group has one rank (RCCL refuses two ranks on one device): the
all-reduce is then an in-place identity, and what is checked is the whole path -- group creation,
the reduction on the handle's stream, PHBase's exchange path (node sums -> exchange -> gated W
update -> solve) driven through ``comm.PhgGroupComm`` -- against the single-GPU PH, bit for bit.
Multi-rank runs of the same exchange go through torch.distributed (tests/test_gpu_dist.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.comm import PhgGroupComm, SingleComm  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def _opts(**kw):
    o = {"solver_name": "phg", "PHIterLimit": 60, "defaultPHrho": 1.0, "convthresh": 1e-10,
         "verbose": False, "display_progress": False}
    o.update(kw)
    return o


def test_group_create_and_allreduce():
    torch.cuda.set_device(0)
    uid = _lib.PhgGroup.unique_id()
    assert len(uid) == 128
    g = _lib.PhgGroup(1, 0, uid, 0)
    lib = _lib.load()
    out = np.zeros(2, np.int32)
    _lib.check(lib.phg_group_size(g.g, out.ctypes.data_as(_lib.i32p)))
    assert out.tolist() == [1, 0]
    # a handle for the stream: a tiny farmer batch
    ph = PH(_opts(), farmer.scenario_names_creator(3), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": 3})
    ph.PH_Prep()
    t = torch.arange(1000, dtype=torch.float64, device="cuda") * 0.5 + 1.0 / 3.0
    ref = t.clone()
    g.allreduce(ph.engine.h, t.data_ptr(), t.numel())
    torch.cuda.synchronize()
    assert torch.equal(t, ref)   # one rank: the SUM is the identity, bit for bit
    with pytest.raises(_lib.PhgError):
        g.allreduce(ph.engine.h, t.data_ptr(), -1)
    g.close()


@pytest.mark.parametrize("pipe", [True, False])
def test_ph_through_library_group_matches_single_gpu(pipe):
    """PH farmer (cm=2, 8 scenarios) with the packed exchange routed through the library's RCCL
    group (pdhg_exchange=True on one rank, comm.PhgGroupComm) vs the single-GPU path (no exchange):
    the same PH iterations, conv history, W, x-bar and nonants, bit for bit -- pipelined
    (phg_node_sums -> phg_group_allreduce -> phg_ph_head) and sequential (Compute_Xbar /
    Update_W / convergence_diff)."""
    torch.cuda.set_device(0)
    out = []
    for grp in (True, False):
        comm = PhgGroupComm(SingleComm(), 0) if grp else None
        ph = PH(_opts(pdhg_exchange=grp, pdhg_pipeline=pipe, convthresh=1e-3, PHIterLimit=300),
                farmer.scenario_names_creator(8), farmer.scenario_creator, mpicomm=comm,
                scenario_creator_kwargs={"crops_multiplier": 2, "num_scens": 8})
        conv, eobj, tb = ph.ph_main()
        if grp:
            assert ph.engine.exchange is not None
        out.append((ph._PHIter, conv, eobj, tb, list(ph.conv_history), ph.Ws().copy(), ph.xbars().copy(),
                    ph.nonants().copy()))
        if comm is not None:
            comm.close()
    (i1, c1, e1, t1, h1, W1, x1, n1), (i0, c0, e0, t0, h0, W0, x0, n0) = out
    assert i1 == i0 < 300 and c1 < 1e-3
    assert (c1, e1, t1) == (c0, e0, t0) and h1 == h0
    assert np.array_equal(W1, W0) and np.array_equal(x1, x0) and np.array_equal(n1, n0)
