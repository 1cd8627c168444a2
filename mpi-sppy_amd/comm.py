"""Communicators for the PH engine (restates the role of ``mpisppy/MPI.py:10-90``).

The reference moves per-node xbar sums and the convergence partials with mpi4py ``Allreduce``
(``phbase.py:88-92, :369``; ``spopt.py:372, 417, 435, 466``).  Here one process drives one GPU and
the same SUM reductions run through ``torch.distributed``: backend ``nccl`` (= RCCL over xGMI on
ROCm) on device tensors, ``gloo`` on host tensors (CPU tests).  ``SingleComm`` is the 1-rank mock
(the reference's fallback when mpi4py is absent, ``MPI.py:14-90``).
"""
import numpy as np


class SingleComm:
    rank = 0
    size = 1

    def Get_rank(self):
        return 0

    def Get_size(self):
        return 1

    def allreduce_sum_(self, t):
        return t

    def allreduce_scalar(self, v):
        return float(v)

    def allreduce_array(self, a):
        return np.asarray(a, dtype=np.float64)

    def barrier(self):
        pass

    Barrier = barrier

    def bcast_object(self, obj, root=0):
        return obj

    def gather_object(self, obj, root=0):
        return [obj]

    def allgather_object(self, obj):
        return [obj]

    def exchange_path(self):
        """(what carries the per-iteration device exchange, ranks the collective library counts)"""
        return "none (one rank: nothing to exchange)", None


class TorchComm:
    """SUM all-reduces over an initialised ``torch.distributed`` process group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("TorchComm needs torch.distributed.init_process_group first")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def allreduce_sum_(self, t):
        """In-place SUM of a torch tensor (device tensor under nccl/RCCL, host under gloo)."""
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t

    def _scratch(self, a):
        import torch
        dev = "cuda" if self.backend == "nccl" else "cpu"
        return torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dev)

    def allreduce_array(self, a):
        t = self._scratch(a)
        self.allreduce_sum_(t)
        return t.cpu().numpy()

    def allreduce_scalar(self, v):
        return float(self.allreduce_array(np.array([v]))[0])

    def barrier(self):
        self.dist.barrier(group=self.group)

    Barrier = barrier

    def bcast_object(self, obj, root=0):
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=root, group=self.group)
        return lst[0]

    def gather_object(self, obj, root=0):
        """Pickled objects of every rank, in rank order, on ``root`` (None elsewhere): the
        ``comm.gather`` of the reference's file writers (control data only, never the data path)."""
        out = [None] * self.size
        self.dist.all_gather_object(out, obj, group=self.group)
        return out if self.rank == root else None

    def allgather_object(self, obj):
        """Pickled objects of every rank, in rank order, on every rank (setup-time control data)."""
        out = [None] * self.size
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def exchange_path(self):
        """(path, ranks): under nccl the device all-reduce is RCCL's, over the process group's ranks;
        gloo stages through host memory (tests put several ranks on one device with it)."""
        if self.backend == "nccl":
            return "torch.distributed nccl (RCCL)", self.dist.get_world_size(self.group)
        return f"torch.distributed {self.backend} (host-staged)", None


def _device_count():
    """Visible HIP devices, without initialising one (torch's count does not, on this image)."""
    try:
        import torch
        return torch.cuda.device_count()
    except ImportError:
        return 1 << 30


class PhgGroupComm:
    """Device all-reduces through libphg.so's own RCCL communicator (``phg_create_group``,
    include/phg.h), everything else through ``host`` (any communicator of this module).

    This is the pure C-ABI multi-GPU path: what a reference-side integration with mpi4py would use
    instead of torch.distributed -- rank 0 makes the 128-byte group id, ``host``
    broadcasts it, every rank joins with its own device.  The PH exchange buffer (a device tensor)
    is summed by ``phg_group_allreduce`` on the engine's stream; ``PHBase`` hands the engine's handle
    over once the engine exists (``attach``)."""

    def __init__(self, host, device):
        from . import _lib
        self.host = host
        self.rank, self.size = host.Get_rank(), host.Get_size()
        # ncclCommInitRank is collective and blocking: a rank that fails BEFORE its call (library
        # load, device, the id) would leave its peers inside it.  So the steps up to the call are
        # agreed first through ``host``: every rank reports, and all proceed or all raise.  (The call
        # itself is non-blocking with a deadline in libphg, PHG_GROUP_TIMEOUT.)
        uid, err, ok = None, None, True
        try:
            _lib.load()
            if not 0 <= int(device) < _device_count():
                raise RuntimeError(f"device {device} not present")
            if self.rank == 0:
                uid = _lib.PhgGroup.unique_id()
        except Exception as e:    # every rank still joins the broadcast and the vote
            ok, err = False, e
        uid = host.bcast_object(uid, root=0)
        ok = ok and isinstance(uid, (bytes, bytearray)) and len(uid) == 128
        n_ok = host.allreduce_scalar(1.0 if ok else 0.0) if self.size > 1 else (1.0 if ok else 0.0)
        if n_ok != self.size:
            if uid is None and err is None:
                err = "phg_group_unique_id failed on rank 0"
            raise RuntimeError(f"libphg RCCL group: set-up failed on {self.size - int(n_ok)} rank(s) before "
                               f"ncclCommInitRank{f': {err}' if err else ''}")
        self.group = _lib.PhgGroup(self.size, self.rank, uid, device)
        self.handle = None

    def attach(self, engine):
        self.handle = engine.h

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def allreduce_sum_(self, t):
        if getattr(t, "is_cuda", False):
            if self.handle is None:
                raise RuntimeError("PhgGroupComm: no engine attached (PHBase attaches its engine)")
            self.group.allreduce(self.handle, t.data_ptr(), t.numel())
            return t
        return self.host.allreduce_sum_(t)

    def close(self):
        self.group.close()

    def exchange_path(self):
        """(path, ranks): the ranks are RCCL's own count of the communicator (ncclCommCount through
        phg_group_size), not the arguments it was created with."""
        n, r = self.group.size()
        if r != self.rank:
            raise RuntimeError(f"libphg RCCL group: RCCL places this process at rank {r}, the host at {self.rank}")
        return "libphg RCCL group (phg_group_allreduce)", n

    def __getattr__(self, name):   # host-side collectives (arrays, scalars, objects, barrier)
        return getattr(self.host, name)


def group_or_host(host, device, log=None):
    """``PhgGroupComm(host, device)`` when every rank creates the library group, else ``host``
    on every rank: each rank reports whether its ``phg_create_group`` succeeded and the ranks agree
    through ``host`` (one scalar SUM), so no rank is left on a different exchange path than the
    others.  The fallback is the same device all-reduce through torch.distributed's RCCL, not a CPU
    path; ``log`` (a callable) receives the reason."""
    from ._lib import PhgError
    comm, err = None, None
    try:
        comm = PhgGroupComm(host, device)
    except (PhgError, OSError, RuntimeError) as e:
        err = e
    n_ok = host.allreduce_scalar(1.0 if comm is not None else 0.0)
    if n_ok == host.Get_size():
        return comm
    if comm is not None:
        comm.close()
    if log is not None:
        log(f"libphg RCCL group not created on {host.Get_size() - int(n_ok)} rank(s)"
            + (f" ({err})" if err is not None else "") + "; exchange through torch.distributed")
    return host


def rank_report(comm, device=None):
    """Evidence of who carried the multi-GPU exchange, for the bench line: the
    exchange path and its collective's own rank count, and every rank's device and PCI bus id
    (gathered through ``comm``; reference: the Allreduces of ``phbase.py:88-92, 369`` and their
    communicator, ``spbase.py``'s ``mpicomm``)."""
    me = {"rank": comm.Get_rank(), "device": device, "pci_bus_id": None, "device_name": None}
    if device is not None:
        try:
            import torch
            pr = torch.cuda.get_device_properties(device)
            me["pci_bus_id"] = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
            me["device_name"] = pr.name
        except Exception:
            pass
    try:
        import socket
        me["host"] = socket.gethostname()
    except Exception:
        me["host"] = None
    ranks = comm.allgather_object(me) if comm.Get_size() > 1 else [me]
    path, n = comm.exchange_path()
    return {"world_size": comm.Get_size(), "exchange_path": path, "collective_ranks": n,
            "distinct_devices": len({(r["host"], r["pci_bus_id"] or r["device"]) for r in ranks}),
            "ranks": ranks}
