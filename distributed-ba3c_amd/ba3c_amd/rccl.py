"""Direct RCCL communicator for the bucketed gradient exchange.

torch's ProcessGroupNCCL runs every collective on a stream of its own: the issuing stream
hands over with an event, and work.wait() hands back with another.  The bucketed step
(trainer.py `_bucketed_sync_step`) pays those two hops per bucket on top of its own exchange
stream, and the conv bucket's hops sit on the critical path between the last backward
kernel and the update.  This module drives the same RCCL library torch loaded
(torch/lib/librccl.so, so one copy of RCCL lives in the process) through its C API, so the
sum runs on a stream we choose: the fc1 + heads bucket on the exchange stream, the conv
bucket directly on the compute stream.

The communicator is created once per (group, device) from a unique id that group rank 0
draws and broadcasts over the existing process group; every rank of the group must create
it at the same point of its program (ncclCommInitRank is collective).  Only the in-place
fp32 sum the exchange needs is bound (the reference's SyncReplicasOptimizer aggregation,
train.py:598-606, summed as multigpu.py:157 clips).
"""
import ctypes
import os

import torch
import torch.distributed as dist

NCCL_FLOAT32 = 7          # ncclDataType_t ncclFloat32 (rccl.h)
NCCL_SUM = 0              # ncclRedOp_t ncclSum


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]        # NCCL_UNIQUE_ID_BYTES


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so")
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId,
                                         ctypes.c_int]
        lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclCommAbort.argtypes = [ctypes.c_void_p]
        for fn in ("ncclCommCount", "ncclCommCuDevice", "ncclCommUserRank"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        lib.ncclGetVersion.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _LIB = lib
    return _LIB


class RcclError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise RcclError("%s failed: %s (ncclResult %d)"
                        % (what, _lib().ncclGetErrorString(rc).decode(), rc))


class RcclComm(object):
    """One RCCL communicator over the ranks of `group` (a 'nccl' process group), on `device`."""

    def __init__(self, group, device):
        lib = _lib()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device(device)
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        raw = ctypes.string_at(ctypes.addressof(uid), 128)       # all 128 bytes (NULs too)
        t = torch.tensor(list(raw), dtype=torch.uint8, device=self.device)
        root = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src=root, group=group)
        ctypes.memmove(ctypes.addressof(uid), bytes(t.cpu().tolist()), 128)
        self._comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank),
                   "ncclCommInitRank")

    def info(self):
        """What RCCL itself reports for this communicator: its rank
        count, this rank's position and the HIP device it drives, plus that device's PCI bus
        id and the RCCL version — world ranks on world distinct devices is what a multi-GPU
        line must show."""
        lib = _lib()
        out = {}
        for key, fn in (("comm_count", "ncclCommCount"), ("comm_user_rank", "ncclCommUserRank"),
                        ("comm_device", "ncclCommCuDevice")):
            v = ctypes.c_int(-1)
            _check(getattr(lib, fn)(self._comm, ctypes.byref(v)), fn)
            out[key] = v.value
        ver = ctypes.c_int(0)
        _check(lib.ncclGetVersion(ctypes.byref(ver)), "ncclGetVersion")
        out["rccl_version"] = ver.value
        props = torch.cuda.get_device_properties(out["comm_device"])
        out["pci_bus_id"] = "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0),
                                                getattr(props, "pci_bus_id", 0),
                                                getattr(props, "pci_device_id", 0))
        return out

    def selftest(self):
        """One exact in-place sum through this communicator on the caller's current stream:
        rank r contributes (r + 1) * i for i < 4096 (small integers, exact in fp32 in any
        summation order), so every element must equal i * world * (world + 1) / 2.  Returns
        True when it does (the caller makes the keep/fallback decision collectively)."""
        n = 4096
        i = torch.arange(n, dtype=torch.float32, device=self.device)
        buf = i * float(self.rank + 1)
        stream = torch.cuda.current_stream(self.device)
        self.all_reduce_sum(buf, stream)
        stream.synchronize()
        return bool(torch.equal(buf, i * float(self.world * (self.world + 1) // 2)))

    def all_reduce_sum(self, buf, stream):
        """In-place sum of the contiguous fp32 device tensor `buf` over the group, enqueued on
        `stream` (a torch.cuda.Stream); returns at once, the sum is ordered on that stream."""
        if buf.dtype != torch.float32 or not buf.is_contiguous() or buf.device != self.device:
            raise ValueError("all_reduce_sum takes a contiguous fp32 tensor on %s" % self.device)
        p = ctypes.c_void_p(buf.data_ptr())
        _check(_lib().ncclAllReduce(p, p, buf.numel(), NCCL_FLOAT32, NCCL_SUM, self._comm,
                                    ctypes.c_void_p(stream.cuda_stream)), "ncclAllReduce")

    def close(self, abort=False):
        """ncclCommDestroy (the caller has synchronised the device), or with `abort`
        ncclCommAbort, which does not wait for collectives still enqueued (exit paths: a peer
        may be dead, so outstanding work may never finish)."""
        if self._comm:
            (_lib().ncclCommAbort if abort else _lib().ncclCommDestroy)(self._comm)
            self._comm = ctypes.c_void_p()
