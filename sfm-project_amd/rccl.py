"""A direct RCCL communicator for the sharded bundle-adjustment solve.

The sharded Schur-complement PCG (sfm_ba_solve_stage) needs one in-place fp64 sum of
8·n_cam doubles per CG iteration, between two kernels on the compute stream.  Going through
torch.distributed's ProcessGroupNCCL puts that collective on RCCL's side stream behind two
cross-queue event waits: ≈10 µs of idle GPU per iteration at 500 cameras, longer than the
collective itself (profiles/r03/ba_sharded_ab.txt).  This module opens its own RCCL
communicator over the same ranks (the unique id travels through the torch.distributed group)
and issues ncclAllReduce straight on the caller's current HIP stream, so the collective is one
more entry in the stream, in order with the CG kernels (and capturable in a HIP graph).

RCCL is torch's own librccl.so (the one ProcessGroupNCCL already loaded), bound with ctypes:
ncclGetUniqueId / ncclCommInitRank / ncclAllReduce(ncclFloat64, ncclSum) / ncclCommDestroy.
"""
import ctypes as C
import os

_NCCL_FLOAT64 = 8
_NCCL_SUM = 0
_lib = None


class _UniqueId(C.Structure):
    _fields_ = [("internal", C.c_ubyte * 128)]  # opaque; bytes(uid) is all 128


def _load():
    global _lib
    if _lib is None:
        import torch
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = C.CDLL(path)
        lib.ncclGetUniqueId.argtypes = [C.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _UniqueId, C.c_int]
        lib.ncclAllReduce.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int,
                                      C.c_void_p, C.c_void_p]
        lib.ncclCommDestroy.argtypes = [C.c_void_p]
        lib.ncclGetErrorString.argtypes = [C.c_int]
        lib.ncclGetErrorString.restype = C.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy"):
            getattr(lib, f).restype = C.c_int
        _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {_lib.ncclGetErrorString(rc).decode()} (ncclResult {rc})")


class RcclComm:
    """RCCL communicator over the ranks of a torch.distributed group (collective to create:
    every rank of the group constructs it at the same point) on GPU `device` (default: the
    current device).  Each rank passes its OWN device (one process per GPU, every GPU visible:
    device = local rank), so the id broadcast, ncclCommInitRank and every collective run on that
    GPU.  `allreduce_(t)` sums the contiguous fp64 device tensor t (on that GPU) over the ranks
    in place, on the current stream of t's device."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        lib = _load()
        self._torch = torch
        self.comm = None
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                           (device.index if isinstance(device, torch.device) else int(device)))
        self.device = dev.index
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        box = [bytes(uid) if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        with torch.cuda.device(dev):
            # the object broadcast stages through this rank's GPU (nccl groups), not GPU 0
            dist.broadcast_object_list(box, src=src, group=group,
                                       device=dev if dist.get_backend(group) == "nccl" else None)
            uid = _UniqueId.from_buffer_copy(box[0])
            comm = C.c_void_p()
            _check(lib.ncclCommInitRank(C.byref(comm), self.world, uid, self.rank),
                   "ncclCommInitRank")
        self.comm = comm

    def allreduce_(self, t):
        torch = self._torch
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.allreduce_: contiguous float64 device tensor required")
        if t.device.index != self.device:
            raise ValueError(f"RcclComm.allreduce_: tensor on cuda:{t.device.index}, communicator "
                             f"on cuda:{self.device}")
        if self.comm is None:
            raise RuntimeError("RcclComm.allreduce_: communicator is closed")
        s = torch.cuda.current_stream(t.device).cuda_stream
        _check(_lib.ncclAllReduce(C.c_void_p(t.data_ptr()), C.c_void_p(t.data_ptr()), t.numel(),
                                  _NCCL_FLOAT64, _NCCL_SUM, self.comm, C.c_void_p(s)),
               "ncclAllReduce")

    def close(self):
        if self.comm is not None:
            self._torch.cuda.synchronize(self.device)
            _check(_lib.ncclCommDestroy(self.comm), "ncclCommDestroy")
            self.comm = None
