"""Python tensor surface of the reference's nanobind module ``madrona_python``
(include/madrona/python.hpp:17-80, src/python/bindings.cpp:24-131): a
``Tensor`` describing device (or host) memory by pointer, element type and
dimensions, convertible to torch zero-copy through DLPack, and a stream sync
object.  DLPack structs are built with ctypes (ABI of dlpack.h v0.8), device
type kDLROCM for HIP memory.

    t = sim.exported_tensor(0, Tensor.ElementType.Float32, (num_worlds, 3))
    obs = t.to_torch()                       # aliases the executor's buffer
    sim.wait_on(torch.cuda.current_stream().cuda_stream)
"""
import ctypes
import enum

__all__ = ["Tensor", "HipSync", "CudaSync"]

_KDL_CPU = 1
_KDL_ROCM = 10
_KDL_INT, _KDL_UINT, _KDL_FLOAT = 0, 1, 2


class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p),
                             ("deleter", _DELETER)]

# Managed tensors handed to a consumer stay alive (with their owner, e.g. the
# executor) until the consumer calls the deleter.
_LIVE = {}


@_DELETER
def _release(mt):
    _LIVE.pop(ctypes.addressof(mt.contents), None)


_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


class Tensor:
    """Reference madrona::py::Tensor: (pointer, ElementType, dims, gpu id)."""

    class ElementType(enum.Enum):      # python.hpp:41-49, same order
        UInt8 = 0
        Int8 = 1
        Int16 = 2
        Int32 = 3
        Int64 = 4
        Float16 = 5
        Float32 = 6

    _DL = {ElementType.UInt8: (_KDL_UINT, 8), ElementType.Int8: (_KDL_INT, 8),
           ElementType.Int16: (_KDL_INT, 16), ElementType.Int32: (_KDL_INT, 32),
           ElementType.Int64: (_KDL_INT, 64), ElementType.Float16: (_KDL_FLOAT, 16),
           ElementType.Float32: (_KDL_FLOAT, 32)}
    max_dimensions = 16                # python.hpp:66

    def __init__(self, torch_tensor):
        """Wrap a torch tensor (bindings.cpp:80-106): contiguous, of one of
        the ElementTypes, on the CPU or a HIP device."""
        import torch
        types = {torch.uint8: "UInt8", torch.int8: "Int8", torch.int16: "Int16",
                 torch.int32: "Int32", torch.int64: "Int64", torch.float16: "Float16",
                 torch.float32: "Float32"}
        if torch_tensor.dtype not in types:
            raise TypeError(f"Tensor: invalid tensor dtype {torch_tensor.dtype}")
        if not torch_tensor.is_contiguous():
            raise ValueError("Tensor: tensor must be contiguous")
        if torch_tensor.dim() > self.max_dimensions:
            raise ValueError(f"Cannot construct Tensor with more than {self.max_dimensions} dimensions")
        if torch_tensor.device.type not in ("cpu", "cuda"):
            raise ValueError("madrona::Tensor: failed to import unknown tensor type")
        gpu = torch_tensor.device.index if torch_tensor.device.type == "cuda" else None
        self._init(torch_tensor.data_ptr(), Tensor.ElementType[types[torch_tensor.dtype]],
                   tuple(torch_tensor.shape), gpu, torch_tensor)

    @classmethod
    def from_device_ptr(cls, ptr, element_type, dims, gpu_id=None, owner=None):
        t = cls.__new__(cls)
        t._init(ptr, element_type, tuple(int(d) for d in dims), gpu_id, owner)
        return t

    def _init(self, ptr, element_type, dims, gpu_id, owner):
        if len(dims) > self.max_dimensions:
            raise ValueError(f"Cannot construct Tensor with more than {self.max_dimensions} dimensions")
        self._ptr = int(ptr)
        self._type = Tensor.ElementType(element_type)
        self._dims = dims
        self._gpu = -1 if gpu_id is None else int(gpu_id)
        self._owner = owner

    def device_ptr(self):
        return self._ptr

    def type(self):
        return self._type

    def is_on_gpu(self):
        return self._gpu != -1

    def gpu_id(self):
        return self._gpu

    def dims(self):
        return self._dims

    # DLPack producer protocol -------------------------------------------------
    def __dlpack_device__(self):
        return (_KDL_ROCM, self._gpu) if self._gpu != -1 else (_KDL_CPU, 0)

    def __dlpack__(self, stream=None, **_):
        n = len(self._dims)
        shape = (ctypes.c_int64 * max(n, 1))(*self._dims)
        code, bits = self._DL[self._type]
        mt = _DLManagedTensor()
        dev_type, dev_id = self.__dlpack_device__()
        mt.dl_tensor = _DLTensor(ctypes.c_void_p(self._ptr), _DLDevice(dev_type, dev_id), n,
                                 _DLDataType(code, bits, 1), shape, None, 0)
        mt.deleter = _release
        _LIVE[ctypes.addressof(mt)] = (mt, shape, self._owner)
        return _PyCapsule_New(ctypes.addressof(mt), b"dltensor", None)

    def to_torch(self):
        """Zero-copy torch tensor over the same memory (bindings.cpp:108-125)."""
        import torch
        return torch.from_dlpack(self)


class HipSync:
    """Reference CudaSync (python.hpp:20-35): ``wait(stream)`` orders a
    consumer stream after the executor's enqueued steps, on the device."""

    def __init__(self, executor):
        self._exec = executor

    def wait(self, strm):
        self._exec.wait_on(int(strm))


CudaSync = HipSync
