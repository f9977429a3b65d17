"""CPU: the madrona_python-compatible Tensor (madrona_mi355x.python) --
reference include/madrona/python.hpp:38-80, src/python/bindings.cpp:24-125:
construction from a torch tensor, element-type mapping, dims limit, and
zero-copy DLPack round trips (host memory here; HIP memory in
test_interop_gpu.py)."""
import gc

import pytest
import torch

from madrona_mi355x import python as mp
from madrona_mi355x.python import Tensor


@pytest.mark.parametrize("dtype,et", [(torch.uint8, "UInt8"), (torch.int8, "Int8"),
                                      (torch.int16, "Int16"), (torch.int32, "Int32"),
                                      (torch.int64, "Int64"), (torch.float16, "Float16"),
                                      (torch.float32, "Float32")])
def test_roundtrip_aliases_memory(dtype, et):
    a = torch.arange(24).to(dtype).reshape(2, 3, 4)
    t = Tensor(a)
    assert t.type() == Tensor.ElementType[et] and t.dims() == (2, 3, 4) and not t.is_on_gpu()
    b = t.to_torch()
    assert b.dtype == dtype and tuple(b.shape) == (2, 3, 4) and b.data_ptr() == a.data_ptr()
    b[1, 2, 3] = 7
    assert int(a[1, 2, 3]) == 7


def test_rejects_what_the_reference_rejects():
    with pytest.raises(TypeError):
        Tensor(torch.zeros(3, dtype=torch.float64))
    with pytest.raises(ValueError):
        Tensor.from_device_ptr(0, Tensor.ElementType.Int32, (1,) * 17)


def test_pointer_view_and_deleter_release():
    a = torch.arange(8, dtype=torch.int32)
    t = Tensor.from_device_ptr(a.data_ptr(), Tensor.ElementType.Int32, (2, 4), owner=a)
    v = t.to_torch()
    assert v.tolist() == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert len(mp._LIVE) >= 1
    del v
    gc.collect()
    assert len(mp._LIVE) == 0


def test_madrona_python_import_name():
    # A reference-side script: import madrona_python, Tensor(t).to_torch()
    # (src/python/bindings.cpp:78-123), CudaSync present (:126-127).
    import madrona_python
    a = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    b = madrona_python.Tensor(a).to_torch()
    assert b.data_ptr() == a.data_ptr() and torch.equal(a, b)
    assert hasattr(madrona_python.CudaSync, "wait")
    assert madrona_python.Tensor is Tensor
