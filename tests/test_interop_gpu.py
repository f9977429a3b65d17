"""GPU: the executor shares one HIP runtime with PyTorch (madrona_mi355x
imports torch first; the library is code object v5 so torch's bundled ROCm
runtime loads it), so exports land in torch tensors without a host copy, and
the C-ABI RCCL hand-off (dlopen'd, torch's RCCL) writes into torch memory.
Reference hand-off surface: src/python/bindings.cpp:78-131 (Tensor /
CudaSync), include/madrona/mw_gpu.hpp:71 (getExported)."""
import numpy as np
import pytest

import oracle_lib as ol
from test_collisions_gpu import _cfg_pair

pytestmark = pytest.mark.gpu


def _sim(W=4, N=16, steps=5):
    import madrona_mi355x as mw
    gcfg, _ = _cfg_pair(num_cubes=N)
    pos, rot = ol.gen_collisions_inits(W, N, seed=2)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    sim.step(steps)
    return mw, sim


def test_single_hip_runtime_with_torch():
    import madrona_mi355x as mw
    import torch
    assert len(mw._mapped_hip_runtimes()) == 1, mw._mapped_hip_runtimes()
    assert torch.cuda.is_available()
    x = torch.arange(16, device="cuda", dtype=torch.float32)
    assert float(x.sum()) == 120.0


def test_export_into_torch_tensor():
    import torch
    mw, sim = _sim()
    want = np.array(sim.exported_array(2, np.float32))
    t = torch.full((4,), -1.0, device="cuda")
    assert sim.copy_exported(2, t.data_ptr(), 16) == 16
    torch.cuda.synchronize()
    assert t.cpu().numpy().tobytes() == want.tobytes()


def test_rccl_single_rank_allgather_into_torch():
    import torch
    mw, sim = _sim()
    want = np.array(sim.exported_array(2, np.float32))
    sim.rccl_init(mw.rccl_unique_id(), 1, 0)
    t = torch.zeros(4, device="cuda")
    sim.allgather_exported(2, t.data_ptr(), 16)
    sim.sync()
    assert t.cpu().numpy().tobytes() == want.tobytes()


def test_exported_tensor_zero_copy_dlpack():
    """getExported -> Tensor -> to_torch aliases the executor's export buffer
    (device kDLROCM): later steps show through without another copy."""
    import torch
    from madrona_mi355x.python import HipSync, Tensor
    mw, sim = _sim()
    t = sim.exported_tensor(2, Tensor.ElementType.Float32, (4,))
    view = t.to_torch()
    assert view.is_cuda and view.data_ptr() == sim.exported(2)[0]
    assert view.cpu().numpy().tobytes() == np.array(sim.exported_array(2, np.float32)).tobytes()
    sim.step_async(3)
    HipSync(sim).wait(torch.cuda.current_stream().cuda_stream)
    after = view.clone()            # ordered after the steps on torch's stream
    torch.cuda.synchronize()
    assert after.cpu().numpy().tobytes() == np.array(sim.exported_array(2, np.float32)).tobytes()


def test_madrona_python_module_on_hip_memory():
    # The reference's import name over HIP memory: a torch tensor on the
    # device round-trips zero-copy, and CudaSync.wait orders a consumer
    # stream after the executor's enqueued steps.
    import madrona_python
    import torch
    a = torch.arange(1000, dtype=torch.int32, device="cuda")
    t = madrona_python.Tensor(a)
    assert t.is_on_gpu() and t.gpu_id() == a.device.index
    b = t.to_torch()
    assert b.device == a.device and b.data_ptr() == a.data_ptr()
    b[7] = -1
    assert int(a[7]) == -1
    _, sim = _sim()
    sim.step_async(2)
    strm = torch.cuda.Stream()
    madrona_python.CudaSync(sim).wait(strm.cuda_stream)
    with torch.cuda.stream(strm):
        ret = torch.from_numpy(sim.exported_array(2, np.float32)).to("cuda")
    strm.synchronize()
    assert ret.numel() == 4
