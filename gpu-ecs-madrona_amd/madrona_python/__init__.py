"""``madrona_python``: the import name of the reference's nanobind module
(``NB_MODULE(madrona_python, m)``, src/python/bindings.cpp:78-128), so a
reference-side script runs unchanged:

    import madrona_python
    t = madrona_python.Tensor(torch_tensor)     # bindings.cpp:80-107
    v = t.to_torch()                            # bindings.cpp:108-123, zero-copy
    sync.wait(stream)                           # CudaSync::wait, bindings.cpp:126-127

Both classes are the framework's own (madrona_mi355x.python: DLPack views
with device type kDLROCM for HIP memory, ``CudaSync`` = ``HipSync`` over
``mw_stream_wait``); importing this module loads the framework (and with it
the gfx950 library), exactly as importing the reference module loads its
executor.
"""
from madrona_mi355x.python import CudaSync, HipSync, Tensor

__all__ = ["Tensor", "CudaSync", "HipSync"]
