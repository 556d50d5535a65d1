"""The GPU run's own evidence that the HIP path ran: the in-tree
libcotix_amd.so is mapped, its kernels are gfx950 code objects, the
checkers the parity tests need are present (a missing checker fails, it
never skips), and a kernel launch through the C-ABI touches device memory."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_library_is_the_in_tree_hip_build():
    import torch
    assert torch.cuda.is_available(), "-m gpu run without a visible GPU"
    import parallax_amd as pa
    from parallax_amd import _ffi
    from conftest import loaded_native_libraries
    want = os.path.realpath(os.path.join(ROOT, "parallax_amd", "_lib", "libcotix_amd.so"))
    assert os.path.realpath(_ffi.LIB_PATH) == want
    assert want in loaded_native_libraries()
    assert "gfx950" in torch.cuda.get_device_properties(0).gcnArchName
    # a launch through the C-ABI writes device memory (no host path exists)
    k = pa.random.PRNGKey(0, "cuda")
    assert pa.random.split(k).cpu().numpy().view(np.uint32).tolist() == [[4146024105, 967050713],
                                                                          [2718843009, 1272950319]]
    with open(want, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob, "no gfx950 code object in the library"


def test_checkers_present():
    from cotix_oracle import cport
    assert os.path.exists(cport.LIB), cport.LIB
    assert os.path.exists(os.path.join(ROOT, "tests", "emu", "build", "libcotix_emu.so"))
