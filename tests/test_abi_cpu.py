"""The C-ABI library loads and exports every symbol include/inf_hip.h declares; the
host-only plan calls (no GPU needed) describe the reference's parameter layout."""
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "inf_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(inf_[a-z_]+)\s*\(", text)))


def test_header_parses():
    names = declared_functions()
    assert "inf_gather" in names and "inf_train_step" in names and len(names) >= 15


def test_library_exports_every_declared_symbol():
    import inf_hip
    for name in declared_functions():
        assert hasattr(inf_hip.lib, name), name
        assert name in inf_hip.EXPORTED, f"{name} has no ctypes signature"
    assert inf_hip.lib.inf_abi_version() == 3


def reference_layout(k, H, L, s):
    shapes = []
    for i in range(L):
        if i == s:
            shapes += [(H, H), (H,), (H, k), (H,)]
        elif i == L - 1:
            shapes += [(3, H), (3,)]
        else:
            shapes += [(H, k if i == 0 else H), (H,)]
    return shapes


@pytest.mark.parametrize("k,H,L,s", [(64, 128, 4, 2), (1023, 128, 6, 3), (1024, 256, 8, 4), (4096, 256, 8, 4),
                                     (37, 64, 3, 1)])
def test_plan_layout_matches_model_parameters(k, H, L, s):
    import ctypes
    import inf_hip
    from inf_hip import MlpDesc, PlanInfo
    desc = MlpDesc(k, H, L, s, 3, inf_hip.MODE_BF16, inf_hip.LOSS_L2)
    h = ctypes.c_void_p()
    inf_hip.check(inf_hip.lib.inf_plan_create(ctypes.byref(desc), 4096, ctypes.byref(h)))
    try:
        info = PlanInfo()
        inf_hip.check(inf_hip.lib.inf_plan_get_info(h, ctypes.byref(info)))
        shapes = reference_layout(k, H, L, s)
        n = len(shapes)
        assert info.num_segments == n
        offs, nums = (ctypes.c_int64 * n)(), (ctypes.c_int64 * n)()
        inf_hip.check(inf_hip.lib.inf_plan_param_layout(h, offs, nums, n))
        o = 0
        for i, shp in enumerate(shapes):
            size = 1
            for d in shp:
                size *= d
            assert offs[i] == o and nums[i] == size
            o += size
        assert info.num_params == o
        assert info.in_pad % 128 == 0 and info.in_pad >= k
        assert info.workspace_bytes > 0 and info.shadow_bytes > 0
        from model import TextureField
        m = TextureField(L, k, H, s)
        assert [tuple(p.shape) for p in m.parameters()] == [tuple(x) for x in shapes]
    finally:
        inf_hip.lib.inf_plan_destroy(h)


@pytest.mark.parametrize("bad", [dict(L=2, s=1), dict(L=4, s=0), dict(L=4, s=3), dict(H=100), dict(out=4)])
def test_plan_rejects_invalid_architectures(bad):
    import ctypes
    import inf_hip
    from inf_hip import MlpDesc
    d = dict(k=64, H=128, L=4, s=2, out=3)
    d.update(bad)
    desc = MlpDesc(d["k"], d["H"], d["L"], d["s"], d["out"], 0, 0)
    h = ctypes.c_void_p()
    rc = inf_hip.lib.inf_plan_create(ctypes.byref(desc), 64, ctypes.byref(h))
    assert rc == -1
    assert b"invalid argument" in inf_hip.lib.inf_last_error()


def test_ctrl_layout_matches_header():
    """inf_ctrl (include/inf_hip.h): the ctypes mirror's field offsets are the C layout (int32
    step / batch_index / prefetch_index / reserved, then double lr and the four sums)."""
    from inf_hip import Ctrl
    assert [(f, getattr(Ctrl, f).offset) for f, _ in Ctrl._fields_] == [
        ("step", 0), ("batch_index", 4), ("prefetch_index", 8), ("reserved", 12), ("lr", 16), ("loss_sum", 24),
        ("sse_sum", 32), ("epoch_loss", 40), ("epoch_sse", 48)]
