"""CNN engine structure on CPU (the kernels themselves run in tests/test_cnn_engine_gpu.py):
program description, stacked parameter/BN-buffer views, optimizer segments, gangs."""

import ctypes

import numpy as np
import pytest
import torch

from myfyp_amd.models import LeNet5, ResNet18
from myfyp_amd.parallel.cnn_engine import CNNEngineHandle, CNNGroup, Segment, arch_of


@pytest.mark.parametrize("cls", [LeNet5, ResNet18])
def test_group_describes_model(cls):
    m = cls(seed=1)
    g = CNNGroup(torch.device("cpu"), m, 8)
    assert g.arch == arch_of(m)
    assert g.n_params == sum(p.numel() for p in m.parameters())
    n_bn = sum(mod.num_features for mod in m.modules() if isinstance(mod, torch.nn.BatchNorm2d))
    assert g.bn_total == n_bn and g.numel == g.n_params + 2 * n_bn
    assert ctypes.sizeof(Segment) == 72
    # every trainable tensor is covered by exactly one optimizer segment
    raw = g.segs.numpy().tobytes()
    segs = (Segment * g.nseg).from_buffer_copy(raw)
    covered = sorted((s.off, s.off + s.n) for s in segs)
    assert covered[0][0] == 0 and covered[-1][1] == g.n_params
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    # the optimizer work table: one item per weight row (kind 1) / per 256-element chunk (kind 0), nothing empty
    work = g.work.numpy()
    assert g.nwork == len(work)
    for si, s in enumerate(segs):
        items = sorted(int(x) for x in work[work[:, 0] == si][:, 1])
        assert items == list(range(s.cout if s.kind == 1 else (s.n + 255) // 256))
    # Wf-layout gradient/shadow regions do not overlap
    offs = sorted((g.shadow_off[c.name], g.shadow_off[c.name] + c.cp_out * c.R * c.S * c.cp_in) for c in g.convs)
    assert all(a[1] <= b[0] for a, b in zip(offs, offs[1:])) and offs[-1][1] <= g.shadow_numel
    assert g.fit_gang is not None and g.eval_gang is not None


def test_handle_views_params_and_bn_buffers():
    m = ResNet18(seed=3)
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    g = CNNGroup(torch.device("cpu"), m, 8)
    h = CNNEngineHandle.__new__(CNNEngineHandle)
    h.addr, h.module, h.learner, h.group, h._data_id = "x", m, None, g, None
    h.slot = g.attach(h)
    h.retarget(copy_in=True)
    for k, v in m.state_dict().items():  # values preserved
        torch.testing.assert_close(v.float(), ref[k].float())
    base, end = g.params.data_ptr(), g.params.data_ptr() + g.params.numel() * 4
    assert all(base <= p.data_ptr() < end for p in m.parameters())
    assert base <= m.layers[2].shortcut[1].running_var.data_ptr() < end
    g.params[h.slot].add_(1.0)  # writes through the views
    torch.testing.assert_close(m.fc.bias, ref["fc.bias"] + 1.0)
    torch.testing.assert_close(m.bn1.running_mean, ref["bn1.running_mean"] + 1.0)
    np.testing.assert_array_equal(h.flat_params().shape, (g.n_params,))
    g.detach(h.slot)
    assert h.slot not in g.handles


def test_native_struct_layouts_match_ctypes_mirrors():
    """The kernel argument structs (ConvGemmArgs, WgradArgs, LenetArgs, Segment) have the same size and
    field offsets in the native library as in their ctypes mirrors: _lib() checks them when it binds
    the library (a mismatch would hand every conv kernel shifted arguments). The library loads
    without a GPU."""
    from myfyp_amd.ops import _native

    try:
        _native.load(required=True)
    except Exception as e:  # not built in this checkout
        pytest.skip(f"native library not built: {e}")
    from myfyp_amd.parallel.cnn_engine import _lib

    lib = _lib()
    assert lib.conv_fin_words() > 0

