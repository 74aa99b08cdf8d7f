"""CPU reference path of the fused ops (the GPU kernels are checked against the same math in
test_kernels_gpu.py)."""

import pytest
import torch

from myfyp_amd import ops


def test_adam_reference_matches_torch():
    p0 = torch.randn(1000)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-2)
    p, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    for t in range(1, 6):
        g = torch.randn(1000)
        p_ref.grad = g.clone()
        opt.step()
        ops.adam_step(p, g, m, v, t, lr=1e-2)
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)


def test_sgd_reference_matches_torch():
    p0 = torch.randn(100)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.SGD([p_ref], lr=0.1, momentum=0.9, weight_decay=1e-3)
    p, buf = p0.clone(), torch.zeros(100)
    for _ in range(4):
        g = torch.randn(100)
        p_ref.grad = g.clone()
        opt.step()
        ops.sgd_step(p, g, buf, lr=0.1, momentum=0.9, weight_decay=1e-3)
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)


def test_reductions_reference():
    a, b = torch.randn(10), torch.randn(10)
    out = ops.weighted_average([[a], [b]], [0.25, 0.75])[0]
    torch.testing.assert_close(out, 0.25 * a + 0.75 * b)
    st = torch.stack([a, b])
    res = torch.empty(10)
    ops.stacked_weighted_sum(st, torch.tensor([1.0, 2.0]), res, 0.5)
    torch.testing.assert_close(res, 0.5 * (a + 2 * b))
    ops.broadcast_rows(res, st, torch.tensor([0.0, 1.0]))
    torch.testing.assert_close(st[1], res)
    med = ops.coordinate_median([[a], [b], [a + b]])[0]
    torch.testing.assert_close(med, torch.median(torch.stack([a, b, a + b]), 0).values)
    t = a.clone()
    ops.scale_add_noise(t, -1.0, 0.0)
    torch.testing.assert_close(t, -a)


@pytest.mark.parametrize("n", [1, 2, 7, 64, 1000, 7500])
def test_epoch_feistel_permutation_is_bijective(n):
    """The fused engine draws each peer's epoch order on the device with a keyed Feistel
    permutation; its host mirror must be a bijection of [0, n) and differ between keys."""
    from myfyp_amd.parallel.mlp_engine import feistel_perm

    for key in (0, 0x1234_5678_9ABC_DEF0):
        perm = [feistel_perm(i, n, key) for i in range(n)]
        assert sorted(perm) == list(range(n))
    if n >= 64:
        a = [feistel_perm(i, n, 1) for i in range(n)]
        b = [feistel_perm(i, n, 2) for i in range(n)]
        assert a != b and a != list(range(n))
