"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references (MI355X only)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from myfyp_amd.ops import _native

    _native.load(required=True)  # the native path must be the one under test
    return torch.device("cuda")


@pytest.fixture
def bf16_engine():
    """The bf16-operand MLP engine (persistent + 3-launch step paths); fp32 is tests/test_mlp_f32_gpu.py."""
    from myfyp_amd.settings import Settings

    old = Settings.MLP_PRECISION
    Settings.MLP_PRECISION = "bf16"
    yield
    Settings.MLP_PRECISION = old


def test_weighted_average(dev):
    from myfyp_amd import ops

    g = torch.Generator(device="cpu").manual_seed(0)
    models = [[torch.randn(37, 13, generator=g).to(dev), torch.randn(1001, generator=g).to(dev)] for _ in range(5)]
    w = [0.1, 0.2, 0.3, 0.15, 0.25]
    out = ops.weighted_average(models, w)
    for layer in range(2):
        ref = sum(wi * m[layer].double() for wi, m in zip(w, models))
        torch.testing.assert_close(out[layer].double(), ref, rtol=1e-5, atol=1e-5)


def test_stacked_sum_and_broadcast(dev):
    from myfyp_amd import ops

    P, N, ld = 6, 5003, 5056
    st = torch.randn(P, ld, device=dev)
    w = torch.tensor([1.0, 0.0, 2.0, 3.0, 0.0, 0.5], device=dev)
    out = torch.empty(N, device=dev)
    ops.stacked_weighted_sum(st[:, :N], w, out, scale=0.25)
    ref = (w.view(-1, 1) * st[:, :N]).sum(0) * 0.25
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    mask = torch.tensor([1, 0, 1, 0, 1, 1], dtype=torch.float32, device=dev)
    before = st.clone()
    ops.broadcast_rows(out, st[:, :N], mask)
    for p in range(P):
        if mask[p] != 0:
            torch.testing.assert_close(st[p, :N], out)
        else:
            torch.testing.assert_close(st[p], before[p])


@pytest.mark.parametrize("N,ld", [(235146, 235200), (5003, 5005)])
def test_fedavg_stacked_local_and_split(dev, N, ld):
    """Single-rank FedAvg in one kernel == reduce + apply (the multi-rank form) == torch."""
    from myfyp_amd import ops

    P = 8
    st = torch.randn(P, ld, device=dev)
    w = np.array([3, 0, 1, 2, 5, 0, 4, 1], dtype=np.float32)
    mask = np.array([1, 1, 1, 0, 1, 1, 1, 0], dtype=np.float32)
    ref = (torch.from_numpy(w).to(dev).view(-1, 1) * st[:, :N]).sum(0) / float(w.sum())
    fast = ops.fast_lib()
    stream = torch.cuda.current_stream().cuda_stream
    a = st.clone()
    ops.check(fast.myfyp_fedavg_stacked_local(a.data_ptr(), P, N, ld, w.ctypes.data, mask.ctypes.data, stream), "local")
    b = st.clone()
    buf = torch.empty(N + 1, device=dev)
    ops.check(fast.myfyp_fedavg_stacked_reduce(buf.data_ptr(), b.data_ptr(), P, N, ld, w.ctypes.data, stream), "reduce")
    ops.check(fast.myfyp_fedavg_stacked_apply(b.data_ptr(), buf.data_ptr(), P, N, ld, mask.ctypes.data, stream), "apply")
    torch.cuda.synchronize()
    for p in range(P):
        if mask[p]:
            torch.testing.assert_close(a[p, :N], ref, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(b[p, :N], ref, rtol=1e-5, atol=1e-5)
        else:
            torch.testing.assert_close(a[p], st[p])
            torch.testing.assert_close(b[p], st[p])
        torch.testing.assert_close(a[p, N:], st[p, N:])  # padding untouched


@pytest.mark.parametrize("P", [3, 8, 16])
def test_neighbor_mix_stacked(dev, P):
    """In-place topology mixing of stacked rows == M @ rows in torch (ring + an idle row + a dead
    neighbour renormalised away)."""
    from myfyp_amd import ops

    N, ld = 62006, 62016
    st = torch.randn(P, ld, device=dev)
    m = np.zeros((P, P), dtype=np.float32)
    for p in range(P):
        for q in {p, (p - 1) % P, (p + 1) % P}:
            m[p, q] = 1.0
    m[P - 1] = 0.0  # an idle row is left alone
    if P > 3:
        m[:, 2] = 0.0  # peer 2 died: nobody reads it
        m[2, 2] = 1.0
    m = m / np.maximum(m.sum(1, keepdims=True), 1e-12)
    m[P - 1] = 0.0
    ref = torch.from_numpy(m).to(dev).double() @ st.double()
    a = st.clone()
    ops.check(ops.fast_lib().myfyp_neighbor_mix_stacked(a.data_ptr(), P, N, ld, m.ctypes.data, torch.cuda.current_stream().cuda_stream), "mix")
    torch.cuda.synchronize()
    for p in range(P - 1):
        torch.testing.assert_close(a[p, :N].double(), ref[p, :N], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(a[P - 1], st[P - 1])
    bad = np.ones((17, 17), dtype=np.float32)
    assert ops.fast_lib().myfyp_neighbor_mix_stacked(a.data_ptr(), 17, N, ld, bad.ctypes.data, torch.cuda.current_stream().cuda_stream) == 2


@pytest.mark.parametrize("P", [10, 16])
def test_neighbor_mix_stacked_full_topology(dev, P):
    """Full / star topologies give a row more than 8 sources (Metropolis weights keep w_ii > 0):
    the single-kernel mix must accept every local peer as a source."""
    from myfyp_amd import ops

    N, ld = 4099, 4100
    st = torch.randn(P, ld, device=dev)
    m = np.full((P, P), 1.0 / P, dtype=np.float32)
    ref = torch.from_numpy(m).to(dev).double() @ st.double()
    a = st.clone()
    ops.check(ops.fast_lib().myfyp_neighbor_mix_stacked(a.data_ptr(), P, N, ld, m.ctypes.data, torch.cuda.current_stream().cuda_stream), "mix")
    torch.cuda.synchronize()
    torch.testing.assert_close(a[:, :N].double(), ref[:, :N], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("k", [1, 2, 5, 8, 16])
def test_coordinate_median(dev, k):
    from myfyp_amd import ops

    models = [[torch.randn(3001, device=dev)] for _ in range(k)]
    out = ops.coordinate_median(models)[0]
    st = torch.stack([m[0] for m in models])
    s, _ = torch.sort(st, 0)
    ref = s[(k - 1) // 2] if k % 2 else 0.5 * (s[k // 2 - 1] + s[k // 2])
    torch.testing.assert_close(out, ref)


@pytest.mark.parametrize("steps", [1, 7])
def test_adam_matches_torch(dev, steps):
    from myfyp_amd import ops

    n = 10_007
    p0 = torch.randn(n, device=dev)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-2, weight_decay=0.01)
    p = p0.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for t in range(1, steps + 1):
        gr = torch.randn(n, device=dev)
        p_ref.grad = gr.clone()
        opt.step()
        ops.adam_step(p, gr, m, v, t, lr=1e-2, weight_decay=0.01)
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)


def test_sgd_momentum_and_prox(dev):
    from myfyp_amd import ops

    n = 4099
    p = torch.randn(n, device=dev)
    anchor = torch.randn(n, device=dev)
    cg, cl = torch.randn(n, device=dev), torch.randn(n, device=dev)
    buf = torch.zeros_like(p)
    p_cpu, buf_cpu = p.cpu().clone(), torch.zeros(n)
    for _ in range(3):
        g = torch.randn(n, device=dev)
        ops.sgd_step(p, g, buf, lr=0.1, momentum=0.9, anchor=anchor, c_global=cg, c_local=cl, mu=0.05)
        ops.sgd_step(p_cpu, g.cpu(), buf_cpu, lr=0.1, momentum=0.9, anchor=anchor.cpu(), c_global=cg.cpu(), c_local=cl.cpu(), mu=0.05)
    torch.testing.assert_close(p.cpu(), p_cpu, rtol=1e-5, atol=1e-5)


def test_sign_flip_and_noise(dev):
    from myfyp_amd import ops

    t = torch.randn(100_000, device=dev)
    ref = -t.clone()
    ops.scale_add_noise(t, -1.0, 0.0)
    torch.testing.assert_close(t, ref)
    z = torch.zeros(200_000, device=dev)
    ops.scale_add_noise(z, 1.0, 0.1, seed=3)
    assert abs(z.mean().item()) < 2e-3 and abs(z.std().item() - 0.1) < 3e-3


def _reference_mlp_run(module, x, y, perm, B, lr, steps):
    """fp32 autograd reference: SGD over the given batches."""
    import torch.nn.functional as F

    opt = torch.optim.SGD(module.parameters(), lr=lr)
    for s in range(steps):
        idx = perm[s * B : (s + 1) * B]
        opt.zero_grad()
        F.cross_entropy(module(x[idx]), y[idx]).backward()
        opt.step()


@pytest.mark.parametrize("persistent", [None, False], ids=["persistent", "steps"])
@pytest.mark.parametrize("B", [32, 48])
def test_fused_mlp_engine_matches_autograd(dev, B, persistent, bf16_engine):
    """One local epoch of the grouped engine (2 peers, SGD) vs per-peer fp32 autograd, on the
    weight-stationary persistent epoch kernel and on the 3-launch step path."""
    import copy

    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchLearner, TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.parallel.mlp_engine import MLPGroup
    from myfyp_amd.settings import Settings

    MLPGroup.reset_all()
    Settings.USE_FUSED_KERNELS = True
    data = synthetic_mnist(400, 100, seed=7)
    parts = data.generate_partitions(2, __import__("myfyp_amd.learning.dataset.partition_strategies", fromlist=["x"]).RandomIIDPartitionStrategy)
    lr = 1e-3  # small step: keeps bf16-vs-fp32 trajectories in the linear regime (raw 0..255 inputs)
    learners, refs = [], []
    for i in range(2):
        m = MLP(seed=10 + i)
        with torch.no_grad():  # small weights: unsaturated softmax keeps bf16/fp32 trajectories close
            for prm in m.parameters():
                prm.mul_(0.05)
        m.optimizer_spec = lambda: {"name": "sgd", "lr": lr}
        refs.append(copy.deepcopy(m).to(dev))
        learners.append(TorchLearner(TorchModel(m), parts[i], f"p{i}", batch_size=B))
    assert all(lr_._engine is not None for lr_ in learners)
    group = learners[0]._engine.group
    group.persistent = persistent
    assert group.uses_persistent() == (persistent is not False)
    n = [parts[i].get_num_samples() for i in range(2)]
    perms = [torch.randperm(n[i], generator=torch.Generator().manual_seed(i)) for i in range(2)]

    def perm_fn(ep):
        out = torch.zeros(group.capacity, group.nmax, dtype=torch.int32)
        for i, lr_ in enumerate(learners):
            out[lr_._engine.slot, : n[i]] = perms[i].to(torch.int32)
        return out.to(dev)

    group.perm_fn = perm_fn
    Settings.GANG_WINDOW = 5.0
    import threading

    threads = [threading.Thread(target=lr_.fit) for lr_ in learners]
    [t.start() for t in threads]
    [t.join() for t in threads]
    for i in range(2):
        x, y = learners[i].device_data(True)
        p0 = [p.detach().clone() for p in refs[i].parameters()]
        _reference_mlp_run(refs[i], x, y, perms[i].to(dev), B, lr, (n[i] + B - 1) // B)
        for (name, pe), pr, pz in zip(learners[i].model.get_model().named_parameters(), refs[i].parameters(), p0):
            d_eng, d_ref = (pe.detach() - pz), (pr.detach() - pz)
            rel = (d_eng - d_ref).norm() / (d_ref.norm() + 1e-12)
            assert rel < 0.1, f"peer {i} {name}: relative update error {rel:.4f}"
    # evaluation: fused forward vs autograd forward on the same (updated) weights
    for i in range(2):
        loss, conf = learners[i].evaluate_raw()
        xt, yt = learners[i].device_data(False)
        with torch.no_grad():
            out = refs[i](xt)
            ref_loss = torch.nn.functional.cross_entropy(out, yt).item()
        assert abs(loss - ref_loss) / max(1e-6, abs(ref_loss)) < 0.05
        assert conf.sum() == xt.shape[0]
    MLPGroup.reset_all()


@pytest.mark.parametrize("persistent", [None, False], ids=["persistent", "steps"])
def test_fused_mlp_single_step_gradients(dev, persistent, bf16_engine):
    """Per-parameter gradient of ONE fused step (SGD, grad = Δw/lr) vs autograd, 3 peers, B=40."""
    import copy
    import threading

    import torch.nn.functional as F

    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchLearner, TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.parallel.mlp_engine import MLPGroup
    from myfyp_amd.settings import Settings

    MLPGroup.reset_all()
    Settings.GANG_WINDOW = 5.0
    B, P, lr = 40, 3, 1e-3
    parts = synthetic_mnist(B * P, 60, seed=11).generate_partitions(P, RandomIIDPartitionStrategy)
    learners, refs = [], []
    for i in range(P):
        m = MLP(seed=20 + i)
        m.optimizer_spec = lambda: {"name": "sgd", "lr": lr}
        refs.append(copy.deepcopy(m).to(dev))
        learners.append(TorchLearner(TorchModel(m), parts[i], f"g{i}", batch_size=B))
    g = learners[0]._engine.group
    g.persistent = persistent
    assert g.uses_persistent() == (persistent is not False)
    n = [parts[i].get_num_samples() for i in range(P)]

    def perm_fn(ep):
        out = torch.zeros(g.capacity, g.nmax, dtype=torch.int32)
        for i, l in enumerate(learners):
            out[l._engine.slot, : n[i]] = torch.arange(n[i], dtype=torch.int32)
        return out.to(dev)

    g.perm_fn = perm_fn
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    ts = [threading.Thread(target=l.fit) for l in learners]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for i in range(P):
        x, y = learners[i].device_data(True)
        refs[i].zero_grad()
        F.cross_entropy(refs[i](x[: min(B, n[i])]), y[: min(B, n[i])]).backward()
        for (name, pe), pr, pz in zip(learners[i].model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
            ge, gr = (pz - pe.detach()) / lr, pr.grad
            cos = F.cosine_similarity(ge.flatten(), gr.flatten(), dim=0).item()
            rel = ((ge - gr).norm() / (gr.norm() + 1e-12)).item()
            assert cos > 0.995 and rel < 0.08, f"peer {i} {name}: cos {cos:.4f} rel {rel:.4f}"
    MLPGroup.reset_all()


@pytest.mark.parametrize("B", [64, 32])
def test_persistent_epoch_matches_step_path_adam(dev, B, bf16_engine):
    """Several Adam epochs on 3 peers: persistent epoch kernel vs 3-launch step path from identical
    weights and batch order (same bf16 rounding points; accumulation order and the epilogue's
    reciprocal differ)."""
    import threading

    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchLearner, TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.parallel.mlp_engine import MLPGroup
    from myfyp_amd.settings import Settings

    Settings.GANG_WINDOW = 5.0
    P = 3
    parts = synthetic_mnist(900, 100, seed=5).generate_partitions(P, RandomIIDPartitionStrategy)
    results = {}
    for mode in (None, False):
        MLPGroup.reset_all()
        learners = []
        for i in range(P):
            m = MLP(seed=30 + i)
            m.optimizer_spec = lambda: {"name": "adam", "lr": 1e-3}
            learners.append(TorchLearner(TorchModel(m), parts[i], f"a{i}", batch_size=B))
        g = learners[0]._engine.group
        g.persistent = mode
        assert g.uses_persistent() == (mode is not False)
        n = [parts[i].get_num_samples() for i in range(P)]

        def perm_fn(ep, g=g, learners=learners, n=n):
            out = torch.zeros(g.capacity, g.nmax, dtype=torch.int32)
            for i, l in enumerate(learners):
                out[l._engine.slot, : n[i]] = torch.randperm(n[i], generator=torch.Generator().manual_seed(100 * ep + i)).to(torch.int32)
            return out.to(dev)

        g.perm_fn = perm_fn
        for lr_ in learners:
            lr_.set_epochs(2)
        ts = [threading.Thread(target=l.fit) for l in learners]
        [t.start() for t in ts]
        [t.join() for t in ts]
        torch.cuda.synchronize()
        results[mode] = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
        results[(mode, "loss")] = [l.evaluate_raw()[0] for l in learners]
    init = [[p.detach().clone() for p in MLP(seed=30 + i).parameters()] for i in range(P)]
    for i in range(P):
        for k, (pp, ps, p0) in enumerate(zip(results[None][i], results[False][i], init[i])):
            d_p, d_s = pp.cpu() - p0, ps.cpu() - p0
            rel = ((d_p - d_s).norm() / (d_s.norm() + 1e-12)).item()
            # Adam normalises every coordinate, so 1-ulp differences (hardware rcp/sqrt in the
            # persistent epilogue vs the IEEE division of the step path) and accumulation order
            # move small-gradient coordinates by ~lr; the SGD tests above pin the gradients tightly
            assert rel < 0.1, f"peer {i} param {k}: persistent vs step-path update mismatch {rel:.4f}"
        lp, ls = results[(None, "loss")][i], results[(False, "loss")][i]
        assert abs(lp - ls) / ls < 0.05, (lp, ls)
    MLPGroup.reset_all()
