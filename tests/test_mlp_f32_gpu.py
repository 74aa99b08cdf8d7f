"""fp32 fused MLP engine (csrc/kernels/mlp_persistent_f32.hip) vs plain PyTorch fp32 references.

The reference trains the MLP in fp32 with ``torch.optim.Adam`` (Lightning's default-precision
Trainer: /root/reference/p2pfl/learning/frameworks/pytorch/lightning_learner.py:82-89,
lightning_model.py:181-183). These tests pin the fp32 engine to fp32 autograd + torch optimizers on
identical batches: relative update error < 1e-3 over whole epochs (the bf16 engine is held to 0.1).
"""

import copy
import random
import threading

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from myfyp_amd.ops import _native

    _native.load(required=True)
    return torch.device("cuda")


@pytest.fixture(autouse=True)
def fp32_settings():
    from myfyp_amd.parallel.mlp_engine import MLPGroup
    from myfyp_amd.settings import Settings

    old = (Settings.MLP_PRECISION, Settings.GANG_WINDOW, Settings.USE_FUSED_KERNELS)
    Settings.MLP_PRECISION, Settings.GANG_WINDOW, Settings.USE_FUSED_KERNELS = "fp32", 5.0, True
    MLPGroup.reset_all()
    yield
    MLPGroup.reset_all()
    Settings.MLP_PRECISION, Settings.GANG_WINDOW, Settings.USE_FUSED_KERNELS = old


def _setup(dev, P, B, n_train, seed, spec, scale=1.0):
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchLearner, TorchModel
    from myfyp_amd.models import MLP

    parts = synthetic_mnist(n_train, 200, seed=seed).generate_partitions(P, RandomIIDPartitionStrategy)
    learners, refs = [], []
    for i in range(P):
        m = MLP(seed=50 + i)
        if scale != 1.0:
            with torch.no_grad():
                for prm in m.parameters():
                    prm.mul_(scale)
        m.optimizer_spec = lambda spec=spec: dict(spec)
        refs.append(copy.deepcopy(m).to(dev))
        learners.append(TorchLearner(TorchModel(m), parts[i], f"f{i}", batch_size=B))
    assert all(l._engine is not None for l in learners), "fp32 engine not attached"
    g = learners[0]._engine.group
    assert g.precision == "fp32" and g.uses_persistent()
    n = [parts[i].get_num_samples() for i in range(P)]
    return learners, refs, g, n


def _pin_perms(dev, g, learners, n, seed=0):
    perms = {}

    def perm_fn(ep):
        out = torch.zeros(g.capacity, g.nmax, dtype=torch.int32)
        for i, l in enumerate(learners):
            perms[(ep, i)] = torch.randperm(n[i], generator=torch.Generator().manual_seed(1000 * ep + 10 * seed + i))
            out[l._engine.slot, : n[i]] = perms[(ep, i)].to(torch.int32)
        return out.to(dev)

    g.perm_fn = perm_fn
    return perms


def _fit_all(learners, extras=None):
    def run(i, l):
        if extras is None:
            l.fit()
        else:
            steps, _ = l._engine.fit(l, l._optimizer_spec(), extras[i])

    ts = [threading.Thread(target=run, args=(i, l)) for i, l in enumerate(learners)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    torch.cuda.synchronize()


def _torch_reference(module, x, y, perms, B, spec, epochs, extra=None):
    """fp32 autograd + torch optimizer, fresh optimizer state per fit (Lightning semantics)."""
    params = list(module.parameters())
    if spec["name"] == "adam":
        opt = torch.optim.Adam(params, lr=spec["lr"], weight_decay=spec.get("weight_decay", 0.0))
    else:
        opt = torch.optim.SGD(params, lr=spec["lr"], momentum=spec.get("momentum", 0.0), nesterov=spec.get("nesterov", False),
                              weight_decay=spec.get("weight_decay", 0.0))
    for ep in range(epochs):
        perm = perms[ep].to(x.device)
        for s in range(0, perm.numel(), B):
            idx = perm[s : s + B]
            opt.zero_grad()
            F.cross_entropy(module(x[idx]), y[idx]).backward()
            if extra:
                off = 0
                with torch.no_grad():
                    for p in params:
                        k = p.numel()
                        if "anchor" in extra:
                            p.grad += extra["mu"] * (p - extra["anchor"][off : off + k].view_as(p))
                        off += k
            opt.step()
            if extra and "c_global" in extra:  # SCAFFOLD: update space, w -= lr·(c − c_i) (common.h opt_update)
                off = 0
                with torch.no_grad():
                    for p in params:
                        k = p.numel()
                        p -= spec["lr"] * (extra["c_global"][off : off + k] - extra["c_local"][off : off + k]).view_as(p)
                        off += k


def _rel_update(pe, pr, p0):
    d_e, d_r = pe.detach().double() - p0.double(), pr.detach().double() - p0.double()
    return ((d_e - d_r).norm() / (d_r.norm() + 1e-30)).item()


def _layout(layout: str):
    """(variant, owner K split) of a test layout id: v1ks1, v1ks2, v1ks4, v1ks8, v2, v3ks1, v3ks2."""
    v = int(layout[1])
    return v, (int(layout.split("ks")[1]) if "ks" in layout else 1)


@pytest.mark.parametrize("layout", ["v2", "v1ks1", "v1ks2", "v1ks4", "v1ks8", "v3ks1", "v3ks2"])
@pytest.mark.parametrize("B", [64, 32])
@pytest.mark.parametrize("epochs", [1, 2])
def test_f32_epoch_matches_torch_adam(dev, B, epochs, layout):
    """Whole local epochs of the fp32 persistent kernel (2 peers, Adam 1e-3, raw 0..255 inputs)
    vs fp32 autograd + torch.optim.Adam on the same batches: relative update error < 1e-3. Every gang
    layout: 2 (16 owners, two hand-offs per step: mlp_persistent_f32v2.hip), layout 1 (owners +
    heads) at owner K split 1 (24-workgroup gangs on one XCD) and at the cross-XCD K splits 2 / 4 / 8
    (one peer's gang over 2 / 4 / 8 XCDs, K parts reduced inside each XCD: 4 / 2 / 1 peers per
    launch, so 2 peers at K split 8 take two launches), and layout 3."""
    if B != 64 and layout in ("v1ks4", "v1ks8"):
        pytest.skip("K splits 4 / 8 are instantiated for the 64-row batch tile")
    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = _setup(dev, 2, B, 1400, 3, spec)
    var, ks = _layout(layout)
    g.force_f32_ks = ks
    g.force_f32_variant = var
    assert g.f32_ks() == ks and g.f32_variant() == var
    perms = _pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    for l in learners:
        l.set_epochs(epochs)
    _fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        _torch_reference(refs[i], x, y, [perms[(ep, i)] for ep in range(epochs)], B, spec, epochs)
        for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
            rel = _rel_update(pe, pr, pz)
            assert rel < 1e-3, f"peer {i} {name}: relative update error {rel:.2e}"


@pytest.mark.parametrize(
    "spec",
    [
        {"name": "sgd", "lr": 1e-4},
        {"name": "sgd", "lr": 1e-4, "momentum": 0.9, "nesterov": True, "weight_decay": 1e-3},
        {"name": "adam", "lr": 1e-3, "weight_decay": 1e-2},
    ],
    ids=["sgd", "sgd-nesterov-wd", "adam-wd"],
)
def test_f32_optimizers_match_torch(dev, spec):
    learners, refs, g, n = _setup(dev, 2, 64, 900, 4, spec, scale=0.5)
    perms = _pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    _fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        _torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1)
        for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
            rel = _rel_update(pe, pr, pz)
            if spec["name"] == "adam" and spec.get("weight_decay"):
                # Adam + L2: coordinates where the gradient balances the decay (g ≈ −wd·w) leave a
                # residue at fp32 rounding level that Adam normalises to ±lr, so ONE such coordinate
                # out of 200k moves the norm-relative error to ~2e-3 between any two fp32
                # implementations with different rounding. Bound the count of those instead.
                d = ((pe.detach() - pz) - (pr.detach() - pz)).abs()
                flips = int((d > 0.5 * spec["lr"]).sum())
                assert flips <= max(2, d.numel() // 10000), f"{name}: {flips} coordinates off by > lr/2 (rel {rel:.2e})"
            else:
                assert rel < 1e-3, f"{spec} peer {i} {name}: relative update error {rel:.2e}"


@pytest.mark.parametrize("layout", ["v2", "v1ks1", "v1ks2", "v3ks1", "v3ks2"])
@pytest.mark.parametrize("kind", ["fedprox", "scaffold", "scaffold_adam"])
def test_f32_fedprox_scaffold_terms_match_torch(dev, kind, layout):
    """FedProx mu·(w − anchor) and SCAFFOLD (c − c_i) gradient terms in the fp32 epoch kernel, at
    both owner K splits.

    The terms are checked under SGD (+ momentum for FedProx). Under Adam this setup is chaotic: the
    prox term drives most W1 coordinates onto their anchor within the epoch, where Adam's normalised
    step turns rounding-level differences into ±lr flips — torch fp32 itself, restarted from weights
    one ulp away, moves by 1.5e-2 relative (scripts/probes/f32_ks_fedprox.py). The Adam update the
    terms feed is the same register code and is pinned by test_f32_epoch_matches_torch_adam."""
    spec = {"fedprox": {"name": "sgd", "lr": 1e-3, "momentum": 0.9}, "scaffold": {"name": "sgd", "lr": 1e-4},
            "scaffold_adam": {"name": "adam", "lr": 1e-3}}[kind]
    learners, refs, g, n = _setup(dev, 2, 64, 900, 5, spec, scale=0.5)
    var, ks = _layout(layout)
    g.force_f32_ks = ks
    g.force_f32_variant = var
    assert g.f32_ks() == ks and g.f32_variant() == var
    perms = _pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    gen = torch.Generator(device="cpu").manual_seed(9)
    extras = []
    for l in learners:
        flat = l.flat_params().detach()
        if kind == "fedprox":
            extras.append({"anchor": (flat + 0.01 * torch.randn(flat.shape, generator=gen).to(dev)).contiguous(), "mu": 0.5})
        else:
            extras.append({"c_global": 0.1 * torch.randn(flat.shape, generator=gen).to(dev), "c_local": 0.1 * torch.randn(flat.shape, generator=gen).to(dev)})
    _fit_all(learners, extras)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        _torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1, extra=extras[i])
        for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
            rel = _rel_update(pe, pr, pz)
            assert rel < 1e-3, f"{kind} peer {i} {name}: relative update error {rel:.2e}"


@pytest.mark.parametrize("kind", ["fedprox", "scaffold"])
def test_f32_adam_extra_defaults_to_spill_free_layout(dev, kind):
    """Adam + FedProx/SCAFFOLD at owner K split 1 runs layout 2 unless a layout is forced: layout 1's
    instantiation spills VGPRs there, layout 2's does not (kernel-resource-usage remarks). Layout 2's
    numerics with these terms are pinned by test_f32_fedprox_scaffold_terms_match_torch."""
    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = _setup(dev, 2, 64, 900, 6, spec, scale=0.5)
    g.force_f32_ks = 1
    g.force_f32_variant = 0
    assert g.f32_variant() == 1  # no extra term yet
    flat = [l.flat_params().detach().clone() for l in learners]
    if kind == "fedprox":
        extras = [{"anchor": f.contiguous(), "mu": 0.01} for f in flat]
    else:
        extras = [{"c_global": torch.zeros_like(f), "c_local": torch.zeros_like(f)} for f in flat]
    _fit_all(learners, extras)
    assert g.f32_variant() == 2 and g.f32_ks() == 1
    for l, f in zip(learners, flat):
        d = l.flat_params().detach() - f
        assert torch.isfinite(d).all() and d.abs().max() > 0


def test_f32_w2_replica_is_bit_identical(dev):
    """Layout 1: the owners' W2 replica (updated from their own dW2 tile) equals the heads' W2 rows
    bit for bit."""
    from myfyp_amd.ops import _native

    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = _setup(dev, 3, 64, 1500, 6, spec)
    g.force_f32_variant = 1
    assert g.f32_variant() == 1
    _pin_perms(dev, g, learners, n)
    chk = torch.full((g.capacity, 128, 256), float("nan"), device=dev)
    lib = _native.load(required=True)
    with g.lock:
        g._ensure_engine()
        _native.check(lib.mlp_engine_set_w2chk(g._engine, chk.data_ptr()), "set_w2chk")
    try:
        for l in learners:
            l.set_epochs(2)
        _fit_all(learners)
    finally:
        with g.lock:
            lib.mlp_engine_set_w2chk(g._engine, None)
    D0, D1, D2 = 784, 256, 128
    off_w2 = D1 * D0 + D1
    for l in learners:
        w2 = g.params[l._engine.slot, off_w2 : off_w2 + D2 * D1].view(D2, D1)
        assert torch.equal(chk[l._engine.slot], w2), "W2 replica diverged from the heads' rows"


def test_f32_eval_matches_torch(dev):
    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = _setup(dev, 2, 64, 600, 7, spec)
    _fit_all(learners)
    for l in learners:
        loss, conf = l.evaluate_raw()
        xt, yt = l.device_data(False)
        with torch.no_grad():
            out = l.model.get_model()(xt).double()
        ref_loss = F.cross_entropy(out, yt).item()
        assert abs(loss - ref_loss) / max(1e-9, abs(ref_loss)) < 1e-4, (loss, ref_loss)
        pred = out.argmax(1).cpu().numpy()
        ref_conf = np.zeros_like(conf)
        np.add.at(ref_conf, (yt.cpu().numpy(), pred), 1)
        assert (conf == ref_conf).all()


def test_f32_partial_last_batch_and_bias(dev):
    """A split whose size is not a multiple of B (partial last batch) and non-zero biases: SGD
    updates of every tensor, b1 included (carried through the bias column of the X tile)."""
    spec = {"name": "sgd", "lr": 1e-4}
    learners, refs, g, n = _setup(dev, 2, 64, 2 * 233, 8, spec, scale=0.5)
    assert any(k % 64 for k in n)
    perms = _pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    _fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        _torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1)
        for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
            rel = _rel_update(pe, pr, pz)
            assert rel < 1e-4, f"peer {i} {name}: relative update error {rel:.2e}"


@pytest.mark.parametrize("layout", [2, 1, 3])
@pytest.mark.parametrize("at_end", [False, True])
def test_f32_giveup_recovered_by_retry_launch(dev, at_end, layout):
    """A gang that gives up (here: forced on its first attempt through the engine's test hook, as a
    non-resident workgroup would) is re-run by the in-stream retry launch from the untouched
    pre-epoch state: the epoch result is bit-identical to a run without the give-up, the other
    peers are unaffected, and the engine counts one recovery per epoch. at_end: the give-up comes
    after every step ran, at the gang commit — no role may have stored anything."""
    spec = {"name": "adam", "lr": 1e-3}
    results = []
    for forced in (False, True):
        from myfyp_amd.parallel.mlp_engine import MLPGroup

        MLPGroup.reset_all()
        learners, refs, g, n = _setup(dev, 3, 64, 1500, 5, spec)
        g.force_f32_variant = layout
        assert g.f32_variant() == layout
        _pin_perms(dev, g, learners, n)
        if forced:
            g.debug_giveup(learners[1]._engine.slot, at_end=at_end)
        _fit_all(learners)
        _ = [l.evaluate() for l in learners]  # results fetched: give-up status checked
        results.append(([l.flat_params().detach().clone() for l in learners], g.recoveries()))
        if forced:
            g.debug_giveup(None)
    (p_ok, rec_ok), (p_rec, rec_rec) = results
    assert rec_ok == 0 and rec_rec == 1, (rec_ok, rec_rec)
    for a, b in zip(p_ok, p_rec):
        assert torch.equal(a, b)


def test_f32_prewarm_is_transparent(dev):
    """Engine prewarm (Node.start: graph capture + upload, code-object load) runs no training work:
    an epoch after prewarm is bit-identical to one without it."""
    from myfyp_amd.parallel.mlp_engine import MLPGroup

    spec = {"name": "adam", "lr": 1e-3}
    results = []
    for warm in (True, False):
        MLPGroup.reset_all()
        learners, refs, g, n = _setup(dev, 2, 64, 1400, 7, spec)
        _pin_perms(dev, g, learners, n)
        if warm:
            for l in learners:
                l.prewarm()
            torch.cuda.synchronize()
        _fit_all(learners)
        results.append([l.flat_params().detach().clone() for l in learners])
    for a, b in zip(*results):
        assert torch.equal(a, b)


@pytest.mark.parametrize("prep_mode,epochs", [("1", 1), ("2", 1), ("2", 2)])
def test_f32_prep_stream_gather_matches_in_graph_gather(dev, monkeypatch, prep_mode, epochs):
    """The epoch batch gather on its own stream into alternating batch buffers (mode 1: after the
    last epoch that read the buffer; mode 2: beside the previous epoch, on a capped grid-strided
    grid, and enqueued one epoch ahead — within a fit and across fits) gives bit-identical training
    to the gather as the first node of the epoch graph: three fits (both buffers used, reused) with
    the in-kernel shuffle of keys from one seeded stream."""
    import random

    from myfyp_amd.parallel.mlp_engine import MLPGroup

    spec = {"name": "adam", "lr": 1e-3}
    results = []
    monkeypatch.setenv("MYFYP_PREP_GATHER_WGS", "6")  # fewer workgroups than row blocks: the stride loop runs
    for prep in (prep_mode, "0"):
        monkeypatch.setenv("MYFYP_PREP_GATHER", prep)
        MLPGroup.reset_all()
        learners, refs, g, n = _setup(dev, 3, 64, 1500, 7, spec)
        for l in learners:
            l.set_epochs(epochs)
        random.seed(4321)
        for _ in range(3):
            _fit_all(learners)
        results.append([l.flat_params().detach().clone() for l in learners])
    for a, b in zip(*results):
        assert torch.equal(a, b)


def test_scaffold_control_variate_matches_formula(dev):
    """SCAFFOLD client on the fused engine: after each fit the device-resident control variate is
    c_i⁺ = c_i − c + (x − y)/(K·lr) (option II; reference scaffold_callback.py:124-140), Δy = y − x and
    Δc = c_i⁺ − c_i, pinned in float64 at rel < 1e-4 over two rounds (the second with c_i ≠ 0)."""
    from myfyp_amd.learning.frameworks.torch.callbacks import SCAFFOLDCallback

    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = _setup(dev, 2, 64, 900, 8, spec)
    cbs = [SCAFFOLDCallback() for _ in learners]
    for l, cb in zip(learners, cbs):
        l.callbacks = [cb]
    gen = torch.Generator(device="cpu").manual_seed(3)
    for rnd in range(2):
        c = [0.01 * torch.randn(l.flat_params().numel(), generator=gen) for l in learners]
        olds = []
        for l, cb, ci in zip(learners, cbs, c):
            cb.additional_info["global_c"] = l.split_flat(ci.to(dev))
            olds.append(None if cb.c_i is None else cb.c_i.detach().double().cpu())
        steps0 = [l.global_step for l in learners]
        ts = [threading.Thread(target=l.fit) for l in learners]
        [t.start() for t in ts]
        [t.join() for t in ts]
        torch.cuda.synchronize()
        for l, cb, ci, old, s0 in zip(learners, cbs, c, olds, steps0):
            k = l.global_step - s0
            assert k == (n[learners.index(l)] + 63) // 64
            x0, y = cb.x0.double().cpu(), l.flat_params().detach().double().cpu()
            ci_old = torch.zeros_like(x0) if old is None else old
            want = ci_old - ci.double() + (x0 - y) / (k * spec["lr"])
            got = cb.c_i.detach().double().cpu()
            rel = ((got - want).norm() / want.norm()).item()
            assert rel < 1e-4, (rnd, rel)
            assert torch.allclose(cb.delta_y.double().cpu(), y - x0, rtol=0, atol=1e-6)
            assert ((cb.delta_c.double().cpu() - (want - ci_old)).norm() / (want - ci_old).norm()).item() < 1e-4


@pytest.mark.parametrize("peers,ks", [(2, 1), (8, 1), (1, 8), (2, 4), (4, 2)])
def test_f32_single_xcd_handoffs_bit_identical(dev, peers, ks):
    """Single-XCD gangs keep their hand-offs in L2 (plain stores, persist::gang_same_xcd): the same
    fit with write-through hand-offs gives bit-identical parameters, and on MI355X every K-split-1
    gang (blocks b = p mod 8) is found on one XCD, so the fast path is the one exercised. The
    cross-XCD K split (ks > 1: one peer over ks XCDs) keeps the hand-offs INSIDE each group (a column
    group's K parts; the heads) plain when the group is found on one XCD (persist::group_same_xcd),
    and writes the H1 / dH2 hand-offs between XCDs through: bit-identical as well."""
    import ctypes

    from myfyp_amd.ops import _native
    from myfyp_amd.parallel.mlp_engine import MLPGroup

    lib = _native.load(required=True)
    spec = {"name": "adam", "lr": 1e-3}
    out = {}
    try:
        for mode in (1, 0):
            lib.mlp_set_plain_pub(mode)
            MLPGroup.reset_all()
            learners, refs, g, n = _setup(dev, peers, 64, 600 * peers, 11, spec)
            g.force_f32_ks = ks
            g.force_f32_variant = 1
            assert g.f32_ks() == ks
            _pin_perms(dev, g, learners, n)
            _fit_all(learners)
            seen = (ctypes.c_int * 64)()
            assert lib.mlp_debug_plain_seen(seen) == 0
            out[mode] = ([l.flat_params().detach().clone() for l in learners], list(seen)[:peers])
    finally:
        lib.mlp_set_plain_pub(-1)
    assert out[0][1] == [0] * peers
    assert out[1][1] == [1] * peers, f"gangs not all on one XCD: {out[1][1]}"
    for a, b in zip(out[1][0], out[0][0]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("peers,ks", [(8, 1), (1, 8)])
def test_f32_flag_block_sparse_zeroing(dev, peers, ks):
    """Between epochs only word 0 of each hand-off flag line, plus the gang-placement slot lines, is
    zeroed (engine.hip k_upload_ctl, profiles/r6x_flags). With every word of the block set to ~0
    before each epoch's zeroing, a flag read anywhere else would release its consumer before the
    hand-off is written: the same fits must still give bit-identical parameters."""
    from myfyp_amd.ops import _native
    from myfyp_amd.parallel.mlp_engine import MLPGroup

    lib = _native.load(required=True)
    spec = {"name": "adam", "lr": 1e-3}
    out = {}
    for poison in (0, 1):
        MLPGroup.reset_all()
        learners, refs, g, n = _setup(dev, peers, 64, 600 * peers, 13, spec)
        g.force_f32_ks = ks
        g.force_f32_variant = 1
        assert g.f32_ks() == ks
        # the device-side epoch shuffle (pinned permutations would leave the prep-stream gather
        # mode, whose control upload is where the sparse zeroing runs), keyed from the same seed
        random.seed(1234)
        with g.lock:
            g._ensure_engine()
            lib.mlp_engine_debug_poison_flags(g._engine, poison)
        for l in learners:
            l.set_epochs(2)
        _fit_all(learners)
        with g.lock:
            done = lib.mlp_engine_debug_poison_flags(g._engine, 0)
        assert (done > 0) == bool(poison), done  # the sparse zeroing ran after the poison
        out[poison] = [l.flat_params().detach().clone() for l in learners]
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
