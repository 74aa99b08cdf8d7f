"""Headline benchmark: rounds/sec (+ wall-clock to target accuracy) of MNIST-MLP FedAvg with 8 peers.

Metric/config come from BASELINE.json: "rounds/sec + wall-clock-to-target-acc, MNIST MLP FedAvg 8 peers
at 1/2/4/8 MI355X". One process per GPU (``torchrun``); the 8 peers are split evenly over the N
ranks (8/N co-located peers per GPU, grouped into each fused launch) — total work is fixed, so the
scaling mode is "strong". Every timed round is a full federated round through the public Node API
and the collective stage workflow:

    vote (all-gather) → evaluate (fused fwd) → local epoch (fused fwd+bwd+Adam, hipGraph replay)
    → FedAvg (weighted local reduction + RCCL all-reduce over xGMI + broadcast) → round bookkeeping

Data: synthetic MNIST-shaped uint8 (60k train / 10k test, IID split, no network), random-init
weights of the reference MLP (784-256-128-10, Adam lr 1e-3, 1 local epoch). Local batch 64
(the reference's batch-1 default is a Lightning export default; see BASELINE.md / README).
Precision: fp32 by default — the reference's (Lightning's default-precision Trainer): the fp32
persistent epoch kernel (exact fp32 products, fp32 accumulation, fp32 weights / Adam state) and
fp32 evaluation; ``--precision bf16`` is the bf16-operand engine (secondary number).
The synthetic classes overlap (similarity 0.75, noise 1.0) so that 0.9 test accuracy takes several
rounds (~7 in a CPU fp32 calibration) and the time-to-target half of the metric measures something.

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node 8 bench.py --gpus 8 --steps 20 --warmup 3

Rank 0 prints ONE JSON line. Timing: barrier + device synchronize on both sides of exactly K rounds
(inside the round-end hook that every rank's gang leader runs after aggregation), MAX over ranks.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rounds/sec + wall-clock-to-target-acc, MNIST MLP FedAvg 8 peers at 1/2/4/8 MI355X"
# the reference publishes no throughput. The comparison point is the MEASURED proxy of
# the reference algorithm (gossip workflow, batch-1 fp32 CPU learner, 8 nodes): 1.20 rounds/s.
BASELINE_ROUNDS_PER_SEC = 1.20


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed federated rounds (~2 ms each on MI355X)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed rounds (graph capture, caches)")
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--n-train", type=int, default=60000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--target-acc", type=float, default=0.9)
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32", help="fused MLP engine precision")
    ap.add_argument("--similarity", type=float, default=0.75, help="synthetic class overlap (difficulty)")
    ap.add_argument("--noise", type=float, default=1.0, help="synthetic stroke noise (difficulty)")
    ap.add_argument("--no-fused", action="store_true", help="autograd path instead of the fused HIP engine")
    ap.add_argument("--eager", action="store_true", help="fused kernels without hipGraph (A/B)")
    ap.add_argument("--force-collective", action="store_true",
                    help="one GPU: run FedAvg through a world-size-1 RCCL group (the multi-rank path: side-stream reduce -> RCCL all-reduce -> apply)")
    ap.add_argument("--no-failover", action="store_true", help="skip the per-round confirmation of the weight collectives (fault tolerance off)")
    ap.add_argument("--no-prewarm", action="store_true", help="do not prepare the fused engine at Node.start (round 0 captures the epoch graph)")
    ap.add_argument("--launch", choices=["auto", "mesh", "ranks"], default="auto",
                    help="ranks: one process per GPU (torchrun, torch.distributed over RCCL); mesh: ONE process drives the N GPUs "
                         "(in-process RCCL mesh, ncclCommInitAll; under torchrun rank 0 drives them and the other ranks wait). "
                         "auto = ranks under torchrun, mesh for one process started with --gpus N")
    ap.add_argument("--mesh-virtual", action="store_true",
                    help="rehearsal: N mesh ranks on the visible device(s) with host-side collectives (n_gpus reports the physical count)")
    return ap.parse_args()


def _engine_label(nodes, eager: bool) -> str:
    """What actually launched the local epochs: the persistent epoch kernel is launched directly
    (``MYFYP_EPOCH_GRAPH=0`` default since round 5); the step path replays a captured hipGraph."""
    eng = getattr(nodes[0].learner, "_engine", None) if nodes else None
    grp = getattr(eng, "group", None)
    kind = getattr(grp, "epoch_launch_kind", None)
    try:
        kind = kind() if callable(kind) else kind
        ks = grp.f32_ks() if getattr(grp, "precision", "") == "fp32" and grp.uses_persistent() else 1
    except Exception:  # noqa: BLE001 — a label only
        kind, ks = None, 1
    if kind and ks > 1:
        kind += f"-xcd-ksplit{ks}"
    if eager:
        return "fused-hip-eager"
    return f"fused-hip-{kind}" if kind else "fused-hip"


def main() -> None:
    args = parse()
    from myfyp_amd.utils import launch

    mode = launch.plan_launch(args.gpus, args.launch, args.mesh_virtual)
    if mode == "park":
        launch.park()
        return
    parked_group = mode == "mesh" and launch.env_world()[0] > 1
    if parked_group:  # rank 0 of a torchrun job in mesh mode: release the waiting ranks at the end
        launch.cpu_group()
    import numpy as np
    import torch

    from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.management.logger import logger
    from myfyp_amd.management.tracing import mark
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.seed import set_seed
    from myfyp_amd.utils.utils import wait_to_finish

    set_seed(1234)
    Settings.LOG_LEVEL = "WARNING"
    logger.set_level("WARNING")
    Settings.HEARTBEAT_PERIOD = 5
    Settings.HEARTBEAT_TIMEOUT = 600
    Settings.GOSSIP_PERIOD = 0
    Settings.TRAIN_SET_SIZE = args.peers  # FedAvg over all 8 peers every round
    Settings.VOTE_TIMEOUT = 600
    Settings.AGGREGATION_TIMEOUT = 600
    Settings.BATCH_SIZE = args.batch_size
    Settings.USE_FUSED_KERNELS = not args.no_fused
    Settings.GANG_WINDOW = 5.0
    Settings.MLP_PRECISION = args.precision
    Settings.FORCE_COLLECTIVE = bool(args.force_collective)
    Settings.COLLECTIVE_FAILOVER = not args.no_failover
    Settings.ENGINE_PREWARM = not args.no_prewarm

    if mode == "mesh":
        Settings.MESH_VIRTUAL = bool(args.mesh_virtual)
        fed = Federation.init(devices=args.gpus)
        launch.check_mesh(fed, args.gpus, bool(args.mesh_virtual), "bench")
        mesh_devs = list(fed.devices)
    else:
        fed = Federation.init()
        mesh_devs = [fed.device]
    world, rank = fed.world, fed.rank
    n_units = fed.mesh_size if fed.mesh is not None else world
    if args.peers % n_units:
        raise SystemExit(f"--peers {args.peers} must be divisible by the number of GPUs {n_units}")
    ppr = args.peers // world  # peers hosted by this process (all of them in mesh mode)
    data = synthetic_mnist(args.n_train, args.n_test, seed=2024, similarity=args.similarity, noise=args.noise)
    parts = data.generate_partitions(args.peers, RandomIIDPartitionStrategy)
    gids = [rank * ppr + j for j in range(ppr)]
    nodes = [
        Node(TorchModel(MLP(seed=100 + g)), parts[g], address=f"peer-{g}", protocol=CollectiveCommunicationProtocol, learner_kwargs={"batch_size": args.batch_size})
        for g in gids
    ]
    prof_start = os.environ.get("MYFYP_PROFILE_START")  # diagnostics: cProfile of the node starts
    if prof_start:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t_ns = time.perf_counter()
    for n in nodes:
        n.start()  # Settings.ENGINE_PREWARM: the fused engine captures its epoch graph here
    node_start_s = time.perf_counter() - t_ns
    if prof_start:
        prof.disable()
        prof.dump_stats(prof_start)
    fed.finalize()
    if args.eager:
        for n in nodes:
            eng = getattr(n.learner, "_engine", None)
            if eng is not None:
                eng.group.eager = True
    fused = all(getattr(n.learner, "_engine", None) is not None for n in nodes)

    total_rounds = args.warmup + args.steps
    marks: dict = {}
    round_end: dict = {}
    cuda_devs = sorted({d.index for d in mesh_devs if d.type == "cuda"})

    def dev_sync() -> None:  # every device this process drives
        for i in cuda_devs:
            torch.cuda.synchronize(i)

    def start_hook(r: int, f) -> None:
        # the first timed round starts here: its train set is known, nothing of it is launched yet,
        # and every warmup round has been launched (barrier + synchronize, then the clock starts)
        if args.warmup > 0 and r == args.warmup:
            f.barrier()
            dev_sync()
            marks["t0"] = time.perf_counter()
            mark("bench:t0")  # roctx (MYFYP_ROCTX=1): the timed window's start on a kernel trace

    def hook(r: int, f) -> None:
        round_end[r] = time.perf_counter()
        if r == total_rounds - 1:  # the last timed round's work is all enqueued
            dev_sync()
            f.barrier()
            marks["t1"] = time.perf_counter()
            mark("bench:t1")

    fed.round_start_hooks.append(start_hook)
    fed.round_hooks.append(hook)
    import gc

    gc_pauses: list = []  # diagnostics: interpreter garbage-collection pauses during the run
    gc_t: dict = {}

    def on_gc(phase, info):
        if phase == "start":
            gc_t["t"] = time.perf_counter()
        elif "t" in gc_t:
            gc_pauses.append((info.get("generation", -1), 1000.0 * (time.perf_counter() - gc_t.pop("t"))))

    gc.callbacks.append(on_gc)
    # evaluations resolve asynchronously: record when each round's accuracy actually landed on the host
    landed: dict = {}
    local_addrs = {n.addr for n in nodes}

    def on_metric(addr, exp_name, rnd, metric, value, step):
        if metric == "test_metric" and step is None and addr in local_addrs:
            landed.setdefault(rnd, []).append((value, time.perf_counter()))

    logger.add_metric_listener(on_metric)
    if args.warmup == 0:
        marks["t0"] = None
    t_start = time.perf_counter()
    if rank == 0:
        nodes[0].set_start_learning(rounds=total_rounds, epochs=args.epochs)
    if args.warmup == 0:
        # no warmup: time from the start barrier of round 0 (includes capture)
        fed.barrier()
        dev_sync()
        marks["t0"] = time.perf_counter()
    wait_to_finish(nodes, timeout=3600)
    t0, t1 = marks.get("t0"), marks.get("t1")
    elapsed = (t1 - t0) if (t0 is not None and t1 is not None) else float("nan")
    # max over the (live) ranks
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=fed.device)
        fed.all_reduce_(tt, op="max")
        elapsed = float(tt.item())

    # accuracy curve of the local peers: test_metric logged at round r = model after round r-1
    logs = logger.get_global_logs().get("experiment", {})
    acc_by_round: dict = {}
    for n in nodes:
        for r, v in logs.get(n.addr, {}).get("test_metric", []):
            acc_by_round.setdefault(r, []).append(v)
    mean_acc = {r: float(np.mean(v)) for r, v in sorted(acc_by_round.items())}
    t_target, r_target = None, None
    for r, a in mean_acc.items():
        if a >= args.target_acc and r >= 1 and r in landed:
            # time at which the last local peer's evaluation of the round-(r-1) model reached the host
            t_target, r_target = max(t for _, t in landed[r]) - t_start, r
            break
    final_acc = mean_acc[max(mean_acc)] if mean_acc else None
    # per-stage wall-time breakdown of the first local peer (stderr, diagnostics only)
    tm = dict(logger.get_timings().get(nodes[0].addr, {}))
    for nd in nodes:  # the round driver logs its host time per round under one of the local peers
        for key in ("driver_round", "driver_round_cpu"):
            if key in logger.get_timings().get(nd.addr, {}):
                tm[key] = logger.get_timings()[nd.addr][key]
    brk = {k: round(1000 * float(np.median(v[args.warmup :] or v)), 3) for k, v in tm.items()}
    first = [round(1000 * (round_end[r] - t_start), 2) for r in sorted(round_end)[:10]]
    print(f"[bench] rank {rank} round-end times since set_start_learning (ms), rounds 0..9: {first}", file=sys.stderr, flush=True)
    ends = [round_end[r] for r in sorted(round_end) if r >= args.warmup - 1]
    if len(ends) > 2:
        d = np.diff(ends) * 1000.0
        print(f"[bench] rank {rank} round-end interval ms: p10 {np.percentile(d, 10):.3f} p50 {np.percentile(d, 50):.3f} "
              f"p90 {np.percentile(d, 90):.3f} max {d.max():.3f}", file=sys.stderr, flush=True)
    if gc_pauses:
        worst = max(gc_pauses, key=lambda g: g[1])
        print(f"[bench] rank {rank} gc pauses: {len(gc_pauses)}, total {sum(g[1] for g in gc_pauses):.2f} ms, max {worst[1]:.2f} ms (gen {worst[0]}), "
              f"gen2: {sum(1 for g in gc_pauses if g[0] == 2)}", file=sys.stderr, flush=True)
    print(f"[bench] rank {rank} median ms per call: {json.dumps(brk)} fed: "
          f"{ {k: round(1000 * float(np.median(v)), 3) for k, v in fed.stats.items()} }", file=sys.stderr, flush=True)
    engine_label = _engine_label(nodes, args.eager) if fused else "autograd"  # (before the nodes stop)
    eng = getattr(nodes[0].learner, "_engine", None)
    if eng is not None and hasattr(eng.group, "graph_launch_stats"):
        print(f"[bench] rank {rank} epoch graph launches: {eng.group.graph_launch_stats()}", file=sys.stderr, flush=True)
    for n in nodes:
        n.stop()

    rps = args.steps / elapsed if elapsed == elapsed and elapsed > 0 else 0.0
    coll = "none (one rank: local weighted-mean kernel)"
    n_phys = len(cuda_devs) if cuda_devs else 0
    if fed.mesh is not None:
        coll = (f"in-process {fed.mesh.kind} mesh over {fed.mesh_size} devices (one process; per device reduce -> grouped all-reduce -> apply)"
                + (" [virtual: members share one device]" if args.mesh_virtual else ""))
        if fed.mesh.kind == "rccl":
            coll = f"rccl mesh: ncclCommInitAll over {fed.mesh_size} GPUs in one process; per GPU reduce -> grouped ncclAllReduce -> apply"
    if fed.collective:
        import torch.distributed as dist

        be = dist.get_backend(fed.group)
        coll = ("rccl" if be == "nccl" else be) + (" world-1 (forced)" if fed.forced else "") + (", failover" if fed._guarded() else "")
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(rps, 3),
            "unit": "rounds/s",
            "n_gpus": n_phys if fed.mesh is not None else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / max(1, args.steps), 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(rps / BASELINE_ROUNDS_PER_SEC, 2),
            "dtype": args.precision if fused else "fp32",
            "data": f"synthetic (MNIST-shaped uint8 {args.n_train // 1000}k/{args.n_test // 1000}k, similarity {args.similarity}, noise {args.noise}, IID over peers), random-init weights",
            "config": {
                "model": "MLP 784-256-128-10 (reference MLP)",
                "global_batch": args.batch_size * args.peers,
                "local_batch": args.batch_size,
                "seq_len": None,
                "parallelism": f"fedavg-{args.peers}peers-dp{n_units}" + ("-mesh" if fed.mesh is not None else ""),
                "peers": args.peers,
                "peers_per_gpu": args.peers // n_units,
                "launch": ("one process drives all GPUs (device mesh)" + (" ; torchrun ranks > 0 idle" if parked_group else "")) if fed.mesh is not None
                else ("one process per GPU" if world > 1 else "single process, one GPU"),
                "train_set_size": args.peers,
                "epochs_per_round": args.epochs,
                "optimizer": "adam lr=1e-3 (fresh per round)",
                "aggregator": "FedAvg (weighted all-reduce)",
                "collective": coll,
                "engine": engine_label,
            },
            # headline time-to-target: Node.start() (incl. the engine prewarm) + set_start_learning
            # -> the evaluation that reaches the target (the prewarm moved setup out of
            # the set_start_learning window; the sum is the honest wall-clock)
            "time_to_target_s": None if t_target is None else round(node_start_s + t_target, 3),
            "time_to_target_from_start_learning_s": None if t_target is None else round(t_target, 3),
            "rounds_to_target": r_target,
            "target_acc": args.target_acc,
            "final_test_acc": None if final_acc is None else round(final_acc, 4),
            "node_start_s": round(node_start_s, 4),
            "node_start_note": "Node.start() of the local peers before set_start_learning, incl. the fused-engine prewarm (epoch-graph capture/upload, code-object load; no training work); time_to_target_s = node_start_s + time_to_target_from_start_learning_s",
            "baseline_note": "vs_baseline = value / 1.20 rounds/s, the measured proxy of the reference algorithm (gossip, batch-1 fp32 CPU learner, 8 nodes; BASELINE.md; the reference publishes no number). Context, not parity: this run trains at local batch 64 on the GPU, the proxy at batch 1 on the CPU",
        }
        print(json.dumps(out), flush=True)
    fed.shutdown()
    if parked_group:
        launch.release_parked()


if __name__ == "__main__":
    main()
