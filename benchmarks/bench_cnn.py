"""CNN federated benchmarks (BASELINE configs 3-5) on the grouped HIP CNN engine.

    python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor      # config 3 (ring neighbour averaging)
    python benchmarks/bench_cnn.py --model resnet18                          # config 4 (FedAvg + fused SGD)
    python benchmarks/bench_cnn.py --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout  # config 5
    python benchmarks/bench_cnn.py --model resnet18 --torch-step             # + torch/MIOpen step A/B

Each timed round is a full federated round through the Node API and the collective workflow
(vote → evaluate → one local epoch → aggregate). One JSON line on rank 0: rounds/s, train images/s,
final accuracy. Data: synthetic CIFAR-10-shaped uint8 (no network), random-init weights.
``--torch-step`` additionally times the same local step in PyTorch (bf16 autocast, channels-last,
MIOpen convolutions, torch.optim.SGD) for one peer and reports both per-peer step times.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["lenet5", "resnet18"], default="resnet18")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs (torchrun: one process per GPU; one process: device mesh; see myfyp_amd/utils/launch.py)")
    ap.add_argument("--launch", choices=["auto", "mesh", "ranks"], default="auto")
    ap.add_argument("--mesh-virtual", action="store_true", help="rehearsal: --gpus mesh ranks on the visible device(s)")
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--batch-size", type=int, default=0, help="0 = 128 for resnet18, 64 for lenet5")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--aggregator", choices=["fedavg", "neighbor", "fedprox"], default="fedavg")
    ap.add_argument("--dirichlet", type=float, default=0.0, help="non-IID Dirichlet alpha (0 = IID)")
    ap.add_argument("--dropout", action="store_true", help="kill one peer at round 1 (fault tolerance)")
    ap.add_argument("--mu", type=float, default=0.01, help="FedProx proximal coefficient")
    ap.add_argument("--no-fused", action="store_true", help="torch autograd learner instead of the HIP engine (A/B oracle)")
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--torch-step", action="store_true")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--delayed-averaging", action="store_true", help="opt-in delayed averaging (numerics change; last round exact)")
    ap.add_argument("--no-overlap", action="store_true", help="synchronous FedAvg (no side-stream bucket pipeline)")
    ap.add_argument("--bucket-mb", type=float, default=0.0, help="all-reduce bucket size (0 = Settings.BUCKET_BYTES)")
    # synthetic-data difficulty (so that time-to-accuracy measures something: the default CIFAR
    # stand-in is learnt to ~100 % in one round by ResNet-18)
    # per-model defaults (None): calibrated on MI355X so that the target takes several rounds and
    # the accuracy does not saturate (profiles/r3c_cifar_difficulty)
    ap.add_argument("--similarity", type=float, default=None, help="class-prototype overlap")
    ap.add_argument("--noise", type=float, default=None, help="per-pixel stroke noise")
    ap.add_argument("--modes", type=int, default=None, help="prototypes per class")
    ap.add_argument("--label-noise", type=float, default=None, help="fraction of training labels randomised")
    ap.add_argument("--target-acc", type=float, default=None, help="time-to-accuracy target (mean test accuracy over the peers)")
    args = ap.parse_args()
    dflt = DIFFICULTY[args.model]
    for k, v in dflt.items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    return args


# synthetic-CIFAR difficulty per model (similarity, noise, modes, label noise) and the accuracy target
DIFFICULTY = {
    "lenet5": {"similarity": 0.8, "noise": 1.2, "modes": 4, "label_noise": 0.1, "target_acc": 0.8},
    "resnet18": {"similarity": 0.85, "noise": 1.2, "modes": 4, "label_noise": 0.1, "target_acc": 0.9},
}


def torch_step_ms(model_name: str, batch: int, iters: int = 20) -> float:
    import torch
    import torch.nn.functional as F

    from myfyp_amd.models import LeNet5, ResNet18

    m = (ResNet18 if model_name == "resnet18" else LeNet5)(seed=0).cuda().to(memory_format=torch.channels_last)
    spec = m.optimizer_spec()
    opt = torch.optim.SGD(m.parameters(), lr=spec["lr"], momentum=spec.get("momentum", 0.0), weight_decay=spec.get("weight_decay", 0.0))
    x = torch.randint(0, 255, (batch, 32, 32, 3), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (batch,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / iters


def main() -> None:
    args = parse()
    from myfyp_amd.utils import launch

    mode = launch.plan_launch(args.gpus, args.launch, args.mesh_virtual)
    if mode == "park":
        launch.park()
        return
    parked_group = mode == "mesh" and launch.env_world()[0] > 1
    if parked_group:
        launch.cpu_group()
    import numpy as np
    import torch

    from myfyp_amd import fault_injection
    from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
    from myfyp_amd.learning.aggregators import FedAvg, FedProx, NeighborAvg
    from myfyp_amd.learning.dataset.partition_strategies import DirichletPartitionStrategy, RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.management.logger import logger
    from myfyp_amd.models import LeNet5, ResNet18
    from myfyp_amd.node import Node
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.seed import set_seed
    from myfyp_amd.utils.utils import wait_to_finish

    set_seed(1234)
    B = args.batch_size or (128 if args.model == "resnet18" else 64)
    logger.set_level("WARNING")
    Settings.LOG_LEVEL = "WARNING"
    Settings.HEARTBEAT_TIMEOUT = 3600
    Settings.TRAIN_SET_SIZE = args.peers
    Settings.VOTE_TIMEOUT = Settings.AGGREGATION_TIMEOUT = 3600
    Settings.BATCH_SIZE = B
    if args.no_fused:
        Settings.USE_FUSED_KERNELS = False
    Settings.GANG_WINDOW = 30.0
    Settings.DELAYED_AVERAGING = bool(args.delayed_averaging)
    Settings.OVERLAP_COLLECTIVES = not args.no_overlap
    if args.bucket_mb > 0:
        Settings.BUCKET_BYTES = int(args.bucket_mb * (1 << 20))
    if mode == "mesh":
        Settings.MESH_VIRTUAL = bool(args.mesh_virtual)
        fed = Federation.init(devices=args.gpus)
        launch.check_mesh(fed, args.gpus, bool(args.mesh_virtual), "bench_cnn")
    else:
        fed = Federation.init()
    world, rank = fed.world, fed.rank
    ppr = args.peers // world
    data = synthetic_cifar10(args.n_train, args.n_test, seed=7, similarity=args.similarity, noise=args.noise, modes=args.modes, label_noise=args.label_noise)
    if args.dirichlet > 0:
        parts = data.generate_partitions(args.peers, DirichletPartitionStrategy, alpha=args.dirichlet)
    else:
        parts = data.generate_partitions(args.peers, RandomIIDPartitionStrategy)
    mk = {"fedavg": FedAvg, "fedprox": lambda: FedProx(proximal_mu=args.mu), "neighbor": lambda: NeighborAvg("ring")}[args.aggregator]
    model_cls = ResNet18 if args.model == "resnet18" else LeNet5
    gids = [rank * ppr + j for j in range(ppr)]
    nodes = [Node(TorchModel(model_cls(seed=100 + g)), parts[g], address=f"cnn-{g}", protocol=CollectiveCommunicationProtocol, aggregator=mk(),
                  learner_kwargs={"batch_size": B}) for g in gids]
    for n in nodes:
        n.start()
    fed.finalize()
    engines = [getattr(n.learner, "_engine", None) for n in nodes]
    fused = all(e is not None for e in engines)
    if args.eager and fused:
        engines[0].group.eager = True
    if args.dropout and rank == world - 1:
        fault_injection.kill_at(nodes[-1], "TrainStage", round=min(1, args.warmup + args.rounds - 1))
    total = args.warmup + args.rounds
    marks, round_end = {}, {}
    cuda_devs = sorted({d.index for d in fed.devices if d.type == "cuda"}) if torch.cuda.is_available() else []

    def sync() -> None:  # every device this process drives
        for i in cuda_devs:
            torch.cuda.synchronize(i)

    def start_hook(r, f):  # the first timed round's train set is known, nothing of it launched
        if args.warmup > 0 and r == args.warmup:
            f.barrier()
            sync()
            marks["t0"] = time.perf_counter()

    def hook(r, f):
        round_end[r] = time.perf_counter()
        if r == total - 1:
            sync()
            f.barrier()
            marks["t1"] = time.perf_counter()

    fed.round_start_hooks.append(start_hook)
    fed.round_hooks.append(hook)
    landed: dict = {}  # round -> [(acc, host time the evaluation landed)]
    local_addrs = {n.addr for n in nodes}

    def on_metric(addr, exp_name, rnd, metric, value, step):
        if metric == "test_metric" and step is None and addr in local_addrs:
            landed.setdefault(rnd, []).append((value, time.perf_counter()))

    logger.add_metric_listener(on_metric)
    t_start = time.perf_counter()
    if args.warmup == 0:  # time from the start (includes graph capture)
        marks["t0"] = t_start
    if rank == 0:
        nodes[0].set_start_learning(rounds=total, epochs=1)
    wait_to_finish(nodes, timeout=7200)
    el = marks["t1"] - marks["t0"]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=fed.device)
        fed.all_reduce_(t, op="max")
        el = float(t.item())
    logs = logger.get_global_logs().get("experiment", {})
    # final accuracy: the peers that evaluated the last round (a peer killed by --dropout stopped
    # logging at its death; its stale last value is not the federation's final accuracy)
    last_r = max((r for n in nodes for r, _ in logs.get(n.addr, {}).get("test_metric", [])), default=None)
    accs = [v for n in nodes for r, v in logs.get(n.addr, {}).get("test_metric", []) if r == last_r]
    # accuracy curve: test_metric logged at round r evaluates the model after round r - 1
    by_round: dict = {}
    for n in nodes:
        for r, v in logs.get(n.addr, {}).get("test_metric", []):
            by_round.setdefault(r, []).append(v)
    curve = {r: float(np.mean(v)) for r, v in sorted(by_round.items())}
    # local training loss per round (mean over the local peers of their last logged value)
    loss_curve: dict = {}
    for r, per_node in sorted(logger.get_local_logs().get("experiment", {}).items()):
        vals = [v["train_loss"][-1][1] for a, v in per_node.items() if a in local_addrs and v.get("train_loss")]
        if vals:
            loss_curve[int(r)] = round(float(np.mean(vals)), 4)
    r_target = t_target = None
    for r, a in curve.items():
        if r >= 1 and a >= args.target_acc and r in landed:
            r_target, t_target = r, max(t for _, t in landed[r]) - t_start
            break
    tm = logger.get_timings().get(nodes[0].addr, {})
    brk = {k: round(1000 * float(np.median(v[args.warmup:] or v)), 2) for k, v in tm.items()}
    print(f"[bench_cnn] rank {rank} median ms per call: {json.dumps(brk)}", file=sys.stderr, flush=True)
    # grouped step time from the round time (the engine's fit only enqueues: its host time is not
    # the device time any more)
    steps = (len(parts[gids[0]].column("label")) + B - 1) // B
    step_ms_engine = round(1000 * el / args.rounds / max(1, steps), 3) if fused else None
    for n in nodes:
        n.stop()
    out = {
        "metric": f"rounds/sec, {args.model} {args.aggregator} {args.peers} peers",
        "value": round(args.rounds / el, 4), "unit": "rounds/s", "n_gpus": len(cuda_devs) if fed.mesh is not None else world,
        "launch": "device mesh (one process)" if fed.mesh is not None else ("one process per GPU" if world > 1 else "single"),
        "rounds": args.rounds, "warmup": args.warmup,
        "ms_per_round": round(1000 * el / args.rounds, 2),
        "train_images_per_s": round(args.n_train * args.rounds / el, 1),
        "engine": ("fused-hip" + ("-eager" if args.eager else "-hipgraph")) if fused else "autograd",
        "dtype": "bf16" if fused else "fp32", "data": "synthetic CIFAR-10-shaped uint8", "local_batch": B,
        "partition": f"dirichlet({args.dirichlet})" if args.dirichlet else "iid", "dropout": args.dropout,
        "final_test_acc_mean": round(float(np.mean(accs)), 4) if accs else None,
        "acc_curve": {int(r): round(a, 4) for r, a in curve.items()},
        "train_loss_curve": loss_curve,
        "target_acc": args.target_acc, "rounds_to_target": r_target, "time_to_target_s": None if t_target is None else round(t_target, 3),
        "data_difficulty": {"similarity": args.similarity, "noise": args.noise, "modes": args.modes, "label_noise": args.label_noise},
        "round_ms_per_local_step": step_ms_engine,
        "collective": ("delayed-averaging" if args.delayed_averaging else ("synchronous" if args.no_overlap else "side-stream-bucketed"))
        + f", bucket {Settings.BUCKET_BYTES >> 20} MiB",
    }
    grp = getattr(engines[0], "group", None) if engines and engines[0] is not None else None
    if grp is not None and getattr(grp, "_wsplit", None):
        out["wgrad_splits"] = {k: v[1] for k, v in grp._wsplit.items()}  # device-tuned split-K per conv layer
    if args.torch_step and rank == 0 and torch.cuda.is_available():
        t_ms = torch_step_ms(args.model, B)
        out["torch_bf16_ms_per_peer_step"] = round(t_ms, 3)
        out["torch_ms_for_all_peers_step"] = round(t_ms * ppr, 3)
    if rank == 0:
        print(json.dumps(out), flush=True)
    fed.shutdown()
    if parked_group:
        launch.release_parked()


if __name__ == "__main__":
    main()
