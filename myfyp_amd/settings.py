"""Global, mutable framework settings.

Parity with the reference ``Settings`` class (``p2pfl/settings.py:28-153``): every flat
attribute keeps its name and default so existing experiment scripts keep working.

Additions (MI355X-first):

* nested groups (``Settings.general.SEED``, ``Settings.training.BATCH_SIZE`` ...) that alias the
  flat names — the FYP scripts use the nested API (``exp_SAVE3.txt:74``);
* device/engine knobs for the GPU data plane (batch size, compute dtype, grouped peers);
* a YAML/JSON experiment loader (``Settings.from_yaml``) — the reference has none.
"""

from __future__ import annotations

import os
from typing import Optional, Any, Dict

_CERT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "certificates")


class _Group:
    """A nested settings group whose attributes alias flat ``Settings`` attributes."""

    def __init__(self, mapping: Dict[str, str]) -> None:
        object.__setattr__(self, "_mapping", mapping)

    def __getattr__(self, name: str) -> Any:
        mapping = object.__getattribute__(self, "_mapping")
        if name in mapping:
            return getattr(Settings, mapping[name])
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        mapping = object.__getattribute__(self, "_mapping")
        if name not in mapping:
            raise AttributeError(f"Unknown setting {name!r}")
        setattr(Settings, mapping[name], value)

    def __dir__(self):  # pragma: no cover - convenience
        return list(object.__getattribute__(self, "_mapping"))


class Settings:
    """Class-level global settings (mutated at runtime, like the reference)."""

    # ---------------- GENERAL (p2pfl/settings.py:34-50)
    GRPC_TIMEOUT: float = 10
    LOG_LEVEL: str = "INFO"
    LOG_DIR: str = "logs"
    EXCLUDE_BEAT_LOGS: bool = True
    DISABLE_RAY: bool = True  # Ray is replaced by the device pool; kept for API compatibility.
    SEED: int | None = None

    # ---------------- HEARTBEAT (p2pfl/settings.py:58-62)
    HEARTBEAT_PERIOD: float = 2
    HEARTBEAT_TIMEOUT: float = 5

    # ---------------- GOSSIP (p2pfl/settings.py:70-94)
    GOSSIP_PERIOD: float = 0.1
    TTL: int = 10
    GOSSIP_MESSAGES_PER_PERIOD: int = 100
    AMOUNT_LAST_MESSAGES_SAVED: int = 100
    GOSSIP_MODELS_PERIOD: float = 1
    GOSSIP_MODELS_PER_ROUND: int = 2
    GOSSIP_EXIT_ON_X_EQUAL_ROUNDS: int = 10

    # ---------------- SSL (p2pfl/settings.py:102-125)
    USE_SSL: bool = False
    CA_CRT: str = f"{_CERT_DIR}/ca.crt"
    SERVER_CRT: str = f"{_CERT_DIR}/server.crt"
    CLIENT_CRT: str = f"{_CERT_DIR}/client.crt"
    SERVER_KEY: str = f"{_CERT_DIR}/server.key"
    CLIENT_KEY: str = f"{_CERT_DIR}/client.key"

    # ---------------- TRAINING (p2pfl/settings.py:130-142)
    TRAIN_SET_SIZE: int = 4
    VOTE_TIMEOUT: float = 60
    AGGREGATION_TIMEOUT: float = 300
    WAIT_HEARTBEATS_CONVERGENCE: float = 0.2 * HEARTBEAT_TIMEOUT

    # ---------------- WEB (p2pfl/settings.py:150)
    RESOURCE_MONITOR_PERIOD: float = 1

    # ---------------- DEVICE / ENGINE (new: MI355X data plane)
    DEVICE: str = "auto"  # "auto" -> cuda if available else cpu
    BATCH_SIZE: int = 1  # reference default (lightning_dataset.py:81); benchmarks override it
    COMPUTE_DTYPE: str = "bf16"  # CNN engines' GEMM operand dtype (fp32 master weights; BASELINE config 4 is bf16)
    # fused MLP engine precision: "fp32" = the reference's (Lightning default fp32 Trainer): exact
    # fp32 products, fp32 accumulation / weights / optimizer state; "bf16" = bf16 MFMA operands
    MLP_PRECISION: str = "fp32"
    USE_FUSED_KERNELS: bool = True  # hand-written HIP path when the extension is present
    GROUP_PEERS: bool = True  # train co-located peers in one grouped launch
    GANG_WINDOW: float = 0.05  # seconds a grouped fit waits for expected co-located peers
    COLLECTIVE_TIMEOUT: float = 300  # RCCL watchdog (seconds)
    # a rank whose control-plane heartbeat is older than this is evicted from the federation (s)
    FAILURE_TIMEOUT: float = 60
    # all-reduce bucket size: large enough that each ring step is bandwidth-bound on the xGMI links,
    # small enough that a 45 MB ResNet-18 buffer pipelines (bucket k's all-reduce overlaps bucket
    # k+1's reduce kernel and bucket k-1's apply kernel on the side stream)
    BUCKET_BYTES: int = 16 << 20
    # stacked-group FedAvg runs on a side HIP stream, bucketed and pipelined (exact numerics)
    OVERLAP_COLLECTIVES: bool = True
    # opt-in delayed averaging (SURVEY §7.4 hard part 4b): the next round trains from the local
    # weights while the all-reduce runs; the averaged delta lands at the next aggregation
    # (x += avg_r - x_r); the last round aggregates exactly. Changes numerics.
    DELAYED_AVERAGING: bool = False
    # ranks > 0 ship their metrics to rank 0 live, every this many seconds (0 disables the relay)
    CENTRAL_LOG_PERIOD: float = 0.5
    SHM_CONTROL_PLANE: bool = True  # single-node jobs: control-plane gathers through shared memory
    # a single-process job still runs its weight collectives through a world-size-1 RCCL group (the
    # multi-rank code path on one GPU: profiling, tests); env MYFYP_FORCE_COLLECTIVE=1 does the same
    FORCE_COLLECTIVE: bool = False
    # failure-aware weight collectives (single-node shm control plane): liveness polled while
    # waiting, watchdog abort, agreement on every collective, re-run over the survivors
    COLLECTIVE_FAILOVER: bool = True
    # deferred confirmation of the device weight collectives (parallel/federation.py
    # confirm_collectives): the newest one, if not yet complete, waits one more weights section
    # instead of blocking the round driver until the GPU reaches it (the host stays up to two rounds
    # ahead; a failure is then recovered one round later). MYFYP_CONFIRM_LAG=0: block as before
    CONFIRM_LAG: bool = True
    # Channels RCCL may use per collective. RCCL launches one workgroup per channel, so this is also
    # the number of CUs a concurrent RCCL kernel can hold. Federation.init exports it as RCCL's own
    # NCCL_MAX_NCHANNELS / NCCL_MAX_CTAS caps unless the environment already sets them; the cap
    # the process ends up with is what the persistent epoch reserves (rccl_reserved_cus). 32
    # channels is ample for the latency-bound 0.94 MB MLP all-reduce and for ResNet-18's 22 MB.
    RCCL_MAX_CHANNELS: int = 32
    # CUs the fp32 MLP persistent epoch leaves to a concurrent RCCL kernel when collectives are
    # active (co-residency: every workgroup of a gang must be resident at once). None: derived from
    # the RCCL channel cap in force (see RCCL_MAX_CHANNELS)
    RCCL_RESERVED_CUS: Optional[int] = None
    # in-process device mesh (parallel/device_mesh.py): ONE process drives this many GPUs, peers
    # placed round-robin, weights over an in-process RCCL mesh (ncclCommInitAll). 1 = off; env
    # MYFYP_MESH_DEVICES overrides. MESH_BACKEND: None (RCCL on distinct GPUs, else host torch ops),
    # "rccl" or "host". MESH_VIRTUAL: a count above the visible GPUs puts every member on cuda:0
    # (one-GPU rehearsal with host collectives) instead of raising.
    MESH_DEVICES: int = 1
    MESH_BACKEND: Optional[str] = None
    MESH_VIRTUAL: bool = False
    # an RCCL mesh over distinct physical GPUs that fails to form raises; True swaps in the host
    # mesh (device-to-device copies), reported as mesh.kind == "host" (benchmarks refuse it)
    MESH_HOST_FALLBACK: bool = False
    # Node.start() prepares the fused engine (epoch-graph capture and upload, code-object load; no
    # training work) so round 0 does not pay it — like building a compiled model at load time
    ENGINE_PREWARM: bool = True
    # interpreter GIL switch interval (s) set by Federation.init: co-located peer threads hand the
    # GIL over often, and a thread returning from a device call waits up to this long for it
    GIL_SWITCH_INTERVAL: float | None = 2e-4
    # objects alive when an experiment starts go to the collector's permanent generation for its
    # duration (utils/gc_tuning.py): no full collection re-walks them mid-run
    GC_FREEZE: bool = True
    # collective workflow: evaluate + fit + FedAvg of co-located fused-engine peers as ONE gang op
    FUSED_ROUND: bool = True
    # ... and the rounds of all co-located fused peers are driven by ONE host thread (driver.py)
    ROUND_DRIVER: bool = True

    # ---------------- SIMULATION (Ray actor pool → device pool, learning/frameworks/simulation)
    SIMULATION_POOL: bool = False  # True: learners run fit/evaluate as jobs on per-device worker streams
    SIMULATION_RESOURCES: Dict[str, float] | None = None  # per virtual client, e.g. {"num_cpus": 1, "num_gpus": 0.25}
    SIMULATION_WORKERS_PER_GPU: int = 4  # default pool shape when GPUs are visible

    # ---------------- DEBUG (new: SURVEY §5.1/§5.2)
    LOCK_CHECK: bool | str = False  # True/"record": lock-order inversions recorded; "raise": raised (utils/lockcheck.py)
    TRACE_MARKERS: bool = False  # roctx ranges around fit / evaluate / aggregation / stages (management/tracing.py)

    # ---------------- CHECKPOINT (new: SURVEY §5.4)
    CHECKPOINT_DIR: str | None = None  # None = off; else save every CHECKPOINT_EVERY rounds
    CHECKPOINT_EVERY: int = 1

    # nested aliases (FYP scripts: Settings.general.SEED)
    general = _Group(
        {
            "SEED": "SEED",
            "GRPC_TIMEOUT": "GRPC_TIMEOUT",
            "LOG_LEVEL": "LOG_LEVEL",
            "LOG_DIR": "LOG_DIR",
            "EXCLUDE_BEAT_LOGS": "EXCLUDE_BEAT_LOGS",
            "DISABLE_RAY": "DISABLE_RAY",
            "SIMULATION_POOL": "SIMULATION_POOL",
            "SIMULATION_RESOURCES": "SIMULATION_RESOURCES",
            "SIMULATION_WORKERS_PER_GPU": "SIMULATION_WORKERS_PER_GPU",
            "CHECKPOINT_DIR": "CHECKPOINT_DIR",
            "CHECKPOINT_EVERY": "CHECKPOINT_EVERY",
        }
    )
    heartbeat = _Group({"PERIOD": "HEARTBEAT_PERIOD", "TIMEOUT": "HEARTBEAT_TIMEOUT", "WAIT_CONVERGENCE": "WAIT_HEARTBEATS_CONVERGENCE"})
    gossip = _Group(
        {
            "PERIOD": "GOSSIP_PERIOD",
            "TTL": "TTL",
            "MESSAGES_PER_PERIOD": "GOSSIP_MESSAGES_PER_PERIOD",
            "AMOUNT_LAST_MESSAGES_SAVED": "AMOUNT_LAST_MESSAGES_SAVED",
            "MODELS_PERIOD": "GOSSIP_MODELS_PERIOD",
            "MODELS_PER_ROUND": "GOSSIP_MODELS_PER_ROUND",
            "EXIT_ON_X_EQUAL_ROUNDS": "GOSSIP_EXIT_ON_X_EQUAL_ROUNDS",
        }
    )
    ssl = _Group(
        {
            "USE_SSL": "USE_SSL",
            "CA_CRT": "CA_CRT",
            "SERVER_CRT": "SERVER_CRT",
            "CLIENT_CRT": "CLIENT_CRT",
            "SERVER_KEY": "SERVER_KEY",
            "CLIENT_KEY": "CLIENT_KEY",
        }
    )
    training = _Group(
        {
            "TRAIN_SET_SIZE": "TRAIN_SET_SIZE",
            "VOTE_TIMEOUT": "VOTE_TIMEOUT",
            "AGGREGATION_TIMEOUT": "AGGREGATION_TIMEOUT",
            "BATCH_SIZE": "BATCH_SIZE",
        }
    )
    device = _Group(
        {
            "DEVICE": "DEVICE",
            "COMPUTE_DTYPE": "COMPUTE_DTYPE",
            "MLP_PRECISION": "MLP_PRECISION",
            "USE_FUSED_KERNELS": "USE_FUSED_KERNELS",
            "GROUP_PEERS": "GROUP_PEERS",
            "GANG_WINDOW": "GANG_WINDOW",
            "COLLECTIVE_TIMEOUT": "COLLECTIVE_TIMEOUT",
            "FAILURE_TIMEOUT": "FAILURE_TIMEOUT",
            "BUCKET_BYTES": "BUCKET_BYTES",
            "OVERLAP_COLLECTIVES": "OVERLAP_COLLECTIVES",
            "DELAYED_AVERAGING": "DELAYED_AVERAGING",
            "CENTRAL_LOG_PERIOD": "CENTRAL_LOG_PERIOD",
            "SHM_CONTROL_PLANE": "SHM_CONTROL_PLANE",
            "FORCE_COLLECTIVE": "FORCE_COLLECTIVE",
            "COLLECTIVE_FAILOVER": "COLLECTIVE_FAILOVER",
            "CONFIRM_LAG": "CONFIRM_LAG",
            "RCCL_RESERVED_CUS": "RCCL_RESERVED_CUS",
            "RCCL_MAX_CHANNELS": "RCCL_MAX_CHANNELS",
            "ENGINE_PREWARM": "ENGINE_PREWARM",
            "GIL_SWITCH_INTERVAL": "GIL_SWITCH_INTERVAL",
            "GC_FREEZE": "GC_FREEZE",
            "FUSED_ROUND": "FUSED_ROUND",
            "ROUND_DRIVER": "ROUND_DRIVER",
            "MESH_DEVICES": "MESH_DEVICES",
            "MESH_BACKEND": "MESH_BACKEND",
            "MESH_VIRTUAL": "MESH_VIRTUAL",
            "MESH_HOST_FALLBACK": "MESH_HOST_FALLBACK",
        }
    )

    # ------------------------------------------------------------------ helpers
    @classmethod
    def snapshot(cls) -> Dict[str, Any]:
        """Return all flat settings as a plain dict (checkpoint sidecars, logging)."""
        out: Dict[str, Any] = {}
        for k in dir(cls):
            if k.isupper():
                v = getattr(cls, k)
                if isinstance(v, (int, float, str, bool)) or v is None:
                    out[k] = v
        return out

    @classmethod
    def update(cls, values: Dict[str, Any]) -> None:
        """Apply a dict of settings. Keys may be flat (``HEARTBEAT_PERIOD``) or nested dicts
        (``{"general": {"SEED": 1}}``)."""
        for k, v in values.items():
            group = getattr(cls, k.lower(), None) if isinstance(v, dict) else None
            if isinstance(group, _Group):
                for gk, gv in v.items():
                    setattr(group, gk.upper(), gv)
                continue
            key = k.upper()
            if not hasattr(cls, key):
                raise KeyError(f"Unknown setting {k!r}")
            setattr(cls, key, v)

    @classmethod
    def from_yaml(cls, path: str) -> Dict[str, Any]:
        """Load an experiment file. The ``settings`` section is applied to ``Settings``; the
        whole parsed document is returned so callers (CLI) can read the experiment section."""
        import yaml

        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        if "settings" in doc:
            cls.update(doc["settings"])
        return doc


def resolve_device() -> str:
    """Resolve ``Settings.DEVICE`` ("auto" → ``cuda`` when a GPU is visible)."""
    if Settings.DEVICE != "auto":
        return Settings.DEVICE
    try:
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"
    except Exception:  # pragma: no cover
        return "cpu"
