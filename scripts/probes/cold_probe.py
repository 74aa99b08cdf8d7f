"""First process on a fresh box: what costs time the first time (device init, first allocations,
first host-to-device copies, code-object load of the native library). One JSON line."""

import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
t = time.perf_counter()
import numpy as np  # noqa: E402
import torch  # noqa: E402

out = {"import_torch_ms": round(1e3 * (time.perf_counter() - t), 2)}


def step(name, fn):
    torch.cuda.synchronize() if torch.cuda.is_initialized() else None
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    out[name] = round(1e3 * (time.perf_counter() - t0), 2)
    return r


step("init_tiny", lambda: torch.zeros(1, device="cuda"))
from myfyp_amd.ops import _native  # noqa: E402

lib = step("native_load", lambda: _native.load(required=True))
a = step("alloc_64MB_1", lambda: torch.empty(64 << 20, dtype=torch.uint8, device="cuda"))
b = step("alloc_64MB_2", lambda: torch.empty(64 << 20, dtype=torch.uint8, device="cuda"))
del a, b
c = step("alloc_64MB_reuse", lambda: torch.empty(64 << 20, dtype=torch.uint8, device="cuda"))
del c
h = np.random.default_rng(0).integers(0, 255, size=(60000, 784), dtype=np.uint8)
x1 = step("h2d_pageable_47MB_1", lambda: torch.from_numpy(h).to("cuda"))
x2 = step("h2d_pageable_47MB_2", lambda: torch.from_numpy(h).to("cuda"))
hp = step("pin_alloc_47MB", lambda: torch.empty(h.shape, dtype=torch.uint8, pin_memory=True))
step("pin_fill", lambda: hp.numpy().__setitem__(slice(None), h))
x3 = step("h2d_pinned_47MB", lambda: hp.to("cuda", non_blocking=True))
small = [np.ascontiguousarray(h[i * 7500:(i + 1) * 7500]) for i in range(8)]
step("h2d_pageable_8x5.9MB", lambda: [torch.from_numpy(s).to("cuda") for s in small])
step("first_kernel_fedavg", lambda: torch.zeros(8, 1024, device="cuda").sum(0))
streams = []
for i in range(5):
    step(f"stream_create_{i}", lambda: streams.append(torch.cuda.Stream()))
evs = []
step("events_x8", lambda: [evs.append(torch.cuda.Event()) for _ in range(8)])
step("warm_all", lambda: lib.myfyp_warm_all(3))
print(json.dumps(out), flush=True)
