"""Cost of HIP stream creation vs torch pool streams (node-start budget, profiles/r5_start)."""
import ctypes
import json
import time

import torch

torch.zeros(1, device="cuda")
torch.cuda.synchronize()
hip = ctypes.CDLL("libamdhip64.so")
out = {}
for i in range(4):
    s = ctypes.c_void_p()
    t = time.perf_counter()
    rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    out[f"hipStreamCreate_{i}"] = round(1e3 * (time.perf_counter() - t), 3)
    t = time.perf_counter()
    ev = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    hip.hipEventRecord(ev, s)
    hip.hipStreamSynchronize(s)
    out[f"first_use_{i}"] = round(1e3 * (time.perf_counter() - t), 3)
for i in range(4):
    t = time.perf_counter()
    st = torch.cuda.Stream()
    out[f"torch_stream_{i}"] = round(1e3 * (time.perf_counter() - t), 3)
    t = time.perf_counter()
    e = torch.cuda.Event()
    e.record(st)
    st.synchronize()
    out[f"torch_first_use_{i}"] = round(1e3 * (time.perf_counter() - t), 3)
for i in range(3):
    s = ctypes.c_void_p()
    t = time.perf_counter()
    hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    out[f"late_hipStreamCreate_{i}"] = round(1e3 * (time.perf_counter() - t), 3)
print(json.dumps(out))
