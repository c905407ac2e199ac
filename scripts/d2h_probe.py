#!/usr/bin/env python3
"""PCIe probe for the host-buffer path: device -> page-locked host copy rate of one 65,536-env obs
plane (805 MB), as one copy and split over 2 / 4 streams, into hipHostMalloc'd (torch pinned) memory
and into hipHostRegister'ed pageable memory (what libenv_set_buffers does with the caller's numpy)."""
import ctypes
import json
import time

import numpy as np
import torch

N = 65536 * 64 * 64 * 3
dev = torch.empty(N, dtype=torch.uint8, device="cuda").fill_(7)
pinned = torch.empty(N, dtype=torch.uint8, pin_memory=True)
hip = ctypes.CDLL("libamdhip64.so")
host_np = np.empty(N, np.uint8)
host_np[:] = 1
assert hip.hipHostRegister(ctypes.c_void_p(host_np.ctypes.data), ctypes.c_size_t(N), 0) == 0
registered = torch.from_numpy(host_np)


def rate(dst, parts, reps=5):
    streams = [torch.cuda.Stream() for _ in range(parts)]
    step = (N + parts - 1) // parts
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                dst[k * step:(k + 1) * step].copy_(dev[k * step:(k + 1) * step], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, N / (time.perf_counter() - t0) / 1e9)
    return round(best, 2)


out = {"bytes": N}
for name, dst in (("pinned", pinned), ("registered", registered)):
    out[name] = {"1_stream_GBps": rate(dst, 1), "2_streams_GBps": rate(dst, 2), "4_streams_GBps": rate(dst, 4)}
print(json.dumps(out))
