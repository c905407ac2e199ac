"""Runs scripts/d2h_probe2.hip's probe (d2h_probe2.so) inside this Python process, after torch has
initialised its HIP context on the device (argv[1] == "torch"), with only torch's bundled HIP runtime
loaded ("torchlib") or without torch ("plain"): do the engine's D2H
copies turn into blit kernels because of something the torch process sets up?  Run under rocprofv3
--kernel-trace --memory-copy-trace."""
import ctypes
import os
import sys

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
if mode == "torchlib":  # torch's bundled HIP runtime, without torch
    ctypes.CDLL(os.path.join(os.path.dirname(__import__("importlib.util").util.find_spec("torch").origin), "lib",
                             "libamdhip64.so"), mode=ctypes.RTLD_GLOBAL)
if mode == "torch":
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "d2h_probe2.so"))
rc = lib.d2h_probe()
import numpy as np  # noqa: E402
buf = np.empty(32768 * 12288, np.uint8)
lib.d2h_probe_host.argtypes = [ctypes.c_void_p]
rc = rc or lib.d2h_probe_host(buf.ctypes.data)
if mode == "torch":
    torch.cuda.synchronize()
sys.exit(rc)
