"""One-off: which pixels of a rendered frame differ from the oracle (game, envs from argv), and the
entity rects drawn there -- for debugging a render-kernel change."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "procgen-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

game = sys.argv[1] if len(sys.argv) > 1 else "coinrun"
num = int(sys.argv[2]) if len(sys.argv) > 2 else 8
torch.cuda.set_device(0)
from procgen_amd import ProcgenGym3Env  # noqa: E402
from oracle_lib import OracleEnv  # noqa: E402
kw = dict(num_levels=200, start_level=0, rand_seed=0) if game == "coinrun" else dict(num_levels=0, rand_seed=3)
env = ProcgenGym3Env(num=num, env_name=game, **kw)
orc = OracleEnv(game, num, **kw)
_, ob, _ = env.observe()
o = orc.observe()["rgb"]
for e in range(num):
    d = np.argwhere(np.any(ob["rgb"][e] != o[e], axis=-1))
    print("env", e, "diff px", len(d))
    if len(d):
        ys, xs = d[:, 0], d[:, 1]
        print("  rows", ys.min(), ys.max(), "cols", xs.min(), xs.max())
        for (y, x) in d[:12]:
            print("   ", y, x, ob["rgb"][e][y, x].tolist(), o[e][y, x].tolist())
np.savez_compressed(os.path.join(REPO, "gpurun_out", "diag_stamp.npz"), got=ob["rgb"], exp=o)
env.close()
if os.environ.get("PG_DIAG_PROF"):
    from procgen_amd import _lib
    lib = _lib.load()
    env2 = ProcgenGym3Env(num=num, env_name=game, **kw)
    raw = np.zeros((num, 16), np.uint64)
    lib.procgen_profile_raw(env2._handle, raw.ctypes.data)
    for e in range(num):
        r = raw[e]
        print("dbg env", e, "total", int(r[0]), "incl0", int(r[1]), "cnt0", int(r[2]), "exn", int(r[3]), "eyn", int(r[4]),
              "bm %x run %x smask %x f0 %x live %x" % (int(r[5]), int(r[6]), int(r[7]), int(r[8]), int(r[9])),
              "y0", int(r[10]), "eyt1", int(r[11]), "ext1", int(r[12]), "calls", int(r[13]))
