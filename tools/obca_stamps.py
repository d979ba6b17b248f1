"""Per-phase cycle breakdown of the OBCA SQP kernel (diagnostic stamps build, run on the GPU box):
PIADMM_LIB=distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_stamps.so python tools/obca_stamps.py [n]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-local-planner-pi-admm_amd"))
from piadmm import obca  # noqa: E402

NAMES = ["linearise", "condense", "hessian", "rows", "modify", "gi", "recover", "linesearch", "init", "out",
         "n_chol", "n_active_end", "qp_steps", "n_trial", "n_sqp", "total"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
b = obca.OBCABatch(0)
recs = obca.scenario_batch(n)
b.upload(recs)
ms = b.time(1)
st = np.zeros(n * 16, np.uint64)
b._check(b._lib.piadmm_obca_debug_stamps(b._h, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n * 16))
st = st.reshape(n, 16).astype(np.float64)
res = b.download(n)
print(f"batch {n}: {ms:.2f} ms per launch, sqp iters mean {res.iters.mean():.2f}, qp steps mean {res.qp_steps.mean():.1f}")
tot = st[:, 15].mean()
for k, name in enumerate(NAMES):
    v = st[:, k].mean()
    if k < 10:
        print(f"{name:12s} {v:12.0f} cycles/problem  {100 * v / tot:5.1f}%  per sqp iter {v / max(st[:, 14].mean(), 1):10.0f}")
    else:
        print(f"{name:12s} {v:12.2f}")

# calibration: launch time vs batch size (768 = 3 workgroups x 256 CUs in flight) and the stamps'
# mean / max total per problem -> the stamp clock's rate
for nb in (64, 256, 768, 1536, 4096):
    bb = obca.OBCABatch(0)
    rr = obca.scenario_batch(nb)
    bb.upload(rr)
    bb.time(1)
    t = bb.time(3)
    s2 = np.zeros(nb * 16, np.uint64)
    bb._check(bb._lib.piadmm_obca_debug_stamps(bb._h, s2.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nb * 16))
    s2 = s2.reshape(nb, 16).astype(np.float64)
    print(f"n={nb:5d}: {t:7.3f} ms/launch, stamp total mean {s2[:, 15].mean():.0f} max {s2[:, 15].max():.0f} "
          f"-> max/time = {s2[:, 15].max() / (t * 1e-3) / 1e6:.0f} M ticks/s")
    bb.close()
