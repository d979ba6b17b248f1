"""Probe (development): the OBCA batch on a few sizes, with wall times (tools, not shipped)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))
import numpy as np
from piadmm import obca
b = obca.OBCABatch(0)
for n in (8, 64, 300, 4096):
    recs = obca.scenario_batch(n, seed=2)
    t = time.time(); r = b.solve(recs); t1 = time.time() - t
    b.upload(recs); ms = b.time(3); r2 = b.download(n)
    print(n, "solve %.3fs" % t1, "time %.3f ms" % ms, "equal", bool(np.array_equal(r.raw, r2.raw)),
          "status", np.bincount(r.status), flush=True)
b.close()
