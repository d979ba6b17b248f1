"""Probe (development): the per-problem cost spread of the OBCA bench batch (QP steps, SQP
iterations) and how long the slowest problems take alone vs in the full batch (tools, not shipped)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))
import numpy as np
from piadmm import obca
b = obca.OBCABatch(0)
n = 4096
recs = obca.scenario_batch(n, seed=2)
b.upload(recs)
ms = b.time(3)
r = b.download(n)
q = r.qp_steps.astype(float)
it = r.iters.astype(float)
print("batch %d: %.3f ms per launch" % (n, ms))
print("qp steps: mean %.1f p50 %.0f p90 %.0f p99 %.0f max %.0f" % (q.mean(), *np.percentile(q, [50, 90, 99]), q.max()))
print("sqp iters: mean %.2f p50 %.0f p90 %.0f p99 %.0f max %.0f" % (it.mean(), *np.percentile(it, [50, 90, 99]), it.max()))
order = np.argsort(-q, kind="stable")
for k in (1, 8, 32, 128, 512):
    sub = recs[order[:k]]
    bk = obca.OBCABatch(0)
    bk.upload(sub)
    t = bk.time(3)
    bk.close()
    print("slowest %4d alone: %.3f ms  (their qp steps %.0f..%.0f)" % (k, t, q[order[k - 1]], q[order[0]]))
rest = recs[order[32:]]
br = obca.OBCABatch(0)
br.upload(rest)
print("all but the slowest 32: %.3f ms" % br.time(3))
br.close()
b.close()
