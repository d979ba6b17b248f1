"""Host CPU facts for the CPU baselines of bench.py (MEASUREMENT INFRASTRUCTURE ONLY).

The cores a baseline uses are shown, not asserted: the CPUs this process may run on
(``os.sched_getaffinity``), the cgroup CPU quota (``cpu.max``, cgroup v2, or
``cpu.cfs_quota_us / cpu.cfs_period_us``, v1), the ``OMP_NUM_THREADS`` share the environment gives,
and the CPU model name (``/proc/cpuinfo``, what ``lscpu`` prints as "Model name").  The baseline
threads = every core the process may run on, capped by the quota and the OMP share when those
are set (a shared GPU box gives each GPU a fixed CPU share: running more threads than the quota
would only time-slice them).
"""
from __future__ import annotations

import math
import os


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cgroup_quota():
    """(text, cores) of the cgroup CPU quota, cores = None when unlimited / unknown."""
    v2 = _read("/sys/fs/cgroup/cpu.max")
    if v2:
        parts = v2.split()
        if parts[0] != "max" and len(parts) == 2 and float(parts[1]) > 0:
            return v2, float(parts[0]) / float(parts[1])
        return v2, None
    q, p = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    if q and p:
        txt = f"cfs_quota_us={q} cfs_period_us={p}"
        if int(q) > 0 and int(p) > 0:
            return txt, int(q) / int(p)
        return txt, None
    return None, None


def cpu_model():
    txt = _read("/proc/cpuinfo") or ""
    for line in txt.splitlines():
        if line.lower().startswith("model name"):
            return line.split(":", 1)[1].strip()
    return None


def host_cpu() -> dict:
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota_txt, quota = cgroup_quota()
    omp = os.environ.get("OMP_NUM_THREADS")
    omp_n = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    threads, rule = affinity, "sched_getaffinity"
    if quota is not None and math.floor(quota) < threads:
        threads, rule = max(1, math.floor(quota)), "cgroup cpu.max quota"
    if omp_n is not None and omp_n < threads:
        threads, rule = omp_n, "OMP_NUM_THREADS share"
    return {"threads": threads, "rule": rule, "sched_getaffinity": affinity, "cgroup_cpu_max": quota_txt,
            "omp_num_threads": omp, "cpus_visible": os.cpu_count(), "model_name": cpu_model()}


def describe(h: dict) -> str:
    return (f"{h['threads']} threads ({h['rule']}): process may run on {h['sched_getaffinity']} cpus "
            f"(sched_getaffinity), cgroup cpu.max {h['cgroup_cpu_max']!r}, OMP_NUM_THREADS "
            f"{h['omp_num_threads']!r}, {h['cpus_visible']} cpus visible, model {h['model_name']!r}")
