"""The host CPUs a process may use, and how the bulk calls divide them among their shards.

Each shard of a bulk call runs on its own context, and each context runs its own reader / copy threads
(TV_OPT_FILE_THREADS, default 16, shared by its two staging lanes).  Without a budget, devices=[0..7] would start
8 x 16 reader threads whatever the process's CPU share.  shard_threads() gives each
concurrently active shard its part of the share: the cgroup quota (or the box's stated share, or the affinity
mask) divided by the active shards, and no more than the CPUs of the shard's NUMA node (where the library runs
its threads: the NUMA binding option) divided by the active shards on that node; capped at 16 (the library's default,
where the page-cache reads already saturate PCIe: profiles/r05/f2_stamps_*.jsonl) and at least 1.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

MAX_THREADS_PER_SHARD = 16


def cpu_share() -> dict:
    """The host cores this process may use: the cgroup CPU quota (cpu.max, v2; cfs_quota_us, v1) when one
    is set, else the box's CPU share as its environment states it (OMP_NUM_THREADS; 16 per GPU on the
    GPU boxes), else the affinity mask.  Everything it looked at is reported."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if quota:
        cores, src = max(1, min(aff, int(quota))), "cgroup CPU quota"
    elif omp and omp.isdigit() and int(omp) > 0:
        cores, src = min(aff, int(omp)), "OMP_NUM_THREADS (the box's stated CPU share; no cgroup quota)"
    else:
        cores, src = aff, "sched_getaffinity (no cgroup quota, no stated share)"
    return {"cores": cores, "source": src, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
            "omp_num_threads": omp}


def node_cpus(node: Optional[int]) -> Optional[int]:
    """CPUs of NUMA node `node` this process may run on (sysfs cpulist & affinity); None when unknown."""
    if node is None or node < 0:
        return None
    try:
        txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return None
    cpus = set()
    for part in txt.split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    n = len(cpus & os.sched_getaffinity(0))
    return n or None


def shard_threads(nodes: Sequence[Optional[int]], share: Optional[int] = None,
                  node_cpu_count: Optional[Dict[int, Optional[int]]] = None) -> List[int]:
    """Reader threads for each of the concurrently active shards whose GPUs sit on NUMA `nodes` (None: unknown).
    sum(result) <= max(share, len(nodes)) (every shard gets at least one thread)."""
    n = len(nodes)
    if n == 0:
        return []
    if share is None:
        share = cpu_share()["cores"]
    per = max(1, share // n)
    on_node: Dict[Optional[int], int] = {}
    for nd in nodes:
        on_node[nd] = on_node.get(nd, 0) + 1
    out = []
    for nd in nodes:
        t = per
        cpus = (node_cpu_count or {}).get(nd) if node_cpu_count is not None else node_cpus(nd)
        if nd is not None and cpus:
            t = min(t, max(1, cpus // on_node[nd]))
        out.append(max(1, min(MAX_THREADS_PER_SHARD, t)))
    return out
