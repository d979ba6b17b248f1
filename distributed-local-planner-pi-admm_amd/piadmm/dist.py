"""Multi-GPU sharding: one process per GPU, whole components per rank.

The reference runs every agent in one Python loop (``casadi/main.py:81``,
``for i_veh in range(num_veh)``); nothing is distributed.  Here the agents of
a scenario are split over ranks by connected component of the candidate-pair
graph; a component never straddles ranks.

* per-component termination (default): the outer loop of a rank needs nothing
  from any other rank -- no data-path collective.
* ``term_global`` (the reference's global flag / termination, quirk B9): the
  library all-reduces the termination partials over RCCL (xGMI) once per outer
  iteration -- or the residual history once per MPC step when ``fixed_iters`` --
  through the communicator :func:`attach_rccl` sets up.

The harness (bench.py) uses torch.distributed (gloo) only for its barrier,
max-over-ranks timing and to ship the RCCL unique id.
"""
from __future__ import annotations

import numpy as np

from .scenario import Scenario


def component_ranges(scn: Scenario):
    """(start, stop) agent ranges of the components, in agent order (components are contiguous)."""
    comp, n_comp = scn.components()
    if np.any(np.diff(comp) < 0) or np.any(np.diff(comp) > 1):
        raise ValueError("components must be contiguous agent ranges in agent order")
    starts = np.searchsorted(comp, np.arange(n_comp))
    stops = np.append(starts[1:], scn.n_agents)
    return list(zip(starts.tolist(), stops.tolist()))


def shard_bounds(scn: Scenario, rank: int, world: int):
    """Contiguous block of components for ``rank``: balanced by agent count."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    rngs = component_ranges(scn)
    N = scn.n_agents
    # assign component k to the rank whose share of agents its start falls in
    owner = [min(world - 1, (a0 * world) // N) for a0, _ in rngs]
    mine = [r for r, o in zip(rngs, owner) if o == rank]
    if not mine:
        return 0, 0
    return mine[0][0], mine[-1][1]


def shard(scn: Scenario, rank: int, world: int) -> Scenario:
    """The sub-scenario of ``rank`` (agents renumbered from 0; pairs kept)."""
    a0, a1 = shard_bounds(scn, rank, world)
    sel = (scn.edges[:, 0] >= a0) & (scn.edges[:, 1] < a1)
    cross = ((scn.edges[:, 0] < a1) & (scn.edges[:, 1] >= a1)) | ((scn.edges[:, 0] < a0) & (scn.edges[:, 1] >= a0))
    if np.any(cross):
        raise ValueError("a candidate pair straddles two ranks")
    return Scenario(spd=scn.spd[a0:a1].copy(), xt0=scn.xt0[a0:a1].copy(), ref=scn.ref[a0:a1].copy(),
                    edges=(scn.edges[sel] - a0).astype(np.int32), n_steps=scn.n_steps)


def attach_rccl(solver, rank: int, world: int, broadcast_bytes):
    """Create the RCCL communicator of a sharded job on ``solver`` (a PI_ADMM_MI355X).

    ``broadcast_bytes(b: bytes | None) -> bytes`` ships rank 0's 128-byte unique id to every
    rank over any out-of-band channel (bench.py uses torch.distributed's gloo group)."""
    from .solver import comm_unique_id
    uid = comm_unique_id() if rank == 0 else None
    uid = broadcast_bytes(uid)
    solver.comm_init(uid, world, rank)
