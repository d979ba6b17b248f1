"""Multi-GPU sharding: one process per GPU.

The reference runs every agent in one Python loop (``casadi/main.py:81``,
``for i_veh in range(num_veh)``); nothing is distributed.  Two ways to split a job:

* :func:`shard` -- whole connected components of the candidate-pair graph per rank.
  Per-component termination needs nothing from any other rank; ``term_global`` (the
  reference's global flag / termination, quirk B9) all-reduces the termination
  partials over RCCL (xGMI) once per outer iteration -- or the residual history once
  per MPC step when ``fixed_iters`` -- through the communicator :func:`attach_rccl`
  sets up.
* :func:`shard_graph` -- any assignment of agents to ranks: candidate
  pairs may cross ranks.  A rank holds its own agents plus a *ghost* copy of each
  neighbour owned elsewhere; every outer iteration the boundary agents' positions and
  controls travel in one all-reduce of a job-wide exchange buffer (each slot written by
  its owner, zero elsewhere), then both ranks of a cross-rank pair solve its pair QP
  bit-identically; its residual counts on the rank of its first agent.

The harness (bench.py) uses torch.distributed (gloo) only for its barrier,
max-over-ranks timing and to ship the RCCL unique id.
"""
from __future__ import annotations

import dataclasses

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


# ----------------------------------------------------------------------- pairs across ranks
@dataclasses.dataclass
class Shard:
    """One rank's part of a job sharded by agent (pairs may cross ranks)."""
    rank: int
    world: int
    scn: Scenario          # local scenario: own agents + ghosts (increasing global id), own pairs
    agents: np.ndarray     # (n_local,) global id of each local agent
    edges: np.ndarray      # (e_local,) global id of each local pair
    owned: np.ndarray      # (n_local,) uint8: 1 own agent, 0 ghost
    counted: np.ndarray    # (e_local,) uint8: this rank counts the pair's residual terms
    slot: np.ndarray       # (n_local,) int32: exchange-buffer slot (-1: interior agent)
    n_slots: int           # boundary agents in the whole job

    @property
    def own(self) -> np.ndarray:
        """Global ids of the rank's own agents (increasing)."""
        return self.agents[self.owned == 1]


def owners_blocks(n_agents: int, world: int) -> np.ndarray:
    """Contiguous agent blocks per rank (the tiled scenario: tiles never straddle when the
    block size is even)."""
    return np.minimum(world - 1, (np.arange(n_agents) * world) // n_agents).astype(np.int32)


def owners_interleaved(n_agents: int, world: int) -> np.ndarray:
    """Agent a on rank a % world -- the adversarial split of SURVEY.md 8d C4: every
    two-vehicle tile straddles two ranks."""
    return (np.arange(n_agents) % world).astype(np.int32)


def boundary_slots(scn: Scenario, owner: np.ndarray):
    """Job-wide exchange slots: agents with a candidate neighbour on another rank, numbered in
    increasing agent id.  Returns (slot (N,), n_slots)."""
    owner = np.asarray(owner)
    bnd = np.zeros(scn.n_agents, bool)
    if scn.n_edges:
        v1, v2 = scn.edges[:, 0], scn.edges[:, 1]
        cross = owner[v1] != owner[v2]
        bnd[v1[cross]] = True
        bnd[v2[cross]] = True
    slot = np.full(scn.n_agents, -1, np.int32)
    slot[bnd] = np.arange(int(bnd.sum()), dtype=np.int32)
    return slot, int(bnd.sum())


def shard_graph(scn: Scenario, rank: int, world: int, owner: np.ndarray | None = None) -> Shard:
    """The local scenario of ``rank`` when agent a belongs to rank ``owner[a]`` (default:
    :func:`owners_blocks`).  Local agents are the rank's own agents and the ghosts (neighbours
    owned elsewhere) in increasing global id; local pairs are the pairs with an own agent, in
    increasing global pair id (the residual-sum order, casadi/main.py:165-173)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    N = scn.n_agents
    owner = owners_blocks(N, world) if owner is None else np.asarray(owner, np.int32)
    if owner.shape != (N,) or owner.min(initial=0) < 0 or owner.max(initial=0) >= world:
        raise ValueError("owner must give a rank in [0, world) per agent")
    gslot, n_slots = boundary_slots(scn, owner)
    mine = owner == rank
    if scn.n_edges:
        v1, v2 = scn.edges[:, 0], scn.edges[:, 1]
        esel = mine[v1] | mine[v2]
    else:
        esel = np.zeros(0, bool)
    keep = mine.copy()
    if scn.n_edges:
        keep[scn.edges[esel].ravel()] = True
    agents = np.nonzero(keep)[0].astype(np.int32)
    loc = np.full(N, -1, np.int32)
    loc[agents] = np.arange(agents.size, dtype=np.int32)
    edges = np.nonzero(esel)[0].astype(np.int32)
    ledges = loc[scn.edges[edges]].astype(np.int32).reshape(-1, 2)
    counted = (owner[scn.edges[edges, 0]] == rank).astype(np.uint8) if edges.size else np.zeros(0, np.uint8)
    sub = Scenario(spd=scn.spd[agents].copy(), xt0=scn.xt0[agents].copy(), ref=scn.ref[agents].copy(),
                   edges=ledges, n_steps=scn.n_steps)
    return Shard(rank=rank, world=world, scn=sub, agents=agents, edges=edges,
                 owned=mine[agents].astype(np.uint8), counted=counted, slot=gslot[agents].copy(),
                 n_slots=n_slots)


def exchange_width(H: int) -> int:
    """Doubles per exchange slot: px (H+1) | py (H+1) | u (H) | one pad."""
    return 3 * (H + 1)


def pack_exchange(sh: Shard, pos_old: np.ndarray, u: np.ndarray) -> np.ndarray:
    """The rank's contribution to the exchange buffer: its own boundary agents' positions and
    controls in their slots, zero elsewhere (so the all-reduce sum is an all-gather)."""
    H = u.shape[1]
    buf = np.zeros((sh.n_slots, exchange_width(H)))
    sel = (sh.owned == 1) & (sh.slot >= 0)
    k = sh.slot[sel]
    buf[k, :H + 1] = pos_old[sel, 0]
    buf[k, H + 1:2 * H + 2] = pos_old[sel, 1]
    buf[k, 2 * H + 2:3 * H + 2] = u[sel]
    return buf


def unpack_exchange(sh: Shard, buf: np.ndarray, pos_old: np.ndarray, u: np.ndarray):
    """Ghost agents take their owner's positions and controls from the all-reduced buffer."""
    H = u.shape[1]
    sel = sh.owned == 0
    k = sh.slot[sel]
    pos_old[sel, 0] = buf[k, :H + 1]
    pos_old[sel, 1] = buf[k, H + 1:2 * H + 2]
    u[sel] = buf[k, 2 * H + 2:3 * H + 2]
