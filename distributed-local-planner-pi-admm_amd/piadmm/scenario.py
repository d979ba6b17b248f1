"""Scenario generation: agents, reference trajectories and the candidate-pair graph.

The reference has exactly one scenario, the two-vehicle intersection:
  * vehicle A starts at (-10, 0, 0) with speed 4, reference x = linspace(-10, 10, Nt/dt), y = 0
  * vehicle B starts at (0, 20, -pi/2) with speed 8, reference x = 0, y = linspace(20, -20, Nt/dt)
(``casadi/PI_ADMM_class.py:21,31-37``, ``casadi/main.py:25``).

Larger problems tile that scenario.  Two decisions keep a tile
equal to the two-vehicle reference:
  * tiles share one world frame (no spatial offset).  The reference's x-step sums
    the augmented-Lagrangian term over every other agent with hat = lam = 0 at the
    first iteration (``PI_ADMM_class.py:126-129``, quirk B8), which pulls toward the
    world origin, so translating a tile would change its answer.
  * the candidate-pair graph is static: pairs inside a tile only.  Agents of
    different tiles never meet in the AL sum, the collision test or the z-step.
Optional seeded perturbations make tiles differ (dx, dy ~ U(-0.5, 0.5) m,
dtheta ~ U(-0.05, 0.05) rad).
"""
from __future__ import annotations

import dataclasses

import numpy as np


@dataclasses.dataclass
class Scenario:
    spd: np.ndarray          # (N,)   float64, constant speed per agent
    xt0: np.ndarray          # (N,3)  float64, initial (x, y, theta)
    ref: np.ndarray          # (N,2,T) float64, reference positions per time index
    edges: np.ndarray        # (E,2)  int32, candidate pairs (v1 < v2)
    n_steps: int             # MPC steps the reference trajectory supports

    @property
    def n_agents(self) -> int:
        return int(self.spd.shape[0])

    @property
    def n_edges(self) -> int:
        return int(self.edges.shape[0])

    def components(self):
        """Connected components of the candidate graph: (comp_of_agent, n_comp)."""
        n = self.n_agents
        parent = list(range(n))

        def find(a):
            while parent[a] != a:
                parent[a] = parent[parent[a]]
                a = parent[a]
            return a
        for v1, v2 in self.edges:
            ra, rb = find(int(v1)), find(int(v2))
            if ra != rb:
                parent[max(ra, rb)] = min(ra, rb)
        roots = [find(a) for a in range(n)]
        ids = {}
        comp = np.empty(n, np.int32)
        for a, r in enumerate(roots):
            comp[a] = ids.setdefault(r, len(ids))
        return comp, len(ids)

    def neighbours(self):
        """CSR candidate adjacency: (ptr (N+1,), nbr (2E,), edge_of (2E,), dir_of (2E,)).

        ``dir_of`` is 0 when the agent is v1 of the edge (it owns hat_{v1 v2}), 1 when v2.
        """
        n = self.n_agents
        lists = [[] for _ in range(n)]
        for e, (v1, v2) in enumerate(self.edges):
            lists[int(v1)].append((int(v2), e, 0))
            lists[int(v2)].append((int(v1), e, 1))
        ptr = np.zeros(n + 1, np.int32)
        nbr, eo, do = [], [], []
        for a in range(n):
            lists[a].sort()
            ptr[a + 1] = ptr[a] + len(lists[a])
            for j, e, d in lists[a]:
                nbr.append(j)
                eo.append(e)
                do.append(d)
        return (ptr, np.asarray(nbr, np.int32), np.asarray(eo, np.int32),
                np.asarray(do, np.int32))


def _ref_line(start: float, stop: float, n_ref: int, T: int) -> np.ndarray:
    """np.linspace(start, stop, n_ref) extended past its end with the same spacing."""
    base = np.linspace(start, stop, n_ref)
    if T <= n_ref:
        return base[:T].copy()
    step = (stop - start) / (n_ref - 1)
    ext = start + step * np.arange(n_ref, T, dtype=np.float64)
    return np.concatenate([base, ext])


def intersection(H: int, n_steps: int | None = None, Nt: float = 5.0, dt: float = 0.1) -> Scenario:
    """The reference's two-vehicle intersection (``casadi/main.py:25``, ``PI_ADMM_class.py:31-37``).

    With ``n_steps=None`` the MPC loop length is the reference's
    ``int(Nt/dt - num_ho)`` (``casadi/main.py:43``).  Asking for more steps extends
    the reference lines with the same spacing (quirk B13: at H=50 the reference
    runs zero steps).
    """
    n_ref = int(Nt / dt)
    steps_ref = int(Nt / dt - H)
    if n_steps is None:
        n_steps = max(steps_ref, 0)
    T = max(n_ref, n_steps + H)
    xa = _ref_line(-10.0, 10.0, n_ref, T)
    yb = _ref_line(20.0, -20.0, n_ref, T)
    ref = np.zeros((2, 2, T))
    ref[0, 0] = xa
    ref[1, 1] = yb
    xt0 = np.array([[-10, 0, 0], [0, 20, -np.pi / 2]], dtype=np.float64)
    spd = np.array([4, 8], dtype=np.float64)
    return Scenario(spd=spd, xt0=xt0, ref=ref, edges=np.array([[0, 1]], np.int32), n_steps=n_steps)


def tiled(n_tiles: int, H: int, n_steps: int | None = None, perturb: bool = True,
          seed: int = 0) -> Scenario:
    """``n_tiles`` copies of the intersection (N = 2*n_tiles agents), tile k seeded with seed+k."""
    base = intersection(H, n_steps)
    N = 2 * n_tiles
    spd = np.tile(base.spd, n_tiles)
    xt0 = np.tile(base.xt0, (n_tiles, 1))
    ref = np.tile(base.ref, (n_tiles, 1, 1))
    if perturb:
        for k in range(n_tiles):
            rng = np.random.default_rng(seed + k)
            d = rng.uniform(-1.0, 1.0, size=(2, 3)) * np.array([0.5, 0.5, 0.05])
            xt0[2 * k:2 * k + 2] += d
    edges = np.stack([np.arange(0, N, 2), np.arange(1, N, 2)], axis=1).astype(np.int32)
    return Scenario(spd=spd, xt0=xt0, ref=ref, edges=edges, n_steps=base.n_steps)


# Approach lanes of the N-vehicle crossing: (x0, y0, theta0, speed, x_end, y_end) over Nt = 5 s.
# Lanes 0 and 1 are the reference's two vehicles (casadi/PI_ADMM_class.py:21,31-37); lanes 2
# and 3 enter from the east and the south, offset so that the four paths cross pairwise.
_LANES = (
    (-10.0, 0.0, 0.0, 4.0, 10.0, 0.0),
    (0.0, 20.0, -np.pi / 2, 8.0, 0.0, -20.0),
    (12.0, 1.5, np.pi, 5.0, -13.0, 1.5),
    (-1.5, -14.0, np.pi / 2, 6.0, -1.5, 16.0),
)


def crossing(n_vehicles: int, H: int, n_steps: int | None = None, pairs: str = "all",
             Nt: float = 5.0, dt: float = 0.1, seed: int | None = None) -> Scenario:
    """An ``n_vehicles`` crossing: the reference's ``num_veh`` loop beyond two vehicles
    (``casadi/main.py:81,110-113``: every agent's AL sum and collision test over the others).

    Vehicle k drives lane k % 4 of :data:`_LANES` (lanes 0, 1 = the reference's A and B), shifted
    3 m sideways per full round of lanes.  ``pairs``: ``"all"`` -- every pair i < j is a
    candidate (the reference's all-pairs semantics, quirk B8); ``"chain"`` -- pairs (k, k+1) only.
    ``seed`` perturbs the start states like :func:`tiled`."""
    n_ref = int(Nt / dt)
    if n_steps is None:
        n_steps = max(int(Nt / dt - H), 0)
    T = max(n_ref, n_steps + H)
    spd = np.empty(n_vehicles)
    xt0 = np.empty((n_vehicles, 3))
    ref = np.zeros((n_vehicles, 2, T))
    for k in range(n_vehicles):
        x0, y0, th, v, x1, y1 = _LANES[k % 4]
        off = 3.0 * (k // 4)
        sx, sy = (0.0, off) if abs(np.cos(th)) > 0.5 else (off, 0.0)
        spd[k] = v
        xt0[k] = (x0 + sx, y0 + sy, th)
        ref[k, 0] = _ref_line(x0 + sx, x1 + sx, n_ref, T)
        ref[k, 1] = _ref_line(y0 + sy, y1 + sy, n_ref, T)
    if seed is not None:
        rng = np.random.default_rng(seed)
        xt0 += rng.uniform(-1.0, 1.0, size=xt0.shape) * np.array([0.5, 0.5, 0.05])
    if pairs == "all":
        edges = [(i, j) for i in range(n_vehicles) for j in range(i + 1, n_vehicles)]
    elif pairs == "chain":
        edges = [(i, i + 1) for i in range(n_vehicles - 1)]
    else:
        raise ValueError("pairs must be 'all' or 'chain'")
    return Scenario(spd=spd, xt0=xt0, ref=ref, edges=np.asarray(edges, np.int32).reshape(-1, 2), n_steps=n_steps)


def concat(scenarios) -> Scenario:
    """Independent copies side by side (agents renumbered, candidate pairs kept per copy)."""
    offs = np.cumsum([0] + [s.n_agents for s in scenarios])
    T = min(s.ref.shape[2] for s in scenarios)
    return Scenario(spd=np.concatenate([s.spd for s in scenarios]),
                    xt0=np.concatenate([s.xt0 for s in scenarios]),
                    ref=np.concatenate([s.ref[:, :, :T] for s in scenarios]),
                    edges=np.concatenate([s.edges + o for s, o in zip(scenarios, offs)]).astype(np.int32),
                    n_steps=min(s.n_steps for s in scenarios))


def n_steps_for(H: int, Nt: float = 5.0, dt: float = 0.1) -> int:
    return max(int(Nt / dt - H), 0)


__all__ = ["Scenario", "intersection", "tiled", "crossing", "concat", "n_steps_for"]
