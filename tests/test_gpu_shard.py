"""GPU parity of a job sharded by agent with candidate pairs ACROSS ranks:
every rank holds its own agents plus ghost copies of their neighbours on other ranks, and one
all-reduce of the boundary exchange buffer per outer iteration carries the boundary agents'
positions and controls (piadmm_set_scenario_shard, piadmm.dist.shard_graph).

The GPU box has one MI355X, so the ranks here are threads of this process, each with its own
handle (own HIP stream) on device 0, joined by the library's host all-reduce transport
(piadmm_set_allreduce) -- the same exchange protocol bench.py runs over RCCL between GPUs.
The sharded job must equal the unsharded job on one handle (and the oracle): identical
iteration counts, states and plans of every agent (to 1e-10), the job's residual history up
to summation order (1e-9)."""
import threading

import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, dist, scenario

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


class ThreadAllReduce:
    """Sum over the ranks (threads) in rank order, identical on every rank."""

    def __init__(self, world):
        self.bar = threading.Barrier(world, timeout=120)
        self.bufs = [None] * world
        self.calls = [0] * world

    def fn(self, rank):
        def f(buf):
            self.bufs[rank] = buf.copy()
            self.bar.wait()
            tot = self.bufs[0].copy()
            for b in self.bufs[1:]:
                tot += b
            self.bar.wait()
            buf[:] = tot
            self.calls[rank] += 1
        return f


def run_sharded(Solver, cfg, scn, owner, world, n_steps):
    shards = [dist.shard_graph(scn, r, world, owner) for r in range(world)]
    ar = ThreadAllReduce(world)
    solvers = []
    for r, sh in enumerate(shards):
        s = Solver(cfg, shard=sh)
        s.set_allreduce(ar.fn(r))
        solvers.append(s)
    out = [[] for _ in range(world)]
    err = [None] * world

    def work(r):
        try:
            for _ in range(n_steps):
                out[r].append(solvers[r].mpc_step())
        except Exception as e:          # noqa: BLE001 -- reported below
            err[r] = e
            ar.bar.abort()
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for s in solvers:
        s.close()
    assert not any(t.is_alive() for t in th), "a rank hung"
    for e in err:
        if e is not None:
            raise e
    return shards, out, ar


def gather(shards, out, k, N, H):
    xt, u = np.full((N, 3), np.nan), np.full((N, H), np.nan)
    for sh, res in zip(shards, out):
        own = sh.owned == 1
        xt[sh.agents[own]] = res[k].xt[own]
        u[sh.agents[own]] = res[k].u[own]
        assert np.all(res[k].status == 0)
    return xt, u


@pytest.mark.parametrize("world,split", [(2, "interleaved"), (3, "blocks")])
def test_sharded_crossings_equal_unsharded(Solver, world, split):
    """Two 4-vehicle all-pairs crossings and a 3-vehicle chain, agents split so that pairs cross
    ranks (interleaved: every pair of the crossings; blocks: a crossing cut in the middle);
    the reference's global stop test (term_global, natural termination)."""
    H = 15
    scn = scenario.concat([scenario.crossing(4, H, n_steps=20, seed=1), scenario.crossing(4, H, n_steps=20, seed=2),
                           scenario.crossing(3, H, n_steps=20, pairs="chain")])
    N = scn.n_agents
    # blocks of 3, 4, 4 agents: both crossings cut between ranks
    owner = dist.owners_interleaved(N, world) if split == "interleaved" else np.repeat([0, 1, 2], [3, 4, 4]).astype(np.int32)
    cfg = config.matlab_pi(H=H, term_global=1)
    n_steps = 10
    shards, out, ar = run_sharded(Solver, cfg, scn, owner, world, n_steps)
    assert shards[0].n_slots > 0 and min(ar.calls) > 0
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s1:
        for k in range(n_steps):
            r1, ro = s1.mpc_step(), orc.mpc_step()
            xt, u = gather(shards, out, k, N, H)
            np.testing.assert_allclose(xt, r1.xt, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            np.testing.assert_allclose(u, r1.u, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            np.testing.assert_allclose(xt, ro.xt, rtol=1e-8, atol=1e-8, err_msg=f"step {k}")
            for res in out:
                assert res[k].global_iters == r1.global_iters == int(ro.iters[0])
                n = r1.global_iters
                np.testing.assert_allclose(res[k].global_resid[:n], r1.global_resid[:n], rtol=1e-9, atol=1e-12)


def test_adversarial_split_of_the_bench_tiles_fixed_iterations(Solver):
    """SURVEY.md 8d C4 'adversarial' case: the tiled bench scenario with every two-vehicle tile
    split across two ranks, fixed iterations under the global scope (the bench's mode): every
    outer iteration exchanges every agent.  Equal to the unsharded run on the fused kernel."""
    H = 30
    scn = scenario.tiled(8, H, n_steps=10, seed=11)
    N = scn.n_agents
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=12, term_global=1)
    shards, out, ar = run_sharded(Solver, cfg, scn, dist.owners_interleaved(N, 2), 2, 4)
    assert shards[0].n_slots == N
    with Solver(cfg, scn) as s1:
        for k in range(4):
            r1 = s1.mpc_step()
            xt, u = gather(shards, out, k, N, H)
            np.testing.assert_allclose(xt, r1.xt, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            np.testing.assert_allclose(u, r1.u, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            for res in out:
                assert res[k].global_iters == 12
                np.testing.assert_allclose(res[k].global_resid, r1.global_resid, rtol=1e-9, atol=1e-12)


def test_shard_argument_errors(Solver):
    """Refused shards fail loudly: pairs across ranks without the global scope."""
    scn = scenario.crossing(4, 10, n_steps=10)
    sh = dist.shard_graph(scn, 0, 2, dist.owners_interleaved(4, 2))
    from piadmm._lib import PiadmmError
    with pytest.raises(PiadmmError, match="term_global"):
        Solver(config.matlab_pi(H=10), shard=sh)


def run_ranks(Solver, cfg, rank_scns, n_steps, shards=None):
    """One handle per rank (threads on device 0, host all-reduce transport); mpc_step n_steps
    times on every rank.  rank_scns: plain per-rank scenarios (whole components per rank), or
    None with ``shards`` (pairs across ranks)."""
    world = len(shards) if shards is not None else len(rank_scns)
    ar = ThreadAllReduce(world)
    solvers = []
    for r in range(world):
        s = Solver(cfg, shard=shards[r]) if shards is not None else Solver(cfg, rank_scns[r])
        s.set_allreduce(ar.fn(r))
        solvers.append(s)
    out = [[] for _ in range(world)]
    err = [None] * world

    def work(r):
        try:
            for _ in range(n_steps):
                out[r].append(solvers[r].mpc_step())
        except Exception as e:          # noqa: BLE001 -- reported below
            err[r] = e
            ar.bar.abort()
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    for s in solvers:
        s.close()
    assert not any(t.is_alive() for t in th), "a rank hung"
    for e in err:
        if e is not None:
            raise e
    return out, ar


@pytest.mark.parametrize("split", ["contiguous", "interleaved"])
def test_config3_1024_agents_over_8_ranks(Solver, split):
    """BASELINE.json configs[3] at its stated shape: 1024 agents x H30 (512 seeded tiles),
    matlab_pi, the reference's global scope with fixed 100 outer iterations (the bench's mode),
    sharded over 8 ranks -- ``contiguous``: whole tiles per rank (bench.py --strong, dist.shard:
    128 agents per rank, no boundary, one all-reduce of the residual history per step);
    ``interleaved``: agent a on rank a % 8, so every pair crosses ranks (bench.py --strong --split
    interleaved: 128 own agents + 128 ghosts per rank, one all-reduce of the 1024-slot boundary
    exchange buffer per outer iteration).  8 ranks = 8 threads with their own handles on the one
    MI355X (host transport).  Equal to the unsharded 1024-agent job on one handle to 1e-10, the
    job's residual history to 1e-9, and sampled tiles equal to the oracle (1e-8)."""
    H, world, n_steps = 30, 8, 3
    full = scenario.tiled(512, H, n_steps=n_steps + 2, perturb=True, seed=0)
    N = full.n_agents
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=100, term_global=1)
    if split == "contiguous":
        scns = [dist.shard(full, r, world) for r in range(world)]
        out, ar = run_ranks(Solver, cfg, scns, n_steps)
        bounds = [dist.shard_bounds(full, r, world) for r in range(world)]
    else:
        shards = [dist.shard_graph(full, r, world, dist.owners_interleaved(N, world)) for r in range(world)]
        assert shards[0].n_slots == N
        out, ar = run_ranks(Solver, cfg, None, n_steps, shards)
    assert min(ar.calls) >= n_steps
    with Solver(cfg, full) as s1:
        ref = [s1.mpc_step() for _ in range(n_steps)]
    for k in range(n_steps):
        if split == "contiguous":
            xt = np.concatenate([out[r][k].xt for r in range(world)])
            u = np.concatenate([out[r][k].u for r in range(world)])
            assert [b[1] - b[0] for b in bounds] == [128] * world
            for r in range(world):
                assert np.all(out[r][k].status == 0)
        else:
            xt, u = gather(shards, out, k, N, H)
        np.testing.assert_allclose(xt, ref[k].xt, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
        np.testing.assert_allclose(u, ref[k].u, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
        for r in range(world):
            assert out[r][k].global_iters == ref[k].global_iters == 100
            np.testing.assert_allclose(out[r][k].global_resid, ref[k].global_resid, rtol=1e-9, atol=1e-12)
    # sampled tiles against the oracle (under fixed iterations a tile's trajectory is its own:
    # the global scope only sums the residual history)
    for k in (0, 357):
        sub = scenario.Scenario(spd=full.spd[2 * k:2 * k + 2], xt0=full.xt0[2 * k:2 * k + 2],
                                ref=full.ref[2 * k:2 * k + 2], edges=np.array([[0, 1]], np.int32),
                                n_steps=full.n_steps)
        orc = O.Oracle(cfg, sub)
        for j in range(n_steps):
            ro = orc.mpc_step()
            np.testing.assert_allclose(ref[j].xt[2 * k:2 * k + 2], ro.xt, rtol=1e-8, atol=1e-8)
            np.testing.assert_allclose(ref[j].u[2 * k:2 * k + 2], ro.u, rtol=1e-8, atol=1e-8)
