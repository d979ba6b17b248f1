"""Multi-rank path on CPU (gloo, world_size 2): sharded runs equal the unsharded run.

Each rank owns whole components (piadmm.dist.shard), runs its shard through the
oracle (the CPU stand-in for one GPU) and the shards are gathered; the result
must equal one process running all agents, because no component straddles ranks.
The same harness (barrier + max-over-ranks timing) is what bench.py uses.

With term_global the ranks exchange their termination partials once per outer
iteration -- the protocol libpiadmm runs over RCCL -- here as a gloo all-reduce.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as tdist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import piadmm_oracle as O
    from piadmm import config, dist, scenario
    scn = scenario.tiled(5, 10, n_steps=30, seed=2)
    sub = dist.shard(scn, rank, world)
    cfg = config.matlab_pi(H=10)
    orc = O.Oracle(cfg, sub)
    for _ in range(3):
        orc.run(10)
    a0, a1 = dist.shard_bounds(scn, rank, world)
    mine = {"a0": a0, "xt": orc.xt}
    gathered = [None] * world
    tdist.all_gather_object(gathered, mine)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)              # bench.py's max-over-ranks timer
    tdist.barrier()
    if rank == 0:
        xt = np.zeros((scn.n_agents, 3))
        for g in gathered:
            xt[g["a0"]:g["a0"] + g["xt"].shape[0]] = g["xt"]
        np.save(out, xt)
        assert float(t) == float(world)
    tdist.destroy_process_group()


def test_two_rank_shards_match_single_process(tmp_path):
    out = str(tmp_path / "xt.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import piadmm_oracle as O
    from piadmm import config, scenario
    scn = scenario.tiled(5, 10, n_steps=30, seed=2)
    orc = O.Oracle(config.matlab_pi(H=10), scn)
    for _ in range(3):
        orc.run(10)
    np.testing.assert_array_equal(np.load(out), orc.xt)


def _global_worker(rank, world, port, out):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import piadmm_oracle as O
    from piadmm import config, dist, scenario
    scn = scenario.tiled(5, 15, n_steps=30, seed=3)
    sub = dist.shard(scn, rank, world)
    orc = O.Oracle(config.casadi_default(H=15, term_global=1), sub)
    calls = [0]

    def allreduce(part):
        calls[0] += 1
        t = torch.tensor(part, dtype=torch.float64)
        tdist.all_reduce(t)                      # libpiadmm: ncclAllReduce(sum) of 5 doubles
        return t.numpy()
    its, ghist = [], []
    for _ in range(12):
        r = orc.mpc_step(reduce=allreduce)
        its.append(r.iters.tolist())
        ghist.append(np.array(r.global_resid).reshape(-1, 2))
    a0, _ = dist.shard_bounds(scn, rank, world)
    gathered = [None] * world
    tdist.all_gather_object(gathered, {"a0": a0, "xt": orc.xt, "its": its, "ghist": ghist, "calls": calls[0]})
    if rank == 0:
        xt = np.zeros((scn.n_agents, 3))
        for g in gathered:
            xt[g["a0"]:g["a0"] + g["xt"].shape[0]] = g["xt"]
        np.savez(out, xt=xt, its0=np.array(gathered[0]["its"][-1]), its1=np.array(gathered[1]["its"][-1]),
                 g0=np.concatenate(gathered[0]["ghist"]), g1=np.concatenate(gathered[1]["ghist"]),
                 calls=np.array([g["calls"] for g in gathered]))
    tdist.destroy_process_group()


def test_two_rank_global_termination_matches_single_process(tmp_path):
    """Sharded term_global (one all-reduce of the partials per outer iteration) equals the
    unsharded job: same states, same job-wide iteration count and residual history."""
    out = str(tmp_path / "g.npz")
    mp.spawn(_global_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import piadmm_oracle as O
    from piadmm import config, scenario
    scn = scenario.tiled(5, 15, n_steps=30, seed=3)
    orc = O.Oracle(config.casadi_default(H=15, term_global=1), scn)
    ghist = []
    for _ in range(12):
        r = orc.mpc_step()
        ghist.append(np.array(r.global_resid).reshape(-1, 2))
    d = np.load(out)
    np.testing.assert_array_equal(d["xt"], orc.xt)
    assert set(d["its0"].tolist()) == set(d["its1"].tolist()) == {int(r.iters[0])}
    np.testing.assert_allclose(d["g0"], np.concatenate(ghist), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(d["g1"], d["g0"], rtol=0, atol=0)
    assert d["calls"][0] == d["calls"][1] > 0


def _cross_worker(rank, world, port, out):
    """One rank of a job sharded by agent with pairs across ranks: own agents + ghosts, the
    boundary exchange (positions and controls) as one gloo all-reduce per outer iteration --
    the protocol libpiadmm runs over RCCL (piadmm_set_scenario_shard)."""
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import piadmm_oracle as O
    from piadmm import config, dist
    scn, cfg = _cross_case()
    sh = dist.shard_graph(scn, rank, world, dist.owners_interleaved(scn.n_agents, world))
    orc = O.Oracle(cfg, sh.scn, owned=sh.owned, counted=sh.counted)
    calls = [0, 0]

    def exchange(pos_old, u):
        calls[0] += 1
        buf = torch.from_numpy(dist.pack_exchange(sh, pos_old, u))
        tdist.all_reduce(buf)
        dist.unpack_exchange(sh, buf.numpy(), pos_old, u)

    def allreduce(part):
        calls[1] += 1
        t = torch.tensor(part, dtype=torch.float64)
        tdist.all_reduce(t)
        return t.numpy()
    its, ghist = [], []
    for _ in range(4):
        r = orc.mpc_step(reduce=allreduce, exchange=exchange)
        its.append(int(r.iters[0]))
        ghist.append(np.array(r.global_resid).reshape(-1, 2))
    gathered = [None] * world
    tdist.all_gather_object(gathered, {"own": sh.own, "xt": orc.xt[sh.owned == 1], "its": its,
                                       "ghist": ghist, "calls": calls})
    if rank == 0:
        xt = np.full((scn.n_agents, 3), np.nan)
        for g in gathered:
            xt[g["own"]] = g["xt"]
        np.savez(out, xt=xt, its=np.array([g["its"] for g in gathered]),
                 g0=np.concatenate(gathered[0]["ghist"]), g1=np.concatenate(gathered[1]["ghist"]),
                 calls=np.array([g["calls"] for g in gathered]))
    tdist.destroy_process_group()


def _cross_case():
    from piadmm import config, scenario
    scn = scenario.concat([scenario.crossing(3, 10, n_steps=12, seed=4), scenario.crossing(3, 10, n_steps=12,
                                                                                           pairs="chain")])
    return scn, config.matlab_pi(H=10, term_global=1)


def test_shard_graph_partitions_the_job():
    """Every agent is owned by exactly one rank, every pair lives on each rank of its agents and
    counts on exactly one; ghosts have exchange slots, and the slots are the job's boundary."""
    from piadmm import dist, scenario
    scn = scenario.concat([scenario.crossing(4, 10, n_steps=5), scenario.tiled(3, 10, n_steps=5)])
    for world, owner in ((2, dist.owners_interleaved(scn.n_agents, 2)), (3, dist.owners_blocks(scn.n_agents, 3))):
        shards = [dist.shard_graph(scn, r, world, owner) for r in range(world)]
        own = np.concatenate([sh.own for sh in shards])
        assert sorted(own.tolist()) == list(range(scn.n_agents))
        counted = np.zeros(scn.n_edges, int)
        for sh in shards:
            counted[sh.edges[sh.counted == 1]] += 1
            assert np.all(sh.slot[sh.owned == 0] >= 0)
            assert np.all(sh.scn.edges[:, 0] < sh.scn.edges[:, 1])
            np.testing.assert_array_equal(sh.scn.xt0, scn.xt0[sh.agents])
            for le, ge in zip(sh.scn.edges, sh.edges):           # local pairs map to the global pairs
                np.testing.assert_array_equal(sh.agents[le], scn.edges[ge])
                assert sh.owned[le[0]] or sh.owned[le[1]]
        np.testing.assert_array_equal(counted, 1)
        assert len({sh.n_slots for sh in shards}) == 1


def test_two_rank_pairs_across_ranks_match_single_process(tmp_path):
    """Pairs across ranks (every pair of a 3-vehicle all-pairs crossing and of a chain, agents
    interleaved over 2 ranks): own agents + ghosts, one exchange all-reduce per outer iteration.
    Equals the unsharded job bit for bit in the states; iteration counts equal; the residual
    history up to summation order."""
    out = str(tmp_path / "x.npz")
    mp.spawn(_cross_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import piadmm_oracle as O
    scn, cfg = _cross_case()
    orc = O.Oracle(cfg, scn)
    its, ghist = [], []
    for _ in range(4):
        r = orc.mpc_step()
        its.append(int(r.iters[0]))
        ghist.append(np.array(r.global_resid).reshape(-1, 2))
    d = np.load(out)
    np.testing.assert_array_equal(d["xt"], orc.xt)
    assert d["its"].tolist() == [its, its]
    np.testing.assert_allclose(d["g0"], np.concatenate(ghist), rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(d["g1"], d["g0"])
    assert np.all(d["calls"][:, 0] == sum(its)) and np.all(d["calls"][:, 1] == sum(its))
