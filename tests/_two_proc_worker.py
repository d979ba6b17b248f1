"""One rank of tests/test_gpu_two_process.py: a separate process with its own libpiadmm handle on
the one MI355X, joined to the other rank by a gloo process group.  The library's exchange goes
through ``piadmm_set_allreduce`` (the host transport: RCCL refuses two ranks on one device), the
same path ``bench.py --gpus N`` takes under ``PIADMM_BENCH_TRANSPORT=host``.

    python tests/_two_proc_worker.py <case> <rank> <world> <port> <out.npz>

Writes every step's xt, u, status, iteration count and job residual history of the rank's own
agents.  Not collected by pytest (the leading underscore)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]


def case(name):
    """The two jobs of the test (the test process builds the same ones for the unsharded run)."""
    from piadmm import config, scenario
    if name == "tiles_fixed":
        # the bench's mode: tiled intersections, fixed outer iterations under the global scope
        H = 20
        return config.matlab_pi(H=H, fixed_iters=1, max_outer=30, term_global=1), \
            scenario.tiled(6, H, n_steps=8, seed=3), 4
    if name == "crossing_natural":
        # a coupled job: two 4-vehicle all-pairs crossings, the reference's natural global stop test
        H = 15
        return config.matlab_pi(H=H, term_global=1), \
            scenario.concat([scenario.crossing(4, H, n_steps=12, seed=1),
                             scenario.crossing(4, H, n_steps=12, seed=2)]), 6
    raise ValueError(name)


def main():
    name, rank, world, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from piadmm import dist
    from piadmm.solver import PI_ADMM_MI355X
    cfg, scn, n_steps = case(name)
    owner = dist.owners_interleaved(scn.n_agents, world)     # every pair crosses the ranks
    sh = dist.shard_graph(scn, rank, world, owner)

    def host_allreduce(buf):
        t = torch.from_numpy(buf.copy())
        tdist.all_reduce(t)                                  # sum: each slot written by one rank
        buf[:] = t.numpy()

    res = {"agents": sh.agents[sh.owned == 1], "n_slots": np.int64(sh.n_slots)}
    xt, u, st, gi, gr = [], [], [], [], []
    with PI_ADMM_MI355X(cfg, shard=sh) as s:
        s.set_allreduce(host_allreduce)
        for _ in range(n_steps):
            r = s.mpc_step()
            own = sh.owned == 1
            xt.append(r.xt[own])
            u.append(r.u[own])
            st.append(r.status[:own.size][own])         # (status: agents, then pairs)
            gi.append(r.global_iters)
            gr.append(np.nan_to_num(r.global_resid, nan=-1.0))
    res.update(xt=np.array(xt), u=np.array(u), status=np.array(st), global_iters=np.array(gi),
               global_resid=np.array(gr))
    np.savez(out, **res)
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
