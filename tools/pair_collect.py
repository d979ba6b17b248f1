"""Development tool: record the pair QPs of the bench workload (oracle, 32 tiles x 6 steps)."""
import sys, numpy as np, time
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/distributed-local-planner-pi-admm_amd')
from oracle import piadmm_oracle as O
from piadmm import config, scenario
H=30
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=2)
scn = scenario.tiled(32, H, n_steps=8, perturb=True, seed=0)
orc = O.Oracle(cfg, scn)
rec=[]
orig=O.solve_edge
cur={'t':0}
def hook(*a):
    r=orig(*a); P,q,A,lo,hi,x,y=r[1]
    rec.append(dict(t=cur['t'],P=P,q=q,A=A,lo=lo,hi=hi,x=x,y=y)); return r
O.solve_edge=hook
t0=time.time()
for t in range(6):
    cur['t']=t
    orc.mpc_step()
print(len(rec), time.time()-t0)
np.save('/tmp/pair_qps.npy', np.array(rec, dtype=object), allow_pickle=True)
