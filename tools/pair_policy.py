"""Development experiment: ADMM penalty policies (fixed / adaptive / restarted rho) on recorded
pair QPs (tools/pair_collect.py) with the kernel's one-step PDAS label update; prints iterations and
reduced solves per policy.  Not shipped, not the oracle."""
import sys, numpy as np, glob
sys.path.insert(0,'/root/repo/tools'); sys.path.insert(0,'/root/repo/distributed-local-planner-pi-admm_amd')
import qp_sim as Q
def classify_cons(gq, x, y, sets, tol=1e-9):
    ax=gq.A@x; new=sets.copy(); hm=gq.hinge; b=~hm
    ty=tol*(1+np.abs(y).max()); tp=tol*(1+np.abs(np.where(np.isfinite(gq.l),gq.l,0)))
    f=b&(sets==Q.FREE)
    new[f&(ax<gq.l-tp)]=Q.LOWER; new[f&(ax>gq.u+tp)]=Q.UPPER
    new[b&(sets==Q.LOWER)&(y>ty)]=Q.FREE; new[b&(sets==Q.UPPER)&(y<-ty)]=Q.FREE
    new[hm&(sets==Q.ZERO)&(ax<gq.l-tp)]=Q.KINK; new[hm&(sets==Q.LINEAR)&(ax>gq.l+tp)]=Q.KINK
    new[hm&(sets==Q.KINK)&(y>ty)]=Q.ZERO; new[hm&(sets==Q.KINK)&(y<-gq.beta-ty)]=Q.LINEAR
    return new
NP=[0]
def pdas_c(gq, Pinv, sets, c, max_steps=8, tol=1e-9):
    for k in range(4):
        NP[0]+=1
        x,y,_=Q.reduced_solve(gq,Pinv,sets)
        if Q.kkt_ok(gq,x,y,sets,tol): return x,y,sets,True,k+1
        new=classify_cons(gq,x,y,sets)
        if np.array_equal(new,sets): return x,y,sets,False,k+1
        sets=new
    return x,y,sets,False,4
Q.pdas=pdas_c
def load(path):
    out=[]
    for r in np.load(path, allow_pickle=True):
        gq=Q.GQP.from_edge_slack(r['P'],r['q'],r['A'],r['lo'],r['hi'],30,1000.0)
        out.append(gq)
    return out
def run_policy(gq, pol):
    Pinv=np.linalg.inv(gq.P); D,E=Q.scale_problem(gq,'ruiz')
    NP[0]=0; total=0; state=None
    for (rho,hr,ad,n) in pol:
        rs=np.where(gq.hinge,hr,1.0)
        x,y,its,ok,ps=Q.admm(gq,rho,1e-6,1.6,n,D,E,state=state,Pinv=Pinv,polish_every=10,rho_scale=rs,adapt_every=ad)
        total+=its
        if ok: return total, NP[0], True
        state=(x/D, E*(gq.A@x), y/E)
    return total, NP[0], False
if __name__=='__main__':
    files=sys.argv[1:]
    qps=[]
    for f in files: qps+= [(f.split('/')[-1],i,g) for i,g in enumerate(load(f))]
    pols={'cur':[(0.05,3,25,4000)],
          'noad':[(0.05,3,0,4000)],
          'r001':[(0.01,3,0,4000)],
          'rst':[(0.05,3,25,300),(0.01,3,0,3700)],
          'rst2':[(0.05,3,25,200),(0.01,10,0,3800)]}
    for name,pol in pols.items():
        res=[run_policy(g,pol) for _,_,g in qps]
        its=np.array([r[0] for r in res]); np_=np.array([r[1] for r in res]); ok=np.array([r[2] for r in res])
        cost=its+20*np_
        print(f"{name:6s} ok {ok.sum()}/{len(ok)} its mean {its.mean():.0f} max {its.max()} pdas mean {np_.mean():.1f} max {np_.max()} cost mean {cost.mean():.0f} p95 {np.percentile(cost,95):.0f} max {cost.max()}", flush=True)
