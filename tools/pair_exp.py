"""Development experiment: can the pair QP polish start from the previous step's labels shifted
by one time slot?  (tools/pair_collect.py records the bench's pair QPs from the oracle.)"""
import sys, numpy as np
sys.path.insert(0,'/root/repo/tools'); sys.path.insert(0,'/root/repo')
import qp_sim as Q
rec=list(np.load('/tmp/pair_qps.npy', allow_pickle=True))
H=30; ntile=32
def gq_of(r):
    return Q.GQP.from_edge_slack(r['P'],r['q'],r['A'],r['lo'],r['hi'],H,1000.0)
def exact_labels(gq, r):
    x=r['x'][:2*H]; ax=gq.A@x
    s=np.zeros(gq.m,np.int8); tol=1e-7
    b=~gq.hinge
    s[b&(ax<=gq.l+tol)]=Q.LOWER; s[b&(ax>=gq.u-tol)]=Q.UPPER
    hm=gq.hinge
    s[hm&(np.abs(ax-gq.l)<=tol)]=Q.KINK; s[hm&(ax<gq.l-tol)]=Q.LINEAR
    return s
def shift(lab):
    # rows: box1 H, rate1 H-1, box2 H, rate2 H-1, hinge H (time k=1..H)
    out=lab.copy(); o=0
    for n in (H,H-1,H,H-1,H):
        seg=lab[o:o+n]; out[o:o+n-1]=seg[1:]; out[o+n-1]=seg[-1]; o+=n
    return out
res=[]
for i,r in enumerate(rec):
    gq=gq_of(r); Pinv=np.linalg.inv(gq.P)
    lab=exact_labels(gq,r)
    nk=(lab[gq.hinge]==Q.KINK).sum(); nb=(lab[~gq.hinge]!=0).sum()
    # PDAS from exact labels (sanity)
    c=np.full(gq.m,1.0)
    _,_,_,ok0,st0=Q.pdas(gq,Pinv,lab.copy(),c)
    # PDAS from shifted labels of previous step (same tile)
    prev = i-ntile
    if prev>=0:
        pl=shift(exact_labels(gq_of(rec[prev]),rec[prev]))
        _,_,_,ok1,st1=Q.pdas(gq,Pinv,pl,c,max_steps=10)
        diff=(pl!=lab).sum()
    else: ok1,st1,diff=None,0,-1
    _,_,_,ok2,st2=Q.pdas(gq,Pinv,np.zeros(gq.m,np.int8),c,max_steps=10)
    res.append((i//ntile,i%ntile,nk,nb,ok0,st0,ok1,st1,diff,ok2,st2))
for x in res[:80]: print(x)
import collections
print('shifted ok', collections.Counter((x[6],x[7]) for x in res if x[6] is not None))
print('zero ok', collections.Counter((x[9],x[10]) for x in res))
