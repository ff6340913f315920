"""Would longest-first ordering shorten the LK level tails?  From measured per-(level, point)
iteration counts (gpurun_out/lk_iters.npz, scripts/lk_iters.py on the GPU box): per level, one XCD's
range (4 pairs) of groups (G = 8 at level 0, 4 above; a group runs max(iters) steps) list-scheduled
on its 768 waves' slots in queue order, longest-first with the true durations, and longest-first
predicted by the same points' iterations at the coarser level.  Also prints the per-point
correlation of iteration counts between consecutive levels.
Usage: python scripts/lk_lpt_sim.py
"""
import heapq, numpy as np
W,H,PS,NLEV=1920,1080,10,5
NX,NY=(W+PS-1)//PS,(H+PS-1)//PS
d=np.load('gpurun_out/lk_iters.npz')
bufs=[d['1920x1080_ps10_s1'],d['1920x1080_ps10_s2']]
def groups(buf,L,G):
    it=buf[L,:,2].reshape(NX,NY).astype(int)
    prev=buf[L+1,:,2].reshape(NX,NY).astype(int) if L+1<NLEV else None
    m=(1<<L)-1
    out=[]
    for gy in range(NY):
        cls={}
        for gx in range(NX):
            cls.setdefault((gx*PS)&m,[]).append(gx)
        for c,xs in cls.items():
            for q in range(0,len(xs),G):
                mem=xs[q:q+G]
                dur=max(it[x,gy] for x in mem)
                pred=max(prev[x,gy] for x in mem) if prev is not None else 0
                out.append((dur,pred))
    return out
def makespan(units,nslots):
    h=[0]*nslots
    for s in units: heapq.heappush(h,heapq.heappop(h)+s)
    return max(h)
# correlation of per-point iters between levels
b=bufs[0]
for L in range(NLEV-1):
    a=b[L,:,2]; c=b[L+1,:,2]
    print("L",L,"mean iters %.2f"%a.mean(),"corr with L+1: %.3f"%np.corrcoef(a,c)[0,1])
tot={'queue':0,'lpt_true':0,'lpt_pred':0}
for L in range(NLEV):
    G=8 if L==0 else 4
    nslots=768*(64//(4*G))
    units=[]
    for p in range(4):   # one XCD range = 4 pairs
        units+=groups(bufs[p%2],L,G)
    ideal=sum(u[0] for u in units)/nslots
    q=makespan([u[0] for u in units],nslots)
    t=makespan(sorted([u[0] for u in units],reverse=True),nslots)
    pr=makespan([u[0] for u in sorted(units,key=lambda u:-u[1])],nslots)
    tot['queue']+=q; tot['lpt_true']+=t; tot['lpt_pred']+=pr
    print(f"L{L} G{G} units {len(units)} ideal {ideal:.1f} queue {q} lpt_true {t} lpt_pred {pr}")
print(tot)
