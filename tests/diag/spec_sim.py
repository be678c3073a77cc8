#!/usr/bin/env python3
"""CPU simulation behind DESIGN.md 5's "speculative start": how many (row, pod) pairs a score workgroup must score
exactly when the rows commit(b - 3) may touch (its SUSPECTS) feed no lower bound.

  python tests/diag/spec_sim.py [own|merged]

own: each workgroup's own top-KC rows of batch b - 3 for every pod (what a workgroup knows locally); merged: the rows
of batch b - 3's merged lists (the global top 16 per pod).  Both add the rows of the two exports commit(b - 3)
inherits.  Node states are the sequential schedule's (oracle, cached in /tmp/screen_sim_c4_idx.npy as
tests/diag/screen_sim.py makes it); keys are the reference formula in numpy f64.  Exploration tool.
"""
import os
import sys, numpy as np
D = os.path.dirname(os.path.abspath(__file__))
R_ = os.path.dirname(os.path.dirname(D))
sys.path[:0] = [D, os.path.join(R_, 'k8s-scheduler_amd'), os.path.join(R_, 'oracle')]
from screen_sim import keys, state_at
from ksched import cluster
MODE = sys.argv[1] if len(sys.argv) > 1 else 'merged'
cl=cluster.make_cluster('c4'); n=cl.n_nodes; G=232; KC=4; B=64
idx=np.load('/tmp/screen_sim_c4_idx.npy')
for t in [64*100, 64*3000, 64*7000, 64*9000]:
    # batch b starts at pod t; b-3 starts at t-192; state for b-3 snapshot: before pod t-192 (approx: sequential state)
    ac,am,ap = state_at(cl, idx, t-3*B)
    Kold = keys(cl, slice(t-3*B, t-2*B), ac, am, ap)   # batch b-3 keys at its snapshot
    ac2,am2,ap2 = state_at(cl, idx, t)
    K = keys(cl, slice(t, t+B), ac2, am2, ap2)        # batch b keys
    R=(n+G-1)//G
    def wg(Kx):
        Kp=np.full((Kx.shape[0],G*R),-np.inf); Kp[:,:n]=Kx; return Kp.reshape(Kx.shape[0],R,G)
    Ko=wg(Kold); Kb=wg(K)
    # suspects: union over pods of b-3 of each WG's top-KC rows
    sus=np.zeros((R,G),bool)
    if MODE == 'own':
        top=np.argsort(-Ko,axis=1)[:,:KC,:]   # [pod, KC, G] row ids
        for g in range(G): sus[np.unique(top[:,:,g]),g]=True
    else:
        u=np.unique(np.argsort(-Kold,axis=1)[:,:16])   # merged lists of b-3: global top-16 nodes per pod
        sus[u//G, u%G]=True
    # touched by exports b-5,b-4 (placements of pods t-5B..t-3B)
    for pl in idx[t-5*B:t-3*B]:
        if pl>=0: sus[pl//G, pl%G]=True
    eps=4e-5
    L_all=-np.sort(-Kb,axis=1)[:,KC-1,:]-eps
    Kx=np.where(sus[None],-np.inf,Kb)
    L_ex=-np.sort(-Kx,axis=1)[:,KC-1,:]-eps
    need_all=(Kb+eps>=L_all[:,None,:]).sum(axis=(0,1))   # pairs per WG
    need_ex=(Kb+eps>=L_ex[:,None,:]).sum(axis=(0,1))
    print(f"t={t}: suspects/WG mean {sus.sum(0).mean():.1f}; pairs/WG exact-L {need_all.mean():.0f} (max {need_all.max()}), suspects excluded {need_ex.mean():.0f} (max {need_ex.max()})")
