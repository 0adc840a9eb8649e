#!/usr/bin/env python
"""How dealing envs to lanes by their last step's contacts would change the
wave-gated rows (fp64 oracle, CPU only): for B envs x T
steps of the bench's workload, the mean over waves of the largest number of
gripper slots, box-box pair slots and PGS iterations per substep that a lane
of the wave needs, with the envs in index order, sorted by the previous step's
contacts, and sorted by the current step's (unknowable in advance).

  python scripts/stack_deal_sim.py stack 1024 30
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
task=sys.argv[1]; B=int(sys.argv[2]); T=int(sys.argv[3])
cfg=O.config(task,"ee")
L=O.lib()
envs=[O.new_env(cfg) for _ in range(B)]
for i,e in enumerate(envs): O.reset(cfg,e,seed=12345+i)
rng=np.random.default_rng(0xC0FFEE)
it=np.zeros((T,B,20),np.int32); nr=np.zeros((T,B),np.int32); npair=np.zeros((T,B),np.int32)
buf=np.zeros(20,np.int32)
for t in range(T):
    a=rng.uniform(-1,1,(B,O.action_dim(cfg))).astype(np.float32)
    for i,e in enumerate(envs):
        L.po_set_pgs_log(buf.ctypes.data,20)
        O.step(cfg,e,a[i],autoreset=True)
        L.po_set_pgs_log(None,0)
        it[t,i]=buf
        nr[t,i]=sum(1 for s in range(4) if e.cache.robot_id[s])
        npair[t,i]=e.cache.pair_n
W=B//64
def cost(order):
    r_slots=[];iters=[];pairs=[]
    for t in range(1,T):
        o=order(t)
        r_slots.append(nr[t][o].reshape(W,64).max(1).mean())
        iters.append(it[t][o].reshape(W,64,20).max(1).mean())
        pairs.append((npair[t][o].reshape(W,64).max(1)).mean())
    return np.mean(r_slots), np.mean(iters), np.mean(pairs)
ident=lambda t: np.arange(B)
prev=lambda t: np.argsort(-(nr[t-1]*8+np.minimum(npair[t-1],4)), kind="stable")
prevp=lambda t: np.argsort(-(np.minimum(npair[t-1],4)*8+nr[t-1]), kind="stable")
cur=lambda t: np.argsort(-(nr[t]*8+np.minimum(npair[t],4)), kind="stable")
print(task, "lane mean robot slots", nr[1:].mean(), "pair", npair[1:].mean(), "iters", it[1:].mean())
print(" index order (robot slots, iters, pair):", cost(ident))
print(" sorted by prev robot->pair:", cost(prev))
print(" sorted by prev pair->robot:", cost(prevp))
print(" sorted by current (oracle):", cost(cur))
print(" persistence corr robot slots t vs t-1:", np.corrcoef(nr[1:-1].ravel(), nr[2:].ravel())[0,1])
