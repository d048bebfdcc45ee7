"""Warm-started lazy re-solve study (round 5, tools only): on the tight |omega| <= 3
loop of tests/test_state_bounds.py, QPs that need lazy rows are re-solved by the
numpy replica of the oracle IPM (tools/warm_ipm_probe.py) cold, and warm from
the round-0 iterate (old slacks / multipliers kept; or reset to sqrt(mu)).
  python tools/lazy_warm_probe.py"""
import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/tools')
from oracle import ffi
from test_state_bounds import tight_config, x0_batch, within_bound
from warm_ipm_probe import ipm
kp=ffi.load_params(); N,M,K=20,2,16
c=tight_config(N); cv=ffi.cfg_vector(c)
B=64
x=x0_batch(B, cv, 11000)
Xo=np.zeros((B,N+1,15)); Uo=np.zeros((B,N,4))
lb=np.array(c["lbx"]); ub=np.array(c["ubx"])
res=[]
for step in range(8):
    for b in range(B):
        st,Xp,Up,_=ffi.prologue(kp,cv,N,M,x[b],Xo[b],Uo[b],warm=int(step>0))
        q=ffi.build_qp(kp,cv,N,M,Xp,Up,want_G=True)
        w,s,z,it0,r0=ipm(q,K,z_init=20.0)
        if r0>=1e-6: continue
        dw=q["D"]*w
        X1=Xp+q["g"]+np.einsum("kin,n->ki",q["G"],dw)
        viol=[]
        for k in range(1,N+1):
            for i in range(1,13):
                xv=X1[k,i]
                if xv<lb[i]-1e-8*max(1,abs(lb[i])): viol.append(((lb[i]-xv)/max(1,abs(lb[i])),k,i,+1))
                if xv>ub[i]+1e-8*max(1,abs(ub[i])): viol.append(((xv-ub[i])/max(1,abs(ub[i])),k,i,-1))
        if not viol: continue
        viol.sort(reverse=True)
        q2=dict(q); C=list(q["C"]); cc=list(q["c"])
        for (_,k,i,side) in viol[:4]:
            bnd=lb[i] if side>0 else ub[i]
            C.append(side*q["G"][k,i]*q["D"]); cc.append(side*(bnd-Xp[k,i]-q["g"][k,i]))
        q2["C"]=np.array(C); q2["c"]=np.array(cc)
        _,_,_,itc,rc=ipm(q2,K,z_init=20.0)
        n=len(w); m_old=len(q["c"]); madd=len(cc)-m_old
        # warm: previous w pulled into the box interior, old slacks/multipliers kept, new rows s=max(resid,0.1), z=z0
        mar=0.05*(q["ub"]-q["lb"]); w0=np.clip(w,q["lb"]+mar,q["ub"]-mar)
        A=np.vstack([np.eye(n),-np.eye(n),q2["C"]]); bb=np.concatenate([q["lb"],-q["ub"],q2["c"]])
        sw=np.maximum(A@w0-bb,1e-2); zw=np.concatenate([np.maximum(z,1e-2), np.full(madd,20.0)])
        _,_,_,itw,rw=ipm(q2,K,w0=w0,s0=sw,z0=zw,z_init=20.0)
        # warm 2: mu-based reset of all multipliers
        mu=max(s@z/len(s),1e-3)
        sw2=np.maximum(A@w0-bb,np.sqrt(mu)); zw2=np.maximum(np.concatenate([z,np.full(madd,20.0)]),np.sqrt(mu))
        _,_,_,itw2,rw2=ipm(q2,K,w0=w0,s0=sw2,z0=zw2,z_init=20.0)
        res.append((itc,rc,itw,rw,itw2,rw2))
    for b in range(B):
        ffi.rti_step(kp,cv,N,M,K,x[b:b+1],Xo[b:b+1],Uo[b:b+1],warm=int(step>0))
    x=Xo[:,1,:].copy()
r=np.array(res)
print("cases",len(r),"cold mean it %.2f (fail %d)"%(r[:,0].mean(),(r[:,1]>=1e-8).sum()),
      "warm %.2f (fail %d)"%(r[:,2].mean(),(r[:,3]>=1e-8).sum()), "warm2 %.2f (fail %d)"%(r[:,4].mean(),(r[:,5]>=1e-8).sum()))
