"""Pivot study of the round-4 frozen-QP outlier (output in
profiles/r05_n40_frozen_analysis.txt): the N = 40 condensed QP of step 3, kite
1 of test_n40_qp_kernels_vs_oracle's sequence (from tools/n40_frozen_dump.py's
gpurun_out/r05a/n40_frozen_qk1.npz), solved by a numpy replica of the oracle's
IPM (tools/warm_ipm_probe.py) with an UNEQUILIBRATED right-looking Cholesky and
the oracle's pivot safeguard: the smallest pivot relative to its diagonal per
IPM iteration, and the spread of the frozen solution under 1e-15 / 1e-14
relative perturbations of H.  Tools only (CPU).
  python tools/n40_pivot_study.py [npz]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tools')): sys.path.insert(0, p)
from oracle import ffi
from test_gpu_parity import condensed_cfgv
import warm_ipm_probe as W
BIG=1e128
fixes=[]
def chol_safe(M):
    A=M.copy(); n=A.shape[0]; L=np.zeros_like(A); nf=0; minp=np.inf
    for j in range(n):
        p=A[j,j]; minp=min(minp,p/ max(1e-300,abs(M[j,j])))
        if p<=0: nf+=1; p=BIG
        d=np.sqrt(p); L[j,j]=d
        L[j+1:,j]=A[j+1:,j]/d
        A[j+1:,j+1:]-=np.outer(L[j+1:,j],L[j+1:,j])
    fixes.append((nf,minp))
    return L
z=np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/r05a/n40_frozen_qk1.npz')
kp=ffi.load_params(); cv=condensed_cfgv(40); s,b=3,1
st,Xp,Up,_=ffi.prologue(kp,cv,40,2,z["x"][s,b],z["Xin"][s,b],z["Uin"][s,b],warm=1)
q=ffi.build_qp(kp,cv,40,2,Xp,Up)
wo,ko=ffi.qp_solve(q["H"],q["h"],q["lb"],q["ub"],q["C"],q["c"],16)
Dv=q["D"]; wg=np.concatenate([(z["ctrl_g"][s,b]-Up).reshape(-1), z["traj_g"][s,b][0,13:15]-Xp[0,13:15]])/Dv
np.linalg.cholesky=chol_safe
w,_,_,it,r=W.ipm(q,16,z_init=20.0)
print("unperturbed: it",it,"r %.1e"%r,"dist oracle %.1e gpu %.1e"%(np.abs(w-wo).max(),np.abs(w-wg).max()))
print(" per-iteration (pivot fixes, min relative pivot):", [(a,'%.0e'%m) for a,m in fixes])
res=[]
for eps in (1e-15,1e-14):
    for seed in range(30):
        fixes.clear()
        E=np.random.default_rng(seed).normal(size=q["H"].shape); E=(E+E.T)/2
        q2=dict(q); q2["H"]=q["H"]*(1+eps*E)
        w,_,_,it,r=W.ipm(q2,16,z_init=20.0)
        res.append((eps,seed,it,r,np.abs(w-wo).max(),np.abs(w-wg).max(),sum(a for a,_ in fixes)))
res=np.array(res)
for eps in (1e-15,1e-14):
    r=res[res[:,0]==eps]
    print(eps,"iters",np.unique(r[:,2]),"dist to oracle median %.1e max %.1e"%(np.median(r[:,4]),r[:,4].max()),"min dist to gpu %.1e"%r[:,5].min(),"resid max %.1e"%r[:,3].max(),"pivot fixes",np.unique(r[:,6]))
