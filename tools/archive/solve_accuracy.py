"""Accuracy of the 4x4 gain solve (H + muI) K = G along the headline quadrotor
Riccati recursion (numpy, fp64): LDLT (the kernel's), cofactors (the distributed
variant, ablation bit 2048) and 2x2-block Schur, each against numpy.linalg.solve.
Output: profiles/r01/solve_accuracy_quadrotor.txt."""
import sys, numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0]=[R, os.path.join(R,'ilqr.jl_amd')]
from ilqr_amd.problems import quadrotor_batch
lq,x,u=quadrotor_batch(16,T=100,seed0=0)
mu=0.01
def ldlt_solve(H,b):
    n=4; L=np.zeros((4,4)); d=np.zeros(4); t=np.zeros((4,4))
    for k in range(n):
        dk=H[k,k]+mu-sum(L[k,p]*t[k,p] for p in range(k))
        d[k]=1/dk
        for i in range(k+1,n):
            v=H[i,k]-sum(L[i,p]*t[k,p] for p in range(k)); t[i,k]=v; L[i,k]=v*d[k]
    x=b.copy()
    for i in range(n):
        for p in range(i): x[i]-=L[i,p]*x[p]
    x*=d[:,None]
    for i in range(n-1,-1,-1):
        for p in range(i+1,n): x[i]-=L[p,i]*x[p]
    return x
def cof_solve(H,b):
    Hr=H+mu*np.eye(4)
    # lower triangle symmetric
    Hs=np.tril(Hr)+np.tril(Hr,-1).T
    C=np.zeros((4,4))
    for q in range(4):
        for c in range(4):
            rr=[k for k in range(4) if k!=q]; cc=[k for k in range(4) if k!=c]
            m=Hs[np.ix_(rr,cc)]
            t0=m[1,1]*m[2,2]-m[1,2]*m[2,1]; t1=m[1,0]*m[2,2]-m[1,2]*m[2,0]; t2=m[1,0]*m[2,1]-m[1,1]*m[2,0]
            C[q,c]=(-1)**(q+c)*(m[0,0]*t0-m[0,1]*t1+m[0,2]*t2)
    det=np.array([C[q]@Hs[q] for q in range(4)])
    X=C/det[:,None]
    return X@b
def schur_solve(H,b):
    Hr=H+mu*np.eye(4); P=Hr[:2,:2]; Q=Hr[:2,2:]; R=Hr[2:,2:]
    Pi=np.linalg.inv(P); W=Pi@Q; S=R-Q.T@W; Si=np.linalg.inv(S)
    y=Pi@b[:2]; c=b[2:]-Q.T@y; x2=Si@c; x1=y-W@x2
    return np.vstack([x1,x2])
errs={'ldlt':[], 'cof':[], 'schur':[]}
conds=[]
for bi in range(16):
    A,B,Q,R,Qf=lq.A[bi],lq.B[bi],lq.Q[bi],lq.R[bi],lq.Qf[bi]
    S=Qf+Qf.T
    for t in range(99,-1,-1):
        H=R+R.T+B.T@S@B; G=B.T@S@A
        ref=np.linalg.solve(H+mu*np.eye(4), G)
        conds.append(np.linalg.cond(H+mu*np.eye(4)))
        for k,f in (('ldlt',ldlt_solve),('cof',cof_solve),('schur',schur_solve)):
            errs[k].append(np.abs(f(H,G)-ref).max()/np.abs(ref).max())
        K=-ref
        S=Q+Q.T+A.T@S@A+K.T@H@K+K.T@G+G.T@K; S=(S+S.T)/2
print('cond max %.2e median %.2e'%(max(conds), np.median(conds)))
for k,v in errs.items(): print(k, 'max %.2e median %.2e'%(max(v), np.median(v)))
