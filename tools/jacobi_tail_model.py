"""Planning model: norm-sorted Jacobi sweeps as eigen_kernel runs them,
against the same sweeps whose confirming last sweep is replaced by a Gram check + conflict-free
rounds over the pairs above tol, both followed by the first-order refinement; scored against LAPACK.
Input: gpurun_out/c4_users.npz (tools/dump_c4_users.py).
usage: python tools/jacobi_tail_model.py kmin kmax n_users switch_count   (e.g. 170 180 8 400)
"""
import sys, numpy as np
sys.path.insert(0,'tools')
from jacobi_gram_model import rotate, schedule, accuracy
f32=np.float32
z=np.load('gpurun_out/c4_users.npz')
kmin,kmax,mx,T=int(sys.argv[1]),int(sys.argv[2]),int(sys.argv[3]),int(sys.argv[4])
DELTA=1e-2;STOP=1e-3
def refine(B):
    Bw=B.astype(np.float64); F=(B.T@B).astype(np.float64)
    mu2=np.diag(F); mu=np.sqrt(mu2); far=np.abs(mu[:,None]-mu[None,:])>DELTA
    K=np.where(far, F/np.where(far, mu2[:,None]-mu2[None,:],1.0),0.0)
    return Bw-Bw@K
def score(A,Bw):
    k=len(A); nrm=np.sqrt((Bw**2).sum(0)); V=Bw/nrm
    rq=np.einsum('ij,ij->j',V,A@V); o=np.argsort(rq); V=V[:,o]
    err=np.abs(rq[o]-np.linalg.eigvalsh(A)).max(); _,res,proj=accuracy(A,rq[o],V)
    return err,proj,np.abs(V.T@V-np.eye(k)).max()
keys=[x for x in z.files if x.startswith('W_') and kmin<=z[x].shape[0]<=kmax][:mx]
tb=tn=0
for key in keys:
    Wu=z[key].astype(np.float64); k=len(Wu)
    d=Wu.sum(1); d[d==0]=1; s=np.sqrt(1/d)
    L2=(s[:,None]*(np.diag(d)-Wu))*s[None,:]; A=np.tril(L2)+np.tril(L2,-1).T
    tol=f32(np.sqrt(k)*2.0**-22); steps=schedule(k); nst=len(steps)
    out=[]
    for scheme in ('base','gram'):
        B=(A+np.eye(k)).astype(f32); sw=0; extra=0; note=''
        while sw<15:
            nrm=(B.astype(np.float64)**2).sum(0); o=np.argsort(-nrm,kind='stable'); B=B[:,o]
            flag=False; n8=0
            for P,Q in steps:
                xp,xq=B[:,P],B[:,Q]; al=(xp*xp).sum(0);be=(xq*xq).sum(0);ga=(xp*xq).sum(0)
                g2=ga*ga;ab=al*be;close=(be-al)**2<=2*DELTA**2*(al+be); rot=g2>tol*tol*ab
                f=(g2>STOP**2*ab)|((g2>(8*tol)**2*ab)&close); flag|=bool((f&rot).any()); n8+=int((f&rot).sum())
                rotate(B,P,Q,tol*tol)
            sw+=1
            if not flag: break
            if scheme=='gram' and n8<=T:
                F=(B.T@B).astype(np.float64); dg=np.diag(F); al=dg[:,None]; be=dg[None,:]
                g2=F*F; ab=al*be; close=(be-al)**2<=2*DELTA**2*(al+be)
                f=(g2>STOP**2*ab)|((g2>(8*tol)**2*ab)&close); iu=np.triu_indices(k,1)
                extra+=1
                if f[iu].any(): note+=f'chk{sw}:fail '; continue
                v=(g2>tol*tol*ab)[iu]; P=iu[0][v]; Q=iu[1][v]; rounds=0
                key_=P*4096+Q; live=np.ones(len(P),bool)
                while live.any():
                    cm=np.full(k,np.iinfo(np.int64).max); idx=np.nonzero(live)[0]
                    np.minimum.at(cm,P[idx],key_[idx]); np.minimum.at(cm,Q[idx],key_[idx])
                    sel=idx[(cm[P[idx]]==key_[idx])&(cm[Q[idx]]==key_[idx])]
                    rotate(B,P[sel],Q[sel],f32(0)); live[sel]=False; rounds+=1
                note+=f'chk{sw}:ok list{len(P)} rd{rounds}'; extra+=rounds*3000/50000; break
        err,pj,orth=score(A,refine(B))
        cyc=sw*nst*2300*(k/180)+extra*50000*(k/180)**3
        if scheme=='base': tb+=cyc
        else: tn+=cyc
        out.append(f"{scheme}: sw={sw} {note} ev={err:.1e} pj={pj:.1e} or={orth:.1e} Mc={cyc/1e6:.2f}")
    print(key,k,' | '.join(out),flush=True)
print('base',tb/len(keys)/1e6,'gram',tn/len(keys)/1e6)
