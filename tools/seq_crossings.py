import numpy as np, scipy.sparse as sp, time
n=256
e=np.ones(n); T=sp.diags([-e[:-1],2*e,-e[:-1]],[-1,0,1])
I=sp.identity(n)
A=(sp.kron(sp.kron(T,I),I)+sp.kron(sp.kron(I,T),I)+sp.kron(sp.kron(I,I),T)).tocsr()
N=n**3
b=A@np.ones(N); x=np.zeros(N)
def stats(p,G=64):
    s=np.cumsum(p)
    ex=np.frexp(s)[1]*np.sign(s)
    ch=np.nonzero(np.diff(ex))[0]+1
    return len(ch),len(np.unique(ch//G))
for cyc in range(10):
    r=b-A@x; beta=np.linalg.norm(r)
    V=[r/beta]; H=np.zeros((31,30))
    for j in range(30):
        w=A@V[-1]
        if j in (23,29):
            res=[stats(w*v) for v in V]
            print(cyc,j,'max subs',max(q[1] for q in res),'argmax',int(np.argmax([q[1] for q in res])),'sum subs',sum(q[1] for q in res),flush=True)
        for i,v in enumerate(V):
            H[i,j]=w@v
        for i,v in enumerate(V): w-=H[i,j]*v
        H[j+1,j]=np.linalg.norm(w); V.append(w/H[j+1,j])
    e1=np.zeros(31); e1[0]=beta
    y=np.linalg.lstsq(H,e1,rcond=None)[0]
    x=x+sum(yi*vi for yi,vi in zip(y,V[:30]))
