import sys, numpy as np, time
sys.path[:0]=['oracle']
import pyoracle
NS=40000; B=990; NB=24; ND=B*NB
p=np.pi/6
for seed in (41,43):
    t=time.time()
    acc=np.zeros(NB)
    for i in range(NS):
        st=pyoracle.rng_init(seed, i)
        _,f=pyoracle.rng_draw(st,ND)
        a=np.fma(f.astype(np.float32),np.float32(2),np.float32(-1)).astype(np.float64).reshape(NB,B//3,3) if hasattr(np,'fma') else (2*f.astype(np.float64)-1).reshape(NB,B//3,3)
        acc+=((a**2).sum(2)<1).sum(1)
    ntr=NS*(B//3)
    z=(acc/ntr-p)/np.sqrt(p*(1-p)/ntr)
    print(seed,'unit-sphere acceptance z per block of %d draws:'%B,np.round(z,1),'(%.0fs)'%(time.time()-t),flush=True)
