import sys, numpy as np, time
sys.path[:0]=['oracle']
import pyoracle
NS=40000; ND=24000; B=1000
for seed in (41,43):
    t=time.time()
    acc=np.zeros(ND//B)
    for i in range(NS):
        st=pyoracle.rng_init(seed, i)
        _,f=pyoracle.rng_draw(st,ND)
        acc+=f.astype(np.float64).reshape(-1,B).sum(1)
    m=acc/(NS*B)
    z=(m-0.5)/(np.sqrt(1/12)/np.sqrt(NS*B))
    print(seed, 'z of mean u per block of %d draws:'%B, np.round(z,1), '(%.0fs)'%(time.time()-t), flush=True)
