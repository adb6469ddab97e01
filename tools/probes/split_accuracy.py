# Dot-product error of the split contractions (DESIGN.md §3b'): bf16 x6 vs scaled fp16 x3 / x4 vs an fp32 fma chain, numpy (CPU).
import numpy as np
rng=np.random.default_rng(0)
def bf_split(x):
    x=x.astype(np.float32); u=x.view(np.uint32)
    hi=(u&0xFFFF0000).view(np.float32); r=(x-hi).astype(np.float32)
    mid=(r.view(np.uint32)&0xFFFF0000).view(np.float32); lo=(r-mid).astype(np.float32)
    return hi,mid,lo
def f16_split(x, scale):
    xs=(x*scale).astype(np.float32)
    hi=xs.astype(np.float16).astype(np.float32); r=(xs-hi).astype(np.float32)
    lo=r.astype(np.float16).astype(np.float32)
    return hi,lo
def dot(a,b): # exact float64 sum of float32 products, then one rounding
    return (a.astype(np.float64)*b.astype(np.float64)).sum(-1)
N=200000; K=32
for mag in [1.0, 1e-3, 30.0]:
    a=(rng.standard_normal((N,K))*mag).astype(np.float32)
    b=(rng.uniform(-0.3,0.3,(N,K))).astype(np.float32)
    ex=dot(a,b); den=np.abs(a.astype(np.float64)*b).sum(-1)
    ah,am,al=bf_split(a); bh,bm,bl=bf_split(b)
    x6=dot(ah,bh)+dot(ah,bm)+dot(am,bh)+dot(ah,bl)+dot(al,bh)+dot(am,bm)
    ea=2.0**(14-np.floor(np.log2(np.abs(a).max(-1,keepdims=True)))); eb=2.0**(14-np.floor(np.log2(np.abs(b).max())))
    Ah,Al=f16_split(a,ea); Bh,Bl=f16_split(b,eb)
    s=(ea[:,0]*eb)
    x3=(dot(Ah,Bh)+dot(Ah,Bl)+dot(Al,Bh))/s
    x4=x3+dot(Al,Bl)/s
    f32=np.zeros(N,np.float32)
    for k in range(K): f32=(f32+a[:,k]*b[:,k]).astype(np.float32)
    for nm,v in [("f32 chain",f32),("bf x6",x6),("f16 x3",x3),("f16 x4",x4)]:
        e=np.abs(v-ex)/den
        print(mag,nm,"max %.2f mean %.2f (log2 of err / sum|ab|)"%(np.log2(e.max()),np.log2(e.mean()+1e-300)))
