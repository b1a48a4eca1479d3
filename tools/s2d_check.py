#!/usr/bin/env python3
"""Index-level float64 emulation of the super-pixel strided dgrad (k_pack_s2d
packing + the stride-1 window conv + the dX block store of k_conv_fwd_p<BN, true>)
against the adjoint of the padded strided conv, at the strided cases of
tests/test_ops_gpu.py and wr_resnet-like shapes.  CPU only.  usage: python tools/s2d_check.py"""
import torch, torch.nn.functional as F, math
torch.manual_seed(0)
def same(n,k,s):
    o=-(-n//s); pad=max((o-1)*s+k-n,0); return o, pad//2
def check(N,H,W,C,K,R,st,padmode):
    if padmode=="same":
        P,pt=same(H,R,st); Q,pl=same(W,R,st)
    else:
        P=(H-R)//st+1; Q=(W-R)//st+1; pt=pl=0
    S=R
    w=torch.randn(K,R,S,C,dtype=torch.float64)
    dy=torch.randn(N,P,Q,K,dtype=torch.float64)
    # reference
    xr=torch.zeros(N,C,H,W,dtype=torch.float64,requires_grad=True)
    xp=F.pad(xr,(pl,max(0,(Q-1)*st+S-W-pl),pt,max(0,(P-1)*st+R-H-pt)))
    (F.conv2d(xp,w.permute(0,3,1,2),stride=st)*dy.permute(0,3,1,2)).sum().backward()
    ref=xr.grad.permute(0,2,3,1)
    # s2d
    mr=-(-R//st); ms=-(-S//st); kout=st*st*C
    Wp=torch.zeros(kout, mr*ms*K, dtype=torch.float64)
    for o in range(kout):
        ab=o//C; c=o%C; a=ab//st; b=ab%st
        for tap in range(mr*ms):
            tr=tap//ms; tc=tap%ms
            r=a+st*(mr-1-tr); sx=b+st*(ms-1-tc)
            if r<R and sx<S:
                Wp[o,tap*K:(tap+1)*K]=w[:,r,sx,c]
    U=-(-(H+pt)//st); V=-(-(W+pl)//st)
    cpt, cpl = mr-1, ms-1
    dyp=F.pad(dy.permute(0,3,1,2),(cpl, V+ms, cpt, U+mr))
    out=torch.zeros(N,U,V,kout,dtype=torch.float64)
    for tap in range(mr*ms):
        tr=tap//ms; tc=tap%ms
        patch=dyp[:,:,tr:tr+U,tc:tc+V].permute(0,2,3,1)  # N U V K
        out+=patch@Wp[:,tap*K:(tap+1)*K].T
    dx=torch.full((N,H,W,C),float('nan'),dtype=torch.float64)
    for u in range(U):
        for v in range(V):
            for a in range(st):
                for b in range(st):
                    h=u*st+a-pt; ww=v*st+b-pl
                    if 0<=h<H and 0<=ww<W:
                        dx[:,h,ww,:]=out[:,u,v,(a*st+b)*C:(a*st+b+1)*C]
    err=(dx-ref).abs().max().item()
    print(N,H,W,C,K,R,st,padmode,"pt",pt,"pl",pl,"err",err, "nan", torch.isnan(dx).any().item())
for case in [(1,16,33,4,8,3,2,"same"),(1,16,33,4,8,1,2,"valid"),(1,22,31,4,8,3,3,"same"),(1,22,31,4,8,1,3,"valid"),
             (1,16,34,4,8,3,2,"same"),(1,21,29,4,4,3,2,"valid"),(1,23,35,4,8,3,3,"same"),(1,3,5,4,4,3,2,"same"),
             (1,128,51,2,4,3,2,"same"),(1,64,25,2,4,3,3,"same"),(1,64,25,2,4,1,3,"valid")]:
    check(*case)
