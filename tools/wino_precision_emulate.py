"""Host emulation of where the Winograd towers' rounding error comes from
(planning tool; nothing in the product depends on it): F(8x8) with each of U,
V, the GEMM / M and the transforms in fp32 or fp64, and F(4x4) for contrast,
against the float64 forward of the same weights (oracle/torch_ref.forward), on
seeded random boards. Activations between layers are fp32 in every case (the
product's storage).

    python tools/wino_precision_emulate.py stress 4 > profiles/r04_f88_precision_emulation.log
"""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fractions import Fraction as Fr
from wino_emulate import toom_cook, _heads
from knightvision_amd.weights import synthetic_state_dict
from knightvision_amd.ai import codes_to_planes
from oracle import torch_ref
F32=np.float32
P88=[Fr(0),Fr(2,5),Fr(-2,5),Fr(4,5),Fr(-4,5),Fr(5,4),Fr(-5,4),Fr(2),Fr(-2)]
P44=[Fr(0),Fr(1),Fr(-1),Fr(2),Fr(-2)]
def conv(x, w, m, AT,G,BT, vp, gp, op, seq):
    # x [B,8,8,C] ; one tile per 8 (m=8) or 2x2 tiles (m=4)
    B,_,_,Cin=x.shape; Cout=w.shape[0]; n=m+2
    U=np.einsum("ak,oikl,bl->abio",G,w,G)
    U=U.astype(gp)
    xp=np.zeros((B,18,18,Cin)); xp[:,1:9,1:9]=x
    out=np.zeros((B,8,8,Cout))
    BTv=BT.astype(vp); ATo=AT.astype(op)
    for ty in range(0,8,m):
      for tx in range(0,8,m):
        d=xp[:,ty:ty+n,tx:tx+n].astype(vp)
        V=np.einsum("ai,bicq->bacq",BTv,d).astype(vp); V=np.einsum("bj,xajq->xabq",BTv,V).astype(vp)
        Vf=V.reshape(B,n*n,Cin); Uf=U.reshape(n*n,Cin,Cout)
        if seq:
            acc=np.zeros((B,n*n,Cout),F32)
            for k in range(0,Cin,2):
                acc=((acc+(Vf[:,:,k,None].astype(F32)*Uf[None,:,k,:].astype(F32)).astype(F32)).astype(F32)+(Vf[:,:,k+1,None].astype(F32)*Uf[None,:,k+1,:].astype(F32)).astype(F32)).astype(F32)
            M=acc
        else:
            M=np.einsum("bxk,xko->bxo",Vf.astype(np.float64),Uf.astype(np.float64))
        M=M.astype(op).reshape(B,n,n,Cout)
        Y=np.einsum("ia,bacq->bicq",ATo,M).astype(op); Y=np.einsum("jc,bicq->bijq",ATo,Y).astype(op)
        out[:,ty:ty+m,tx:tx+m]=Y
    return out
def fwd(sd,planes,m,tabs,vp,gp,op,seq):
    t={k:np.asarray(v,dtype=np.float64) for k,v in sd.items()}
    def fold(c,b):
        sc=t[b+".weight"]/np.sqrt(t[b+".running_var"]+1e-5); return sc, t[b+".bias"]+(t[c+".bias"]-t[b+".running_mean"])*sc
    x=torch.nn.functional.conv2d(torch.from_numpy(planes.astype(np.float64)),torch.from_numpy(t["conv1.weight"]),torch.from_numpy(t["conv1.bias"]),padding=1).numpy()
    sc,sh=fold("conv1","bn1")
    x=np.maximum((x-t["conv1.bias"][None,:,None,None])*sc[None,:,None,None]+sh[None,:,None,None],0).transpose(0,2,3,1).astype(F32)
    def cbr(x,c,b,res=None):
        y=conv(x,t[c+".weight"],m,*tabs,vp,gp,op,seq); sc,sh=fold(c,b)
        y=(y*sc+sh).astype(F32)
        if res is not None: y=(y+res).astype(F32)
        return np.maximum(y,0).astype(F32)
    x=cbr(x,"conv2","bn2")
    for r in range(5):
        h=cbr(x,f"res_blocks.{r}.conv1",f"res_blocks.{r}.bn1"); x=cbr(h,f"res_blocks.{r}.conv2",f"res_blocks.{r}.bn2",res=x)
    sdt={k:torch.from_numpy(v) for k,v in t.items()}
    return _heads(sdt, torch.from_numpy(x.transpose(0,3,1,2).astype(np.float64)))
def main():
    variant=sys.argv[1]; nb=int(sys.argv[2])
    sd=synthetic_state_dict(42,variant)
    rng=np.random.default_rng(5); codes=rng.integers(0,13,size=(nb,64))*(rng.random((nb,64))<0.4)
    planes=codes_to_planes(codes)
    p64,v64=torch_ref.forward({k:torch.from_numpy(np.asarray(v,dtype=np.float64)) for k,v in sd.items()},torch.from_numpy(planes.astype(np.float64)))
    p64=p64.numpy(); v64=v64.numpy().reshape(-1)
    T88=toom_cook(P88,8); T44=toom_cook(P44,4)
    D=np.float64
    cases=[("F88 all fp32 seq",8,T88,F32,F32,F32,True),
           ("F88 V,U f32; GEMM f64; M,out f64",8,T88,F32,F32,D,False),
           ("F88 V f64,U f32; GEMM f64; out f64",8,T88,D,F32,D,False),
           ("F88 V f32,U f64; GEMM f64; out f64",8,T88,F32,D,D,False),
           ("F88 all f64",8,T88,D,D,D,False),
           ("F88 V,U,GEMM f64; M,out f32",8,T88,D,D,F32,False),
           ("F44 all fp32 seq",4,T44,F32,F32,F32,True),
           ("F44 V,U f32, GEMM f64, out f64",4,T44,F32,F32,D,False)]
    for name,m,tabs,vp,gp,op,seq in cases:
        p,v=fwd(sd,planes,m,tabs,vp,gp,op,seq)
        print(f"{variant} {name:40s} dlogit {np.abs(p-p64).max():.3e} dvalue {np.abs(v-v64).max():.3e}",flush=True)


if __name__ == "__main__":
    main()
