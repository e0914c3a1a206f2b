"""Host emulation (planning only): F(8x8) with one conv layer at a time in fp32 and the rest in fp64,
stress weights (profiles/r04_f88_precision_emulation.log). Reuses tools/wino_precision_emulate.py."""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'wino_precision_emulate.py')).read().split("variant=sys.argv[1]")[0])
F32=np.float32; D=np.float64
def fwd_mixed(sd, planes, tabs, f32_layers):
    t={k:np.asarray(v,dtype=np.float64) for k,v in sd.items()}
    def fold(c,b):
        sc=t[b+".weight"]/np.sqrt(t[b+".running_var"]+1e-5); return sc, t[b+".bias"]+(t[c+".bias"]-t[b+".running_mean"])*sc
    x=torch.nn.functional.conv2d(torch.from_numpy(planes.astype(np.float64)),torch.from_numpy(t["conv1.weight"]),torch.from_numpy(t["conv1.bias"]),padding=1).numpy()
    sc,sh=fold("conv1","bn1")
    x=np.maximum((x-t["conv1.bias"][None,:,None,None])*sc[None,:,None,None]+sh[None,:,None,None],0).transpose(0,2,3,1).astype(F32)
    li=[1]
    def cbr(x,c,b,res=None):
        l=li[0]; li[0]+=1
        if l in f32_layers: y=conv(x,t[c+".weight"],8,*tabs,F32,F32,F32,False)
        else: y=conv(x,t[c+".weight"],8,*tabs,D,D,D,False)
        sc,sh=fold(c,b)
        y=(y*sc+sh).astype(F32)
        if res is not None: y=(y+res).astype(F32)
        return np.maximum(y,0).astype(F32)
    x=cbr(x,"conv2","bn2")
    for r in range(5):
        h=cbr(x,f"res_blocks.{r}.conv1",f"res_blocks.{r}.bn1"); x=cbr(h,f"res_blocks.{r}.conv2",f"res_blocks.{r}.bn2",res=x)
    sdt={k:torch.from_numpy(v) for k,v in t.items()}
    return _heads(sdt, torch.from_numpy(x.transpose(0,3,1,2).astype(np.float64)))
variant=sys.argv[1]; nb=int(sys.argv[2])
sd=synthetic_state_dict(42,variant)
rng=np.random.default_rng(5); codes=rng.integers(0,13,size=(nb,64))*(rng.random((nb,64))<0.4)
planes=codes_to_planes(codes)
p64,v64=torch_ref.forward({k:torch.from_numpy(np.asarray(v,dtype=np.float64)) for k,v in sd.items()},torch.from_numpy(planes.astype(np.float64)))
p64=p64.numpy(); v64=v64.numpy().reshape(-1)
T88=toom_cook(P88,8)
cfgs=[("all f64",set())]+[(f"layer {l} fp32",{l}) for l in range(1,12)]+[("layers 1-6 fp32",set(range(1,7))),("layers 7-11 fp32",set(range(7,12)))]
for name,s in cfgs:
    p,v=fwd_mixed(sd,planes,T88,s)
    print(f"{variant} {name:18s} dlogit {np.abs(p-p64).max():.3e} dvalue {np.abs(v-v64).max():.3e}",flush=True)
