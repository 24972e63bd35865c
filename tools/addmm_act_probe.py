import torch, json
d="cuda"
res={}
for B in (2048, 16384):
    f=torch.randn(B,512,device=d); W=torch.randn(512,512,device=d); b=torch.randn(512,device=d)
    h3=torch.randn(B,3136,device=d); Wf=torch.randn(512,3136,device=d)
    def t(fn, it=30):
        for _ in range(3): fn()
        torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it): fn()
        e.record(); torch.cuda.synchronize(); return s.elapsed_time(e)/it
    r1=torch.addmm(b,f,W.t()).relu_(); r2=torch._addmm_activation(b,f,W.t())
    res[f"{B}_equal_extra"]=bool(torch.equal(r1,r2))
    res[f"{B}_extra_addmm_relu"]=t(lambda: torch.addmm(b,f,W.t()).relu_())
    res[f"{B}_extra_addmm_act"]=t(lambda: torch._addmm_activation(b,f,W.t()))
    res[f"{B}_fc_addmm_relu"]=t(lambda: torch.addmm(b,h3,Wf.t()).relu_())
    res[f"{B}_fc_addmm_act"]=t(lambda: torch._addmm_activation(b,h3,Wf.t()))
    r1=torch.addmm(b,h3,Wf.t()).relu_(); r2=torch._addmm_activation(b,h3,Wf.t())
    res[f"{B}_equal_fc"]=bool(torch.equal(r1,r2))
print(json.dumps({k:(round(v,4) if isinstance(v,float) else v) for k,v in res.items()}))
