import torch, time
M,N,K=2600,4096,4096
x=torch.randn(M,K,device="cuda").to(torch.float8_e4m3fn)
w=torch.randn(N,K,device="cuda").to(torch.float8_e4m3fn)
sa=torch.rand(M,1,device="cuda")+0.5; sb=torch.rand(1,N,device="cuda")+0.5
for name,kw in [("rowwise",dict(scale_a=sa,scale_b=sb)),("tensor",dict(scale_a=torch.tensor(1.0,device="cuda"),scale_b=torch.tensor(1.0,device="cuda")))]:
    try:
        y=torch._scaled_mm(x,w.t(),out_dtype=torch.bfloat16,**kw)
        ref=(x.float()*(kw["scale_a"] if kw["scale_a"].dim() else 1))@(w.float()*(kw["scale_b"].t() if kw["scale_b"].dim() else 1)).t()
        print(name,"ok err",((y.float()-ref).abs().max()/ref.abs().max()).item())
        for MM,NN,KK in [(2600,6144,4096),(2600,28672,4096),(2600,4096,14336),(512,28672,4096)]:
            xx=torch.randn(MM,KK,device="cuda").to(torch.float8_e4m3fn); ww=torch.randn(NN,KK,device="cuda").to(torch.float8_e4m3fn)
            a=(torch.rand(MM,1,device="cuda")+0.5) if name=="rowwise" else kw["scale_a"]; b=(torch.rand(1,NN,device="cuda")+0.5) if name=="rowwise" else kw["scale_b"]
            for _ in range(3): torch._scaled_mm(xx,ww.t(),out_dtype=torch.bfloat16,scale_a=a,scale_b=b)
            torch.cuda.synchronize(); t=time.perf_counter()
            for _ in range(20): torch._scaled_mm(xx,ww.t(),out_dtype=torch.bfloat16,scale_a=a,scale_b=b)
            torch.cuda.synchronize(); dt=(time.perf_counter()-t)/20
            print(f"  {name} {MM}x{NN}x{KK}: {dt*1e6:.1f} us {2*MM*NN*KK/dt/1e12:.0f} TF")
    except Exception as e:
        print(name,"FAIL",repr(e)[:300])
xb=torch.randn(2600,28672//7*7,device="cuda",dtype=torch.bfloat16)
