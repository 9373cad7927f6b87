import torch, statistics, sys
sys.path.insert(0, '.')
from exploring_flash_attention_amd import ops
B,H,L,d = 32,8,4096,128
g = torch.Generator(device='cuda').manual_seed(0)
q,k,v = (torch.randn(B,H,L,d,device='cuda',dtype=torch.bfloat16,generator=g) for _ in range(3))
res = {}
for name, pd in (("fp32", torch.float32), ("bf16", torch.bfloat16), ("f16s", ops.PARTIAL_FP16_SCALED)):
    nb, ns = ops.v2_workspace_bytes(B,H,L,d,4,q.dtype,pd)
    ws = torch.empty(nb, dtype=torch.uint8, device='cuda')
    out = torch.empty_like(q)
    for _ in range(30): ops.attention_v2(q,k,v,4,partial_dtype=pd,out=out,workspace=ws)
    ts=[]
    for _ in range(5):
        e0,e1=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): ops.attention_v2(q,k,v,4,partial_dtype=pd,out=out,workspace=ws)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1)/10)
    ms = statistics.median(ts)
    print(f"C4 KVTPB=4 partials {name}: {ms:.3f} ms {4*B*H*L*L*d/ms/1e9:.0f} TFLOP/s workspace {nb/1e9:.2f} GB splits {ns}", flush=True)
