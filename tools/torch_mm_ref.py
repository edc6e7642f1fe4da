import torch
dev='cuda'
M,H=32000,512
D=2*H
x=torch.randn(M,D,dtype=torch.bfloat16,device=dev)
w=torch.randn(8*H,D,dtype=torch.bfloat16,device=dev)
dg=torch.randn(M,8*H,dtype=torch.bfloat16,device=dev)
def t(f,fl,name):
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    us=e0.elapsed_time(e1)*1000/20
    print('%s %.1f us %.0f TF/s'%(name,us,fl/us/1e6))
t(lambda: x@w.t(), 2*M*8*H*D, 'fwd bf16out')
t(lambda: torch.mm(x, w.t(), out_dtype=torch.float32) if hasattr(torch.mm,'__call__') else None, 2*M*8*H*D, 'fwd f32out')
t(lambda: dg@w, 2*M*8*H*D, 'dX')
t(lambda: dg.t()@x, 2*M*8*H*D, 'dW')
