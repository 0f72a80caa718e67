"""Probe: can timing events be captured inside a hipGraph (torch.cuda.Event(external=True))?"""
import torch
x = torch.randn(1 << 24, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.Stream()
evs = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(4)]
with torch.cuda.stream(s):
    y.copy_(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        evs[0].record()
        y.copy_(x)
        evs[1].record()
        y.mul_(2)
        y.mul_(2)
        evs[2].record()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print("copy ms", evs[0].elapsed_time(evs[1]), "2x mul ms", evs[1].elapsed_time(evs[2]))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); y.copy_(x); b.record(); torch.cuda.synchronize()
    print("eager copy ms", a.elapsed_time(b))
