import torch, time
x = torch.zeros(1, device="cuda")
big = torch.zeros(1 << 20, device="cuda")
def run(fn, n=500):
    for _ in range(10): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n): fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    tg = e0.elapsed_time(e1) * 1e3 / n
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    te = e0.elapsed_time(e1) * 1e3 / n
    return tg, te
print("tiny add graph/eager us:", run(lambda: x.add_(1)))
print("4MB add graph/eager us:", run(lambda: big.add_(1)))
