import torch, time
torch.cuda.set_device(0)
for mb in (41, 64, 256):
    n = mb * 1024 * 1024 // 8
    bufs = [torch.empty(n, dtype=torch.float64, device='cuda') for _ in range(8)]
    for b in bufs: b.fill_(0.5)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for it in range(50):
        b = bufs[it % 8]
        s.record(); b.fill_(1.0); e.record(); e.synchronize(); ts.append(s.elapsed_time(e))
    ts.sort()
    t = ts[len(ts)//2]
    print(f"fill {mb} MB: median {t*1e3:.1f} us -> {n*8/t/1e6:.0f} GB/s", flush=True)
