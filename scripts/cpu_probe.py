"""Probe the host CPU speed of the reference's fp16 CPU ops (for the bench cpu_baseline sizing)."""
import os, time, torch, torch.nn.functional as F
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), "torch threads", torch.get_num_threads(), flush=True)
torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
x = torch.randn(2, 320, 64, 64).half(); w = torch.randn(320, 320, 3, 3).half() * 0.02
for dt in (torch.float16, torch.float32):
    xx, ww = x.to(dt), w.to(dt)
    F.conv2d(xx, ww, padding=1)
    t = time.time(); F.conv2d(xx, ww, padding=1); d = time.time() - t
    print(dt, f"conv320@64 b2: {d*1e3:.1f} ms = {2*2*4096*320*2880/d/1e9:.1f} GFLOP/s", flush=True)
a = torch.randn(8192, 320).half(); b = torch.randn(2560, 320).half()
for dt in (torch.float16, torch.float32):
    aa, bb = a.to(dt), b.to(dt); F.linear(aa, bb)
    t = time.time(); F.linear(aa, bb); d = time.time() - t
    print(dt, f"linear 8192x2560x320: {d*1e3:.1f} ms = {2*8192*2560*320/d/1e9:.1f} GFLOP/s", flush=True)
