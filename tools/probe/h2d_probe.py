import time, numpy as np, torch
torch.cuda.set_device(0)
n = 2 << 30
a = np.ones(n, dtype=np.uint8)
t = time.perf_counter(); b = a.copy(); dt = time.perf_counter() - t
print(f"host numpy copy 2 GiB: {n/dt/1e9:.1f} GB/s")
d = torch.empty(n, dtype=torch.uint8, device="cuda")
src = torch.from_numpy(a)
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(src); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"pageable H2D 2 GiB: {n/dt/1e9:.1f} GB/s")
p = torch.empty(n, dtype=torch.uint8).pin_memory()
p.copy_(src)
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(p, non_blocking=True); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"pinned H2D 2 GiB: {n/dt/1e9:.1f} GB/s")
import os; print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
