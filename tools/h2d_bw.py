"""H2D bandwidth: pageable vs pinned host memory (sizing the bytes-API design)."""
import time
import torch
n = 1 << 30
for kind in ("pageable", "pinned"):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
    h.fill_(1)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d.copy_(h); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        d.copy_(h, non_blocking=(kind == "pinned"))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(kind, "H2D %.1f GB/s" % (n / dt / 1e9))
    t0 = time.perf_counter()
    for _ in range(3):
        h.copy_(d, non_blocking=(kind == "pinned"))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(kind, "D2H %.1f GB/s" % (n / dt / 1e9))
