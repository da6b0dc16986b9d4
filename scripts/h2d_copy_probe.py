"""H2D rate of one page-locked buffer copied whole vs in many pieces (the stripped staging's
runs): is the link's effective rate lost to per-copy overheads?"""
import time

import torch

n = 2_660_000_000
host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
host.fill_(1)
dev = torch.empty(n, dtype=torch.uint8, device="cuda:0")
st = torch.cuda.Stream()
for pieces in (1, 22, 88, 350, 1400):
    step = -(-n // pieces)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            for a in range(0, n, step):
                dev[a:a + step].copy_(host[a:a + step], non_blocking=True)
        st.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"{pieces:5d} copies of {step / 1e6:8.1f} MB: {n / best / 1e9:5.1f} GB/s", flush=True)
