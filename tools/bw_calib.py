"""Diagnostic: achievable HBM bandwidth of plain streaming kernels on this box (torch ops,
HIP events, min of 10): read-only (sum), write-only (fill), copy; sizes like C2's streams."""
import torch

dev = torch.device("cuda", 0)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t(fn):
    ts = []
    for _ in range(10):
        ev0.record()
        fn()
        ev1.record()
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    return min(ts)


a = torch.ones(10**8, dtype=torch.int64, device=dev)  # 800 MB
b = torch.empty(10**8, dtype=torch.int64, device=dev)
c = torch.empty(75 * 10**6, dtype=torch.int64, device=dev)  # 600 MB
ms = t(lambda: a.sum())
print(f"read 800 MB (sum): {ms:.3f} ms = {0.8 / ms:.2f} TB/s")
ms = t(lambda: c.fill_(3))
print(f"write 600 MB (fill): {ms:.3f} ms = {0.6 / ms:.2f} TB/s")
ms = t(lambda: b.copy_(a))
print(f"copy 800 -> 800 MB: {ms:.3f} ms = {1.6 / ms:.2f} TB/s")
