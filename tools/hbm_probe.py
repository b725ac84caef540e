#!/usr/bin/env python3
"""HBM reference rates with stock torch kernels (diagnostic)."""
import torch

dev = torch.device("cuda")
n_w = 1_258_291_200          # the C2 repair bytes
n_r = 5_033_164_800          # the C2 source bytes
a = torch.empty(n_w, dtype=torch.uint8, device=dev)
b = torch.empty(n_w, dtype=torch.uint8, device=dev)
big = torch.randint(0, 255, (n_r // 8,), dtype=torch.int64, device=dev)


def t(f, reps=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ms = t(lambda: a.fill_(7))
print(f"fill 1.26GB: {ms:.3f} ms {n_w / ms / 1e6:.0f} GB/s write")
ms = t(lambda: a.zero_())
print(f"zero 1.26GB: {ms:.3f} ms {n_w / ms / 1e6:.0f} GB/s write")
ms = t(lambda: b.copy_(a))
print(f"copy 1.26GB: {ms:.3f} ms {2 * n_w / ms / 1e6:.0f} GB/s r+w")
ms = t(lambda: big.sum())
print(f"sum 5.03GB: {ms:.3f} ms {n_r / ms / 1e6:.0f} GB/s read")
a32 = a.view(torch.int32)
ms = t(lambda: a32.fill_(3))
print(f"fill int32 1.26GB: {ms:.3f} ms {n_w / ms / 1e6:.0f} GB/s write")
