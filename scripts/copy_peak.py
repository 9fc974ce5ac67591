"""Practical HBM rates on one MI355X: torch copy (read + write), fill (write only) and sum (read
only) over 2 GiB fp32 tensors, best of 10 (HIP events)."""
import torch

n = 1 << 29
x = torch.empty(n, device="cuda")
y = torch.empty(n, device="cuda")
x.uniform_()
torch.cuda.synchronize()


def best(fn, nbytes):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(10):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    t = min(ts)
    return nbytes / (t * 1e-3) / 1e12, t


for name, fn, nb in (("copy", lambda: y.copy_(x), 8 * n), ("fill", lambda: y.fill_(1.0), 4 * n),
                     ("sum", lambda: x.sum(), 4 * n)):
    bw, t = best(fn, nb)
    print(f"{name:5s} {t:.3f} ms  {bw:.2f} TB/s")
