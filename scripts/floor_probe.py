"""What does moving N MB cost on this GPU at the layer sizes of DBL-n bs32?  torch copy_ (read N + write N)
timed with HIP events over back-to-back launches: the floor a per-layer kernel of that traffic can reach."""
import torch

for mb in (0.5, 3.3, 6.5, 13, 26, 52, 105, 210):
    n = int(mb * 1e6 / 2)
    x = torch.randn(n, device="cuda").half()
    y = torch.empty_like(x)
    for _ in range(5):
        y.copy_(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    a.record()
    for _ in range(reps):
        y.copy_(x)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(f"copy {mb:6.1f} MB -> {mb:6.1f} MB: {us:7.2f} us  {2 * mb / us:6.2f} TB/s", flush=True)
