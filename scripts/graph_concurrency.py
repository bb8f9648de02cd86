"""Do independent branches of a captured hipGraph run concurrently on this ROCm?  (probe)

Chains of small elementwise kernels: all on one stream vs split over 2 / 4 forked streams.
"""
import torch

torch.cuda.init()
dev = torch.device("cuda")
N = 24
bufs = [torch.randn(2 * 1024 * 1024 // 4, device=dev) for _ in range(8)]


def chain(x, n):
    for _ in range(n):
        x.mul_(1.0001).add_(0.5)


def capture(nstreams):
    g = torch.cuda.CUDAGraph()
    main = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(nstreams)]
    # warm up outside capture
    chain(bufs[0], 1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        for s in side:
            s.wait_stream(cur)
        for i, s in enumerate(side):
            with torch.cuda.stream(s):
                chain(bufs[i], N // nstreams)
        for s in side:
            cur.wait_stream(s)
    return g


def timeit(g, reps=50):
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for ns in (1, 2, 4, 8):
    print(f"{ns} branch(es), {2 * N} kernels total: {timeit(capture(ns)):8.1f} us / replay", flush=True)
