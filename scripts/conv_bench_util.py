"""HIP-event timing of a launch plan replayed back to back (shared by the micro-benchmarks)."""
import torch


def bench(plan, reps=20):
    plan.run()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(5e7))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        plan.run()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
