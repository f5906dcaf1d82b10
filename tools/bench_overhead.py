#!/usr/bin/env python3
"""Host overhead of bench.py's timed region at the driver's launch size (development tool,
GPU): wall time of one K-move launch bracketed by synchronize, with the Python wrapper vs
the prebuilt launcher, with and without the HIP event pair, against the kernel time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-general-ori_amd"))
import torch  # noqa: E402


def main():
    from splendor.env import RolloutBatch, SplendorEngine
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    e = SplendorEngine(2, device="cuda:0")
    rb = RolloutBatch(e, 32768, seed=0x5EED)
    out = rb.run(K)
    rb.run(K, out=out)
    launch = rb.launcher(K, out)
    torch.cuda.synchronize()

    def region(fn, events):
        best = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if events:
                e0.record()
            fn()
            if events:
                e1.record()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best.append((dt * 1e6, e0.elapsed_time(e1) * 1e3 if events else 0.0))
        best.sort()
        return best[len(best) // 2]
    print("empty sync", region(lambda: None, False))
    print("empty sync+events", region(lambda: None, True))
    print("wrapper", region(lambda: rb.run(K, out=out), True))
    print("launcher", region(launch, True))
    print("launcher no events", region(launch, False))


if __name__ == "__main__":
    main()
