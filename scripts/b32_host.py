"""B=32 step: host issue time vs GPU time (is the small-batch step host-bound?).

Prints, per step: host time to issue the step's calls (no synchronisation), wall time with a
final synchronize, and the hipGraph replay time.  usage: python scripts/b32_host.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-ba3c_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    tr, batch = bench.build_trainer(32, 128, 4, 4, 1, 0)
    for _ in range(20):
        tr.train_step(*batch)
    torch.cuda.synchronize()
    for n in (50, 100):
        t0 = time.perf_counter()
        for _ in range(n):
            tr.train_step(*batch)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("eager n=%d: host issue %.1f us/step, wall %.1f us/step" % (n, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6))
    # engine calls only (no Python trainer / model layers)
    eng = tr.engine
    st, ac, R = batch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        eng.train_grads(st, ac, R)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("train_grads only: host issue %.1f us/call, wall %.1f us/call" % ((t1 - t0) / 100 * 1e6, (t2 - t0) / 100 * 1e6))
    replay = tr.capture_step(*batch)
    for _ in range(20):
        replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("graph: host issue %.1f us/step, wall %.1f us/step" % ((t1 - t0) / 200 * 1e6, (t2 - t0) / 200 * 1e6))


if __name__ == "__main__":
    main()
