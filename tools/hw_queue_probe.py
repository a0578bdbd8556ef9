#!/usr/bin/env python3
"""Whether GPU_MAX_HW_QUEUES set AFTER torch.cuda.device_count() (and before the first HIP
call, as bench.py does for N > 1) takes effect: 8 streams each run one single-thread spin
kernel (torch.cuda._sleep) at once.  Streams beyond the process's hardware queues share one,
and a queue runs its kernels one after another, so with 4 queues the 8 spins take ~2x one
spin, with >= 8 queues ~1x.

    python tools/hw_queue_probe.py QUEUES    (prints one JSON line)
"""
import json
import os
import sys
import time

import torch

q = sys.argv[1] if len(sys.argv) > 1 else "16"
ndev = torch.cuda.device_count()
os.environ["GPU_MAX_HW_QUEUES"] = q
torch.cuda.set_device(0)
streams = [torch.cuda.Stream() for _ in range(8)]
cycles = int(5e7)


def spin(ss):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


spin(streams)   # warm-up
one = min(spin(streams[:1]) for _ in range(3))
eight = min(spin(streams) for _ in range(3))
print(json.dumps({"devices": ndev, "GPU_MAX_HW_QUEUES": q, "one_spin_ms": round(one * 1e3, 2),
                  "eight_streams_ms": round(eight * 1e3, 2), "ratio": round(eight / one, 2)}),
      flush=True)
