#!/usr/bin/env python3
"""Device-to-host copy rate on the box, alone (analysis aid): 8.3 MB frames
(1920x1080 RGBA8) into pinned host memory, one or two streams, no traces
running.  Tells whether the async pipeline's readback (profiles/r02/async)
is bound by the link."""
import json
import time

import torch


def main():
    n = 1920 * 1080 * 4
    dev = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    hosts = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    for streams in (1, 2):
        ss = [torch.cuda.Stream() for _ in range(streams)]
        half = n // streams
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(400):
                for j, s in enumerate(ss):
                    with torch.cuda.stream(s):
                        hosts[k % 4][j * half:(j + 1) * half].copy_(dev[j * half:(j + 1) * half], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"streams": streams, "frames": 400, "ms_per_frame": round(dt / 400 * 1e3, 4),
                              "GBps": round(400 * n / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
