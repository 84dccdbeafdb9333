#!/usr/bin/env python3
"""Streaming HBM ceilings on this box, for the roofline placement of the
write-heavy builds: fill (write only), copy (read + write) and a sum reduction
(read only) over 8 GiB tensors, timed with HIP events.  One JSON line."""
import json

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    n = 8 << 30
    x = torch.empty(n // 4, dtype=torch.int32, device="cuda")
    y = torch.empty_like(x)
    t_fill = timed(lambda: x.fill_(7))
    t_copy = timed(lambda: y.copy_(x))
    t_sum = timed(lambda: x.sum(dtype=torch.int64))
    print(json.dumps({"bytes": n, "write_GBps": n / t_fill / 1e9, "copy_GBps_rw": 2 * n / t_copy / 1e9,
                      "read_GBps": n / t_sum / 1e9, "device": torch.cuda.get_device_name()}))


if __name__ == "__main__":
    main()
