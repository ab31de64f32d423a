#!/usr/bin/env python3
"""Device copy ceilings: the library's k_copy_calib, torch copy_, and
hipMemcpyAsync D2D (torch), 1 GiB, event-timed medians."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench
dev = torch.device("cuda:0")
print("calib_kernel_GBps", round(bench.device_copy_gbs(torch, dev), 1))
a = torch.empty(1 << 30, dtype=torch.uint8, device=dev); b = torch.empty_like(a); a.fill_(1)
ts = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); b.copy_(a); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) * 1e-3)
print("torch_copy_GBps", round(2 * (1 << 30) / np.median(ts) / 1e9, 1))
