#!/usr/bin/env python3
"""all_to_all_single on a one-rank RCCL group: which sizes / dtypes copy
correctly (the exchange path moves up to 2 GB per relation)."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29534")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for rows in (32_000_000, 64_000_000, 100_000_000, 128_000_000):
    for dt, cols in ((torch.int64, 2), (torch.int32, 4), (torch.uint8, 16)):
        src = torch.randint(0, 1 << 30, (rows, cols), dtype=torch.int32, device="cuda").to(dt)
        dst = torch.empty_like(src)
        dist.all_to_all_single(dst, src, [rows], [rows])
        torch.cuda.synchronize()
        print(rows, dt, "bytes", src.numel() * src.element_size(), "ok", torch.equal(dst, src),
              flush=True)
        del src, dst
        torch.cuda.empty_cache()
dist.destroy_process_group()
