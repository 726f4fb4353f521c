#!/usr/bin/env python3
"""Where does all_to_all_single start to corrupt on a one-rank RCCL group?

For three element types the message size is stepped in BYTES; if the first
corrupt size is the same number of bytes for every dtype the limit is a byte
count (e.g. a 32-bit byte offset somewhere), if it is the same number of
ELEMENTS it is an element count.  A plain device copy of the same tensors is
the control.  Prints one line per probe.  (DESIGN.md §8 records the result.)"""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29535")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
MB = 1 << 20
sizes = [int(x) for x in sys.argv[1:]] or [1024, 1100, 1200, 1300, 1400, 1500, 1536, 2048, 3000]
for dt in (torch.uint8, torch.int32, torch.int64):
    esz = torch.tensor([], dtype=dt).element_size()
    for mb in sizes:
        n = mb * MB // esz
        src = torch.randint(0, 100, (n,), dtype=torch.int32, device="cuda").to(dt)
        dst = torch.zeros_like(src)
        dist.all_to_all_single(dst, src, [n], [n])
        torch.cuda.synchronize()
        ok = torch.equal(dst, src)
        first_bad = -1
        if not ok:
            first_bad = int((dst != src).to(torch.uint8).argmax().item()) * esz
        ctl = torch.zeros_like(src)
        ctl.copy_(src)
        print(f"dtype {str(dt):12s} MiB {mb:5d} elems {n:11d} bytes {n * esz:11d} "
              f"a2a_ok {ok} first_bad_byte {first_bad} copy_ok {torch.equal(ctl, src)}",
              flush=True)
        del src, dst, ctl
        torch.cuda.empty_cache()
dist.destroy_process_group()
