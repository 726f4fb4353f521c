"""Repeat a 16M Zipf join and locate the first output error."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402
w = int(os.environ.get("W", "16"))
lib = smj.Library(w)
n = 16_000_000
R, S = lib.empty(n), lib.empty(n)
lib.dev_gen_pk(R, 0, n, 12345)
lib.dev_gen_zipf(S, 0, n, 0.75, 54321)
ref = torch.sort(S[:, 1].to(torch.int64)).values
refR = torch.sort(R[:, 1].to(torch.int64)).values
sR, sS = lib.empty(n), lib.empty(n)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
for it in range(6):
    lib.dev_join(R, S, sR, sS, cnt, 10, 1, n)
    torch.cuda.synchronize()
    k = sS[:, 1].to(torch.int64)
    bad = (k != ref).nonzero()
    badR = (sR[:, 1].to(torch.int64) != refR).nonzero()
    print(f"it {it} count {int(cnt.item())} badS {bad.numel()} badR {badR.numel()}", flush=True)
    if bad.numel():
        i0, i1 = int(bad[0]), int(bad[-1])
        print(f"   S bad range [{i0}, {i1}] got {k[i0:i0+4].tolist()} want {ref[i0:i0+4].tolist()}", flush=True)
    if badR.numel():
        i0, i1 = int(badR[0]), int(badR[-1])
        print(f"   R bad range [{i0}, {i1}]", flush=True)
