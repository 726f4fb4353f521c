"""Zipf join count at several sizes, sampled vs exact level-1 partition."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:
    for s in ("0", "1"):
        env = dict(os.environ, SMJ_SAMPLED=s)
        subprocess.run([sys.executable, __file__, "run"], env=env, check=True)
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402
for w in (8, 16):
    lib = smj.Library(w)
    for n in (1_000_000, 16_000_000, 128_000_000):
        for bits in (9, 10):
            R, S = lib.empty(n), lib.empty(n)
            lib.dev_gen_pk(R, 0, n, 12345)
            lib.dev_gen_zipf(S, 0, n, 0.75, 54321)
            sR, sS = lib.empty(n), lib.empty(n)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            lib.dev_join(R, S, sR, sS, cnt, bits, 1, n)
            torch.cuda.synchronize()
            k = sS[:, 1].to(torch.int64)
            srt = bool((k[1:] >= k[:-1]).all())
            print(f"sampled={os.environ.get('SMJ_SAMPLED')} w{w} n={n} bits={bits} count={int(cnt.item())} ok={int(cnt.item()) == n} S_sorted={srt} S_keysum={int(k.sum())} in_keysum={int(S[:,1].to(torch.int64).sum())}", flush=True)
            del R, S, sR, sS
            torch.cuda.empty_cache()
