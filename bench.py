#!/usr/bin/env python3
"""bench.py -- m-way sort-merge join throughput on MI355X.

Metric (BASELINE.json): join throughput in Mtuples/s of R+S input
(128M x 128M, 16-byte tuples = the reference's 8B-key/8B-payload KEY_8B
build) per GPU, weak-scaled over N GPUs (each rank owns a 128M slice of R and
of S; the slices of all ranks form one relation of N*128M tuples).

One step = one full sortmergejoin_multiway over the device-resident synthetic
relations: radix partition, sort, merge-join count (N>1: range partition, an
RCCL all-to-all over xGMI, then the local join and an all-reduce of the
count).  Inputs are generated in HBM before the timed region.

Prints ONE JSON line (rank 0).  See DESIGN.md §7 for the fields.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (owns the HIP runtime before the library loads)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--n", type=int, default=128_000_000,
                   help="tuples per relation per GPU")
    p.add_argument("--width", type=int, default=16, choices=(8, 16))
    p.add_argument("--dist", default="uniform", choices=("uniform", "zipf"))
    p.add_argument("--theta", type=float, default=0.75)
    p.add_argument("--fanout-bits", type=int, default=9)
    p.add_argument("--cpu-n", type=int, default=64_000_000,
                   help="tuples per relation of the bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--check", action="store_true",
                   help="also verify sortedness/multiset of the sorted outputs")
    p.add_argument("--exchange-path", action="store_true",
                   help="run the multi-GPU code path (range partition, all-to-all, "
                        "segmented local join) even at N=1 (a one-rank RCCL group)")
    return p.parse_args()


# --------------------------------------------------------------------------
def alg_bytes_per_launch(name, n_rel, nR, nS, w):
    """Algorithmic HBM bytes of one launch: a materialising
    pass reads and writes every tuple once (2w), a histogram reads once (w)."""
    return {
        "k_hist": n_rel * w,                 # one relation per launch
        "k_scatter": 2 * n_rel * w,          # one relation per launch
        "k_tilepass": 2 * (nR + nS) * w,     # R and S in one launch
        "k_groupsort": 2 * (nR + nS) * w,    # R and S in one launch
    }.get(name)


def cpu_baseline(width, n):
    """Reference m-way join on the host cores (oracle/_ref/cpu_baseline*)."""
    exe = os.path.join(ROOT, "oracle", "_ref", f"cpu_baseline{width}")
    threads = 1
    cores = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores
    cores = min(cores, cap)
    while threads * 2 <= cores and threads * 2 <= 1024:
        threads *= 2
    if os.path.exists(exe):
        try:
            r = subprocess.run([exe, str(n), str(n), str(threads), "128"],
                               capture_output=True, text=True, timeout=600,
                               cwd="/tmp")
            m = re.search(r"SMJ_CPU_BASELINE (\{.*\})", r.stdout)
            if m:
                d = json.loads(m.group(1))
                t = d["seconds"]
                m2 = re.search(r"TOTAL-TIME-USECS = ([0-9.]+)", r.stderr)
                if m2:  # the reference's own timer (joincommon.c:214-227)
                    t = float(m2.group(1)) * 1e-6
                ok = d["count"] == n
                return {"value": round(2 * n / t / 1e6, 3), "unit": "Mtuples/s",
                        "cores": threads, "kind": "reference",
                        "sample": f"sortmergejoin_multiway {n}x{n} {width}B tuples, "
                                  f"{threads} threads, PK/FK uniform, "
                                  f"{'scalar' if width == 16 else 'AVX'} path, "
                                  f"count {'ok' if ok else 'MISMATCH'}"}
        except Exception as e:  # pragma: no cover
            print(f"[bench] reference CPU baseline failed: {e}", file=sys.stderr)
    # fall back to the single-threaded C restatement
    import numpy as np
    import oracle
    try:
        orc = oracle.Oracle(width)
    except FileNotFoundError:
        oracle.build()
        orc = oracle.Oracle(width)
    m = min(n, 8_000_000)
    orc.seed(12345)
    R = orc.create_relation_mway(m, m)
    orc.seed(54321)
    S = orc.create_relation_mway(m, m)
    t0 = time.time()
    c, _, _ = orc.sortmergejoin(R, S)
    t = time.time() - t0
    return {"value": round(2 * m / t / 1e6, 3), "unit": "Mtuples/s", "cores": 1,
            "kind": "port", "sample": f"oracle restatement {m}x{m} {width}B tuples, "
                                      f"count {'ok' if c == m else 'MISMATCH'}"}


def load_traffic(kernel, cfg_key):
    """HBM bytes per launch of `kernel` (FETCH_SIZE*2 + WRITE_SIZE, separate
    rocprofv3 --pmc passes of this same bench command; tools/make_traffic.py
    wrote profiles/pmc_traffic.json).  None when not profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(cfg_key, {}).get(kernel)
        return int(e["bytes"]) if e else None
    except Exception:
        return None


# --------------------------------------------------------------------------
def main():
    a = parse()
    # stdout carries exactly the one JSON line: native libraries (RCCL prints
    # a version banner at communicator setup) write to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    N = max(world, 1)
    if a.gpus != N and world > 1:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dist = None
    exchange = N > 1 or a.exchange_path
    if exchange:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import smj
    lib = smj.load(a.width)
    w = a.width
    n = a.n
    total = n * N
    first = n * rank
    R = lib.empty(n)
    S = lib.empty(n)
    lib.dev_gen_pk(R, first, total, 12345)
    if a.dist == "uniform":
        lib.dev_gen_fk(S, first, total, total, 54321)
    else:
        lib.dev_gen_zipf(S, first, total, a.theta, 54321)
    torch.cuda.synchronize()

    count = torch.zeros(1, dtype=torch.int64, device="cuda")
    if not exchange:
        sR, sS = lib.empty(n), lib.empty(n)

        def step():
            lib.dev_join(R, S, sR, sS, count, a.fanout_bits, 1, total)
    else:
        from smj.dist import DeviceOps, DistributedJoin
        dj = DistributedJoin(DeviceOps(lib), a.fanout_bits, 1, total)

        def step():
            dj.step(R, S, count)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    if exchange:
        dj.stats_reset()
    lib.trace(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = lib.trace_read()
    lib.trace(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    xchg = None
    if exchange:
        st = dj.stats_read()
        k = max(st["steps"], 1)
        # xGMI bytes per GPU per step and S's row all-to-all rate (SURVEY.md
        # §8(d): against 7 links x 153 GB/s, not HBM)
        xchg = {"xgmi_bytes_sent_per_gpu": st["sent_B"] // k,
                "xgmi_bytes_recv_per_gpu": st["recv_B"] // k,
                "packed_words": bool(dj.last_packed),
                "exchange_S_ms": round(st["xS_ms"] / k, 3),
                "exchange_S_GBps": round(st["sent_B"] / 2 / k / (st["xS_ms"] / k * 1e-3) / 1e9, 1)
                if st["xS_ms"] > 0 and st["sent_B"] > 0 else None,
                "xgmi_peak_GBps": 7 * 153}
    got = int(count.item())
    expect = total  # every S key exists once in R (PK/FK and Zipf over 1..|R|)
    ok = got == expect
    ms_step = elapsed / a.steps * 1e3
    value = 2 * total / (elapsed / a.steps) / 1e6

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    # dominant kernel roofline (this rank's trace over the timed region)
    best = None
    for name, (ms, launches) in kern.items():
        nrel = n if N == 1 else None
        b = alg_bytes_per_launch(name, n, n, n, w)
        if b is None:
            continue
        if best is None or ms > best[1]:
            best = (name, ms, launches, b)
    roof = None
    if best:
        name, ms, launches, b = best
        avg_s = ms / launches / 1e3
        ach = b / avg_s / 1e9
        cfg_key = f"n{n}_w{w}_{a.dist}"
        tr = load_traffic(name, cfg_key)
        roof = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": tr, "alg_bytes_per_launch": b,
                "avg_launch_ms": round(ms / launches, 4)}
    pipeline_gbs = 5 * 2 * total * w / (elapsed / a.steps) / 1e9

    cpu = None
    if N == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(w, a.cpu_n)

    out = {
        "metric": "join throughput Mtuples/s (R⋈S) + achieved HBM GB/s, 128M⋈128M at 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "Mtuples/s",
        "n_gpus": N,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64" if w == 16 else "int32",
        "data": "synthetic",
        "config": {"workload": f"sortmergejoin_multiway R={n} S={n} per GPU, "
                               f"{w}-byte tuples, {a.dist}"
                               + (f" theta={a.theta}" if a.dist == "zipf" else "")
                               + ", PK/FK keys 1..|R|",
                   "tuples_per_relation_per_gpu": n, "tuple_bytes": w,
                   "distribution": a.dist, "parallelism": f"range-partition x{N}"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "result_ok": ok,
        "matches": got,
        "detail": {
            "S_tuples_per_s_M": round(total / (elapsed / a.steps) / 1e6, 2),
            "pipeline_alg_GBps_5w": round(pipeline_gbs, 1),
            "pipeline_frac": round(pipeline_gbs / HBM_PEAK_GBS, 4),
            "kernels_ms_per_step": {k: round(v[0] / a.steps, 4) for k, v in kern.items()},
            "device": lib.lib.smj_device_name().decode(),
            "exchange": xchg,
        },
    }
    print(json.dumps(out), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
