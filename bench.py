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


def set_payloads(R, S, kind, first):
    """--payload: rewrite the payload column of both relations in HBM (before
    the timed region).  wide48: 2^40 + global row id -- more than the 48 - s1
    bits a 48-bit word keeps at the headline plan, within the 64 - s1 of a
    packed 64-bit word; full64: a 64-bit avalanche hash of the global row id,
    negative for half the rows -- no packed word holds them: the join moves
    12-byte elements (payload + 32-bit key offset, LayP96)."""
    if kind == "rowid" or R.dtype != torch.int64:
        return
    for t, salt in ((R, 0), (S, 1 << 62)):
        i = torch.arange(first, first + t.shape[0], dtype=torch.int64, device=t.device)
        if kind == "wide48":
            t[:, 0] = i + (1 << 40)
        else:
            z = (i + salt) * -7046029254386353131  # 0x9E3779B97F4A7C15
            z = (z ^ (z >> 31)) * 0x1B873593CA5A7E35
            t[:, 0] = z ^ (z >> 29)


def shares(a, N):
    """(tuples per relation on each rank, first global row of each, total):
    weak scaling gives every rank --n; --n-total splits a fixed total."""
    if a.n_total is not None:
        total = a.n_total
        base = total // N
        ns = [base] * (N - 1) + [total - base * (N - 1)]
    else:
        total = a.n * N
        ns = [a.n] * N
    return ns, [sum(ns[:g]) for g in range(N)], total


def make_relations(lib, a, n, first, total, device="cuda"):
    """This rank's slices of R (PK: keys first+1.. of a permutation of
    1..total) and S (FK uniform, or Zipf) generated in HBM on `device`."""
    R = lib.empty(n, device=device)
    S = lib.empty(n, device=device)
    lib.dev_gen_pk(R, first, total, 12345)
    if a.zipf_gen == "auto":
        a.zipf_gen = "reference" if total <= (1 << 28) else "fast"
    if a.dist == "uniform":
        lib.dev_gen_fk(S, first, total, total, 54321)
    elif a.zipf_gen == "reference":
        lib.dev_gen_zipf_ref(S, first, total, a.theta, 54321)
    else:
        lib.dev_gen_zipf(S, first, total, a.theta, 54321)
    set_payloads(R, S, a.payload, first)
    torch.cuda.synchronize()
    return R, S


def _close(dist):
    """Destroy the process group (and the join's cached row communicators)."""
    mod = sys.modules.get("smj.dist")
    if mod is not None:
        mod.release_row_groups()
    dist.destroy_process_group()


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--op", default="join",
                   choices=("join", "sort", "partition", "merge", "exchange"),
                   help="join: sortmergejoin_multiway (the headline); sort: bench_sort's "
                        "avxsort_tuples on 2^27 tuples; partition: bench_partitioning's "
                        "partition_relation_optimized on 2^27 tuples; merge: "
                        "bench_multiwaymerge's avx_multiway_merge, --fanin runs of --n; "
                        "exchange: the join's row all-to-all alone (numabench's memory "
                        "bandwidth study, tputbench.c:665-1171, as xGMI bandwidth)")
    p.add_argument("--n", type=int, default=None,
                   help="tuples per relation per GPU (join: 128M; sort/partition: 2^27)")
    p.add_argument("--n-total", type=int, default=None,
                   help="join: tuples per relation over ALL GPUs (strong scaling: each "
                        "GPU gets n_total / N)")
    p.add_argument("--width", type=int, default=None, choices=(8, 16),
                   help="tuple bytes (join: 16 = the reference's KEY_8B build; "
                        "sort/partition: 8 = the reference's default tuple)")
    p.add_argument("--bits", type=int, default=10, help="partition: radix bits")
    p.add_argument("--fanin", type=int, default=64, help="merge: number of sorted runs")
    p.add_argument("--shift", type=int, default=0, help="partition: shift bits")
    p.add_argument("--dist", default="uniform", choices=("uniform", "zipf"))
    p.add_argument("--theta", type=float, default=0.75)
    p.add_argument("--zipf-gen", default="auto", choices=("auto", "reference", "fast"),
                   help="zipf S: the reference's own create_relation_zipf after "
                        "srand(54321), bit-exact (refgen.hip), or the fast "
                        "rejection-inversion sampler.  The reference stream needs the "
                        "alphabet permutation and CDF table over 1..|R| built on the host "
                        "(a serial shuffle) and held on the device: 12 bytes per key, "
                        "~13 GB on every rank at N = 8 x 128M.  auto: the reference "
                        "stream up to 2^28 keys, the fast sampler above")
    p.add_argument("--payload", default="rowid", choices=("rowid", "wide48", "full64"),
                   help="join payloads: rowid = the generators' row ids (R: 5 + i; they "
                        "fit 48-bit words: the intermediates move 6 bytes an element); "
                        "wide48 = 2^40 + row id (64-bit packed words, 8 bytes); full64 = "
                        "random 64-bit values, negative ones included (12-byte "
                        "elements: the payload and a 32-bit key offset)")
    p.add_argument("--sim-world", type=int, default=8,
                   help="--op exchange on ONE GPU: time the exchange's device side as rank 0 "
                        "of a world of this many GPUs would run it (its slice of the weak-scaled "
                        "relation, the exact range partition into that world's partitions and "
                        "layout, the table kernels; nothing crosses xGMI on one GPU)")
    p.add_argument("--exchange-form", default="exact", choices=("exact", "sampled"),
                   help="--op exchange on one GPU: the range partition form timed (exact: what "
                        "ranks use across GPUs; sampled: the one-rank form, whose region slack "
                        "would travel with the rows)")
    p.add_argument("--fanout-bits", type=int, default=8,
                   help="level-1 partitions (2^bits) of the join; the library raises it "
                        "as the relation size needs")
    p.add_argument("--cpu-n", type=int, default=128_000_000,
                   help="tuples per relation of the bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-trace", action="store_true",
                   help="lab: no per-kernel HIP events in the timed loop (measures what "
                        "the trace costs; the line then has no roofline)")
    p.add_argument("--no-check", action="store_true",
                   help="skip the output check after the timed loop (default: the sorted "
                        "outputs are checked on the device for (key, payload) order and "
                        "against the inputs' order-independent checksum; result_ok "
                        "carries it)")
    p.add_argument("--exchange-path", action="store_true",
                   help="run the multi-GPU code path (range partition, all-to-all, "
                        "segmented local join) even at N=1 (a one-rank RCCL group)")
    p.add_argument("--impl", default="c", choices=("python", "c"),
                   help="multi-GPU join under a launcher (one process per GPU): the C entry "
                        "smj_mgpu_rank_join (mgpu_orch.hpp, its own RCCL communicators per "
                        "rank; the line carries every rank's phases) or the torch.distributed "
                        "orchestration (smj.dist)")
    p.add_argument("--launch", default="auto", choices=("auto", "threads", "spawn"),
                   help="--gpus N > 1 without a launcher (no WORLD_SIZE): threads = one "
                        "process, one host thread per GPU through smj_mgpu_join_slices (the "
                        "reference's T join threads, joincommon.c:118-165; the join only); "
                        "spawn = start N processes under torch.distributed.run (the driver's "
                        "form) and print rank 0's line; auto = threads for the join, spawn "
                        "for the other ops")
    p.add_argument("--api", action="store_true",
                   help="join: time the reference-named entry point sortmergejoin_multiway "
                        "(relation_t over device-resident tuples, no key-range hint: the "
                        "plan is derived from |R| as the reference does) instead of "
                        "smj_dev_join")
    return p.parse_args()


# --------------------------------------------------------------------------
def alg_bytes_per_launch(name, n_rel, nR, nS, w, op="join"):
    """Algorithmic HBM bytes of one launch: a materialising
    pass reads and writes every tuple once (2w), a histogram reads once (w).
    The join's tile and group passes take R and S in one launch; a sort's
    take its one relation.  SURVEY.md §8(d) credits the join 5w a tuple:
    the partition 2w (k_scatter), the sort 2w and the merge-join scan 1w.
    The sort is two passes here, so the tile pass (an intermediate level,
    in place) is credited 1w and the group pass, which writes the sorted
    relation and counts, 2w: the per-kernel credits add up to 5w."""
    both = (nR + nS) if op == "join" else n_rel
    return {
        "k_hist": n_rel * w,                 # one relation per launch
        "k_scatter": 2 * n_rel * w,          # one relation per launch
        "k_tilepass": both * w,
        "k_groupsort": 2 * both * w,
        "k_km_merge": 2 * n_rel * w,         # every tuple of the runs, once
    }.get(name)


def _ref_exe(name):
    """A reference binary built by oracle/build_ref.sh (shipped in-tree).  The
    CPU baseline is the reference itself: no silent fallback."""
    exe = os.path.join(ROOT, "oracle", "_ref", name)
    if not os.path.exists(exe):
        raise FileNotFoundError(
            f"{exe} missing: run oracle/build_ref.sh where /root/reference exists "
            "(or pass --no-cpu-baseline)")
    return exe


def host_cores():
    """(threads for the CPU baseline, facts about the host).

    BASELINE.md §3 asks for T = the largest power of two within the host's
    cores.  The cores this job may use are the process's affinity mask,
    further limited by a cgroup CPU quota and by OMP_NUM_THREADS, which the
    GPU pool sets to the job's CPU share (16 per GPU); lscpu reports the
    machine.  All of them go into the line."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:  # cgroup v2: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    share = min(x for x in (aff, quota, omp) if x)
    lscpu = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=30).stdout
        per = re.search(r"Core\(s\) per socket:\s+(\d+)", out)
        sock = re.search(r"Socket\(s\):\s+(\d+)", out)
        if per and sock:
            lscpu = int(per.group(1)) * int(sock.group(1))
    except Exception:  # pragma: no cover
        pass
    return share, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
                   "host_cores_lscpu": lscpu}


def _heartbeat(what):
    """A thread that prints a line to stderr every 30 s while a long CPU run
    goes on (a GPU job that writes nothing for minutes is taken as hung).
    Returns a stop() function."""
    import threading
    done = threading.Event()
    t0 = time.time()

    def beat():
        while not done.wait(30):
            print(f"[bench] {what}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()

    def stop():
        done.set()
        th.join()
    return stop


def _join_once(exe, n, threads, skew=0.0):
    stop = _heartbeat(f"CPU baseline {n}x{n}, {threads} thread(s)")
    try:
        r = subprocess.run([exe, str(n), str(n), str(threads), "128", str(skew)],
                           capture_output=True, text=True, timeout=900, cwd="/tmp")
    finally:
        stop()
    m = re.search(r"SMJ_CPU_BASELINE (\{.*\})", r.stdout)
    if not m:
        raise RuntimeError(f"{exe} printed no result (rc {r.returncode}): {r.stderr[-400:]}")
    d = json.loads(m.group(1))
    t = d["seconds"]
    m2 = re.search(r"TOTAL-TIME-USECS = ([0-9.]+)", r.stderr)
    if m2:  # the reference's own timer (joincommon.c:214-227)
        t = float(m2.group(1)) * 1e-6
    return t, d["count"] == n


def cpu_baseline(width, n, skew=0.0, t1=True):
    """The reference m-way join (oracle/_ref/cpu_baseline*: compiled from the
    reference's sources) on this host: T = the largest power of two within
    the job's CPU share (host_cores), and T = 1 on the same 128M x 128M
    (BASELINE.md §3).  16-byte tuples take the reference's scalar path,
    8-byte tuples its AVX path.  skew > 0: S is the reference driver's --skew
    input (create_relation_zipf, srand(54321)), the relation the GPU line
    joins with --dist zipf."""
    exe = _ref_exe(f"cpu_baseline{width}")
    share, facts = host_cores()
    threads = 1
    while threads * 2 <= share and threads * 2 <= 1024:
        threads *= 2
    t, ok = _join_once(exe, n, threads, skew)
    t1v, ok1 = None, True
    # T = 1 on the same relations; a Zipf S on a quarter of them: the
    # reference generates it single-threaded (create_relation_zipf) and
    # the one-thread join of 128M x 128M with it takes minutes
    n1 = n if skew <= 0 else max(n // 4, 1)
    if t1:
        ts, ok1 = _join_once(exe, n1, 1, skew)
        t1v = round(2 * n1 / ts / 1e6, 3)
    path = "scalar" if width == 16 else "AVX"
    return {"value": round(2 * n / t / 1e6, 3), "unit": "Mtuples/s",
            "cores": threads, "kind": "reference", **facts,
            "t1_value": t1v,
            "sample": f"sortmergejoin_multiway {n}x{n} {width}B tuples, {threads} threads "
                      f"(the job's CPU share: affinity {facts['affinity_cpus']}, cgroup quota "
                      f"{facts['cgroup_cpu_quota']}, OMP_NUM_THREADS {facts['omp_num_threads']}; "
                      f"t1_value: 1 thread on {n1}x{n1}"
                      f"{'' if n1 == n else ', a quarter: the Zipf S is generated on one thread'}), "
                      f"{f'PK / Zipf {skew} FK (create_relation_zipf)' if skew > 0 else 'PK/FK uniform'}, "
                      f"{path} path, "
                      f"count {'ok' if ok and ok1 else 'MISMATCH'}"}


def cpu_baseline_op(op, width, n, bits, shift, fanin=64):
    """The reference's single-core partition_relation_optimized / avxsort_tuples
    (oracle/_ref/cpu_baseline_ops*) on create_relation_pk(n), seed 12345."""
    exe = _ref_exe(f"cpu_baseline_ops{width}")
    args = [exe, op, str(n)] + ([str(bits), str(shift)] if op == "partition" else
                                [str(fanin)] if op == "merge" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=900, cwd="/tmp")
    m = re.search(r"SMJ_CPU_OPS (\{.*\})", r.stdout)
    if not m:
        raise RuntimeError(f"{exe} printed no result (rc {r.returncode}): {r.stderr[-400:]}")
    d = json.loads(m.group(1))
    _, facts = host_cores()
    what = {"partition": f"partition_relation_optimized {n} tuples, {bits} bits, shift {shift}",
            "sort": f"{'avxsort_tuples' if width == 8 else 'scalarsort_tuples'} {n} tuples",
            "merge": f"{'avx' if width == 8 else 'scalar'}_multiway_merge of {fanin} runs "
                     f"of {n} (generate_rand_ordered_tuples), 4 MiB FIFO"}[op]
    if op == "merge":
        n = n * fanin
    return {"value": round(n / d["seconds"] / 1e6, 3), "unit": "Mtuples/s", "cores": 1,
            "kind": "reference", **facts,
            "sample": f"{what}, {width}B tuples, create_relation_pk seed 12345, "
                      f"single core (as the reference bench), "
                      f"{'ok' if d['ok'] else 'FAILED'}"}


def _pmc(cfg_key):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(cfg_key, {})
    except Exception:
        return {}


def load_traffic(kernel, cfg_key):
    """HBM bytes per launch of `kernel` (FETCH_SIZE*2 + WRITE_SIZE, separate
    rocprofv3 --pmc passes of this same bench command; tools/make_traffic.py
    wrote profiles/pmc_traffic.json).  None when not profiled."""
    e = _pmc(cfg_key).get(kernel)
    return int(e["bytes"]) if e else None


def step_traffic(kernel, launches_per_step, cfg_key):
    """PMC bytes of one whole step: every library kernel of the profiled run
    (data generators excluded), its per-launch bytes times its launches, over
    the profiled run's step count (the dominant kernel's launches there over
    its launches per step).  None when the config was not profiled."""
    d = _pmc(cfg_key)
    if kernel not in d or not launches_per_step:
        return None
    steps = d[kernel]["launches"] / launches_per_step
    tot = sum(e["bytes"] * e["launches"] for k, e in d.items()
              if k.startswith("k_") and not k.startswith("k_gen"))
    return int(tot / steps)


def _checksum(t):
    """Order-independent checksum of (n, 2) rows (payload, key) as a wrapping
    int64 tensor: sums of the keys, the payloads and of two 64-bit avalanche
    hashes of each row (a lost row and a duplicated one cancel only if their
    hashes collide, ~2^-64).  Sums over disjoint parts add up (mod 2^64)."""
    k = t[:, 1].to(torch.int64)
    p = t[:, 0].to(torch.int64)
    z = (k * 0x2545F4914F6CDD1D) ^ (p + 0x632BE59BD9B4E019)
    z = (z ^ (z >> 31)) * 0x1B873593CA5A7E35
    z = (z ^ (z >> 29)) * 0x3C79AC492BA7B653
    z = z ^ (z >> 32)
    return torch.stack([k.sum(), p.sum(), z.sum(), (z * (z | 1)).sum()])


def _is_sorted(t, w):
    """Rows in the library's order: (key, payload) ascending; 8-byte tuples
    compare as the signed 64-bit word key << 32 | unsigned payload."""
    if t.shape[0] < 2:
        return True
    k = t[:, 1].to(torch.int64)
    p = t[:, 0].to(torch.int64)
    if w == 8:
        p = p & 0xFFFFFFFF
    ok = (k[1:] > k[:-1]) | ((k[1:] == k[:-1]) & (p[1:] >= p[:-1]))
    return bool(ok.all().item())


def output_check(pairs, w, dist=None):
    """[(input rows, sorted output rows), ...] -> dict: every output sorted and
    a permutation of its input (checksums; over a process group the sums of
    all ranks are compared, as each rank sorts its key range of everyone's
    rows)."""
    res = {"sorted": True, "checksum_equal": True}
    for src, out in pairs:
        res["sorted"] = res["sorted"] and _is_sorted(out, w)
        a, b = _checksum(src), _checksum(out)
        if dist is not None:
            dist.all_reduce(a)
            dist.all_reduce(b)
        res["checksum_equal"] = res["checksum_equal"] and bool(torch.equal(a, b))
    if dist is not None:
        f = torch.tensor([0 if res["sorted"] else 1], device="cuda")
        dist.all_reduce(f)
        res["sorted"] = int(f.item()) == 0
    return res


# --------------------------------------------------------------------------
def _json_stdout():
    """stdout carries exactly the one JSON line: native libraries (RCCL
    prints a version banner at communicator setup) write to stderr instead.
    Returns the file the line goes to."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def standalone(a):
    """--gpus N > 1 with no launcher (no WORLD_SIZE): N GPUs must be
    visible, else exit 2 (a line for fewer GPUs than asked would be
    mislabelled).  Then the join runs in this process with one host thread
    per GPU (--launch threads), or N processes start under
    torch.distributed.run (--launch spawn) and rank 0's line is relayed.
    Returns the exit code.  Nothing here touches the GPU before the spawn
    (device_count does not initialise it on this image)."""
    vis = torch.cuda.device_count()
    if vis < a.gpus:
        print(f"[bench] ERROR: --gpus {a.gpus} but {vis} GPU(s) visible; no line is printed "
              f"(run on a node with {a.gpus} GPUs, or under torch.distributed.run)",
              file=sys.stderr)
        return 2
    launch = a.launch if a.launch != "auto" else ("threads" if a.op == "join" else "spawn")
    if launch == "threads":
        if a.op != "join" or a.exchange_path or a.api:
            print("[bench] ERROR: --launch threads runs the join (smj_mgpu_join_slices) only",
                  file=sys.stderr)
            return 2
        run_threads_join(a, _json_stdout())
        return 0
    import socket
    with socket.socket() as sk:  # a free port for the rendezvous
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] spawning: {' '.join(cmd)}", file=sys.stderr, flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    sys.stdout.write(r.stdout)
    sys.stdout.flush()
    return r.returncode


def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and (a.gpus > 1 or a.launch == "threads"):
        sys.exit(standalone(a))
    world = int(world_env or "1")
    N = max(world, 1)
    if a.gpus != N:
        print(f"[bench] ERROR: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} "
              "rank(s); no line is printed", file=sys.stderr)
        sys.exit(2)
    json_out = _json_stdout()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    exchange = a.op == "join" and (N > 1 or a.exchange_path)
    if a.op not in ("join", "exchange") and N > 1:  # replicas: barrier and max
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if exchange:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    if a.op == "exchange":
        run_exchange(a, json_out, N, rank, local)
        return
    import smj
    if a.width is None:
        a.width = 16 if a.op == "join" else 8
    if a.n is None:
        a.n = {"join": 128_000_000, "merge": 65536}.get(a.op, 1 << 27)
    lib = smj.load(a.width)
    if a.op != "join":
        run_op(a, lib, json_out, dist, N, rank)
        return
    w = a.width
    ns_, firsts, total = shares(a, N)
    n, first = ns_[rank], firsts[rank]
    R, S = make_relations(lib, a, n, first, total)

    count = torch.zeros(1, dtype=torch.int64, device="cuda")
    tracer = lib
    if a.api and not exchange:
        # sortmergejoin_multiway(relation_t*, relation_t*, joinconfig_t*) on
        # hipMalloc'd tuples (used in place, no PCIe); the reference's default
        # configuration (src/main.c: PARTFANOUT 128), one thread
        import ctypes
        os.environ["SMJ_QUIET"] = "1"  # no per-call stats lines in the timed loop
        rR = smj.Relation(R.data_ptr(), n)
        rS = smj.Relation(S.data_ptr(), n)
        cfg = smj.JoinConfig(1, 128, int(w == 16), int(w == 16), 20 << 20, 2)
        libc = ctypes.CDLL(None)
        libc.free.argtypes = [ctypes.c_void_p]
        api_count = [0]

        def step():
            res = lib.lib.sortmergejoin_multiway(ctypes.byref(rR), ctypes.byref(rS),
                                                 ctypes.byref(cfg))
            api_count[0] = int(res.contents.totalresults)
            libc.free(res.contents.resultlist)
            libc.free(ctypes.cast(res, ctypes.c_void_p))

        tracer = _WsTracer(lib, lib.lib.smj_context_workspace())
    elif not exchange:
        sR, sS = lib.empty(n), lib.empty(n)

        def step():
            lib.dev_join(R, S, sR, sS, count, a.fanout_bits, 1, total)
    elif a.impl == "c":
        comm = lib.mgpu_comm(N, rank)
        mg_st = {"steps": 0, "sent_B": 0, "recv_B": 0, "layout": None,
                 "ph": dict.fromkeys(PHASES, 0.0)}

        def step():
            c, _, _, st = comm.join(R, S, key_range=(1, total))
            count.fill_(c)
            mg_st["steps"] += 1
            mg_st["sent_B"] += st["sent_bytes"]
            mg_st["recv_B"] += st["recv_bytes"]
            mg_st["layout"] = st["layout"]
            for p in PHASES:
                mg_st["ph"][p] += st[p]
        tracer = _WsTracer(lib, lib.lib.smj_mgpu_comm_workspace(comm.h))
    else:
        from smj.dist import DeviceOps, DistributedJoin
        # n_hint: the same on every rank (the largest share)
        dj = DistributedJoin(DeviceOps(lib), a.fanout_bits, 1, total,
                             n_hint=total - total // N * (N - 1))
        last = [None, None]

        def step():
            last[0], last[1] = dj.step(R, S, count)

    def reset():
        if exchange and a.impl == "c":
            mg_st.update(steps=0, sent_B=0, recv_B=0, ph=dict.fromkeys(PHASES, 0.0))
        elif exchange:
            dj.stats_reset()

    elapsed, kern, brk = timed_loop(a, tracer, dist, step, reset)
    # the intermediate layout the last step ran in (the 1-GPU join: p48 for
    # row-id payloads, words or tuples for wider ones)
    layout = None if exchange else lib.last_layout(api=a.api)
    if a.api and not exchange:
        count.fill_(api_count[0])

    xchg = None
    if exchange and a.impl == "c":
        k = max(mg_st["steps"], 1)
        # every rank's phases and bytes, averaged over the timed steps
        mine = torch.tensor([mg_st["ph"][p] / k for p in PHASES]
                            + [mg_st["sent_B"] / k, mg_st["recv_B"] / k],
                            dtype=torch.float64, device="cuda")
        rows = [mine]
        if N > 1:
            rows = [torch.empty_like(mine) for _ in range(N)]
            dist.all_gather(rows, mine)
        xchg = {"impl": "c (smj_mgpu_rank_join, one process per GPU)",
                **rank_phases([r.tolist() for r in rows]),
                "exchange_layout": mg_st["layout"], "xgmi_peak_GBps": 7 * 153}
    elif exchange:
        st = dj.stats_read()
        k = max(st["steps"], 1)
        # xGMI bytes per GPU per step and S's row all-to-all rate (SURVEY.md
        # §8(d): against 7 links x 153 GB/s, not HBM)
        xchg = {"xgmi_bytes_sent_per_gpu": st["sent_B"] // k,
                "xgmi_bytes_recv_per_gpu": st["recv_B"] // k,
                # region slack of the sampled exchange partition received
                # with the rows (own rows included)
                "slack_bytes_recv_per_gpu": st.get("gap_B", 0) // k,
                "packed_words": bool(dj.last_packed),
                "exchange_layout": dj.last_layout,
                "exchange_S_ms": round(st["xS_ms"] / k, 3),
                "exchange_S_GBps": round(st["sent_B"] / 2 / k / (st["xS_ms"] / k * 1e-3) / 1e9, 1)
                if st["xS_ms"] > 0 and st["sent_B"] > 0 else None,
                "xgmi_peak_GBps": 7 * 153}
    got = int(count.item())
    expect = total  # every S key exists once in R (PK/FK and Zipf over 1..|R|)
    ok = got == expect
    # the last timed step's sorted relations, checked on the device (order and
    # checksums against the inputs); the reference-named entry point keeps its
    # sorted relations internal, so --api checks the count only
    chk = None
    if not a.no_check and not (a.api and not exchange):
        if exchange and a.impl == "c":
            last = list(comm.sorted())
        outs = (sR, sS) if not exchange else tuple(last)
        chk = output_check([(R, outs[0]), (S, outs[1])], w, dist if exchange and N > 1 else None)
        ok = ok and chk["sorted"] and chk["checksum_equal"]
    ms_step = elapsed / a.steps * 1e3
    value = 2 * total / (elapsed / a.steps) / 1e6

    if exchange and a.impl == "c":
        comm.close()
    if rank != 0:
        if dist:
            _close(dist)
        return

    cfg_key = f"n{n}_w{w}_{a.dist}" + ("" if a.payload == "rowid" else f"_{a.payload}")
    roof = dominant_roofline(kern, lambda name: alg_bytes_per_launch(name, n, n, n, w), cfg_key)
    pipeline_gbs = 5 * 2 * total * w / (elapsed / a.steps) / 1e9

    cpu = None
    if N == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(w, a.cpu_n, a.theta if a.dist == "zipf" else 0.0)

    strong = a.n_total is not None
    out = {
        "metric": "join throughput Mtuples/s (R⋈S) + achieved HBM GB/s, 128M⋈128M at 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "Mtuples/s",
        "n_gpus": N,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "int64" if w == 16 else "int32",
        "data": "synthetic",
        "config": {"workload": (f"sortmergejoin_multiway R={total} S={total} over {N} GPU(s)"
                                if strong else
                                f"sortmergejoin_multiway R={n} S={n} per GPU")
                               + f", {w}-byte tuples, {a.dist}"
                               + (" (reference entry point sortmergejoin_multiway, "
                                  "no key-range hint)" if a.api else "")
                               + (f" theta={a.theta} ({'create_relation_zipf, srand(54321)' if a.zipf_gen == 'reference' else 'rejection-inversion sampler'})"
                                  if a.dist == "zipf" else "")
                               + ", PK/FK keys 1..|R|"
                               + {"rowid": ", row-id payloads (48-bit intermediates)",
                                  "wide48": ", payloads 2^40 + row id (64-bit packed "
                                            "intermediates)",
                                  "full64": ", random 64-bit payloads (12-byte "
                                            "intermediates)"}[a.payload if w == 16 else "rowid"],
                   "tuples_per_relation_per_gpu": n, "tuples_per_relation_total": total,
                   "tuple_bytes": w, "payload": a.payload if w == 16 else "rowid",
                   "distribution": a.dist, "parallelism": f"range-partition x{N}"
                   + (" (C orchestration)" if exchange and a.impl == "c" else "")},
        "roofline": roof,
        "cpu_baseline": cpu,
        "result_ok": ok,
        "matches": got,
        "output_check": chk if chk is not None else
        ("count only (--api: the entry point keeps its sorted relations internal)"
         if a.api else "skipped (--no-check)"),
        "detail": {
            "S_tuples_per_s_M": round(total / (elapsed / a.steps) / 1e6, 2),
            "pipeline_alg_GBps_5w": round(pipeline_gbs, 1),
            "pipeline_frac": round(pipeline_gbs / HBM_PEAK_GBS, 4),
            **step_phys(roof, brk, ms_step, cfg_key),
            # untimed steps, every kernel traced (timed_loop)
            "kernels_ms_per_step": {k: round(v[0], 4) for k, v in brk.items()},
            "device": lib.lib.smj_device_name().decode(),
            "intermediate_layout": layout,
            "exchange": xchg,
        },
    }
    print(json.dumps(out), file=json_out, flush=True)
    if dist:
        _close(dist)


PHASES = ("partition_ms", "tables_ms", "wait_ms", "join_ms", "reduce_ms", "busy_ms", "rows_ms")


def rank_phases(rows):
    """rows[g] = rank g's PHASES + (bytes sent, bytes received) per step ->
    the line's multi-GPU detail: every rank's device phases (smj_mgpu_stats:
    the five before busy_ms are consecutive on the rank's main stream and add
    up to it; rows_ms, the row exchange on its own stream, overlaps them), the
    slowest rank's, and the xGMI bytes per GPU (the most any rank sent)."""
    per = [{p: round(v, 4) for p, v in zip(PHASES, r)} for r in rows]
    slow = max(range(len(rows)), key=lambda g: rows[g][PHASES.index("busy_ms")])
    return {"phases_ms_per_rank": per, "slowest_rank": slow,
            "xgmi_bytes_sent_per_gpu": int(max(r[len(PHASES)] for r in rows)),
            "xgmi_bytes_recv_per_gpu": int(max(r[len(PHASES) + 1] for r in rows))}


def run_threads_join(a, json_out):
    """--gpus N > 1 without a launcher: the multi-GPU join in THIS process,
    one host thread per GPU (smj_mgpu_join_slices: the in-process group of
    sortmergejoin_mpsm, ncclCommInitAll over the N GPUs, the reference's T join
    threads of joincommon.c:118-165).  Rank g's slices of R and S are
    generated on GPU g before the timed region and read in place.  One step =
    one call (it returns when every rank's count is in); value = all tuples
    / the call's host time, which is the slowest rank's by construction."""
    import smj
    N = a.gpus
    w = a.width or 16
    a.width = w
    if a.n is None:
        a.n = 128_000_000
    ns_, firsts, total = shares(a, N)
    libs, Rs, Ss = [], [], []
    for g in range(N):
        dev = torch.device("cuda", g)
        with torch.cuda.device(dev):
            L = smj.Library(w)  # a workspace of its own on this GPU
            R, S = make_relations(L, a, ns_[g], firsts[g], total, device=dev)
        libs.append(L)
        Rs.append(R)
        Ss.append(S)
    lib = libs[0]
    acc = {"steps": 0, "rows": [[0.0] * (len(PHASES) + 2) for _ in range(N)], "layout": None}
    last = {"count": None}

    def step():
        c, _, sts = lib.mgpu_join_slices(Rs, Ss, 0, key_range=(1, total))
        last["count"] = c
        acc["steps"] += 1
        acc["layout"] = sts[0]["layout"]
        for g, st in enumerate(sts):
            vals = [st[p] for p in PHASES] + [st["sent_bytes"], st["recv_bytes"]]
            acc["rows"][g] = [x + y for x, y in zip(acc["rows"][g], vals)]

    def reset():
        acc["steps"] = 0
        acc["rows"] = [[0.0] * (len(PHASES) + 2) for _ in range(N)]
    step()  # the group's setup (communicators, buffers) stays out of the timing
    tracer = _WsTracer(lib, lib.lib.smj_mgpu_group_workspace(0))
    elapsed, kern, brk = timed_loop(a, tracer, None, step, reset)
    k = max(acc["steps"], 1)
    xchg = {"impl": "c (smj_mgpu_join_slices: one process, one host thread per GPU)",
            **rank_phases([[v / k for v in r] for r in acc["rows"]]),
            "exchange_layout": acc["layout"], "xgmi_peak_GBps": 7 * 153}
    got = last["count"]
    ok = got == total
    chk = None
    if not a.no_check:
        # every rank's sorted shares: sorted, one key range per rank in rank
        # order, and together a permutation of the inputs (checksums)
        chk = {"sorted": True, "checksum_equal": True, "ranks_in_key_order": True}
        sums = [torch.zeros(4, dtype=torch.int64) for _ in range(4)]
        prev_hi = [None, None]
        for g in range(N):
            dev = torch.device("cuda", g)
            with torch.cuda.device(dev):
                outs = lib.mgpu_last_sorted(g, dev)
                for r, (src, out) in enumerate(((Rs[g], outs[0]), (Ss[g], outs[1]))):
                    chk["sorted"] = chk["sorted"] and _is_sorted(out, w)
                    sums[2 * r] += _checksum(src).cpu()
                    sums[2 * r + 1] += _checksum(out).cpu()
                    if out.shape[0]:
                        lo, hi = int(out[0, 1].item()), int(out[-1, 1].item())
                        if prev_hi[r] is not None and lo < prev_hi[r]:
                            chk["ranks_in_key_order"] = False
                        prev_hi[r] = hi
                del outs
        chk["checksum_equal"] = bool(torch.equal(sums[0], sums[1]) and
                                     torch.equal(sums[2], sums[3]))
        ok = ok and all(chk.values())
    ms_step = elapsed / a.steps * 1e3
    value = 2 * total / (elapsed / a.steps) / 1e6
    n0 = ns_[0]
    cfg_key = f"n{n0}_w{w}_{a.dist}" + ("" if a.payload == "rowid" else f"_{a.payload}")
    roof = dominant_roofline(kern, lambda name: alg_bytes_per_launch(name, n0, n0, n0, w),
                             cfg_key)
    strong = a.n_total is not None
    out = {
        "metric": "join throughput Mtuples/s (R⋈S) + achieved HBM GB/s, 128M⋈128M at 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "Mtuples/s",
        "n_gpus": N,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "int64" if w == 16 else "int32",
        "data": "synthetic",
        "config": {"workload": (f"sortmergejoin_mpsm R={total} S={total} over {N} GPUs"
                                if strong else
                                f"sortmergejoin_mpsm R={ns_[0]} S={ns_[0]} per GPU")
                               + f", {w}-byte tuples, {a.dist}"
                               + (f" theta={a.theta}" if a.dist == "zipf" else "")
                               + ", PK/FK keys 1..|R|, payload " + a.payload,
                   "tuples_per_relation_per_gpu": ns_[0], "tuples_per_relation_total": total,
                   "tuple_bytes": w, "payload": a.payload, "distribution": a.dist,
                   "parallelism": f"range-partition x{N}, one process, one host thread per GPU "
                                  "(smj_mgpu_join_slices, RCCL)"},
        "roofline": roof,
        "cpu_baseline": None,
        "result_ok": ok,
        "matches": got,
        "output_check": chk if chk is not None else "skipped (--no-check)",
        "detail": {
            "S_tuples_per_s_M": round(total / (elapsed / a.steps) / 1e6, 2),
            "pipeline_alg_GBps_5w_per_gpu": round(5 * 2 * total * w / N / (elapsed / a.steps)
                                                  / 1e9, 1),
            "kernels_ms_per_step_rank0": {kk: round(v[0], 4) for kk, v in brk.items()},
            "device": lib.lib.smj_device_name().decode(),
            "exchange": xchg,
        },
    }
    print(json.dumps(out), file=json_out, flush=True)
    lib.lib.smj_mgpu_release()


class _WsTracer:
    """smj_trace_* on another workspace of the library (the calling thread's
    context behind the reference-named entry points)."""

    def __init__(self, lib, ws):
        self.lib, self.ws = lib, ws

    def trace(self, on, only=None):
        self.lib.lib.smj_trace_enable(self.ws, int(on))
        self.lib.lib.smj_trace_only(self.ws, only.encode() if only else None)
        self.lib.lib.smj_trace_reset(self.ws)

    def trace_read(self):
        saved, self.lib._ws = self.lib._ws, self.ws
        try:
            return self.lib.trace_read()
        finally:
            self.lib._ws = saved


def timed_loop(a, lib, dist, step, reset=None):
    """W untimed warm-up steps and a few untimed steps with every kernel
    traced (the per-kernel breakdown, which also names the dominant kernel),
    then exactly K steps between a barrier + synchronize on both sides with
    only the dominant kernel traced (one HIP event pair per launch: the other
    kernels' events would perturb the step).  Returns (max-over-ranks
    seconds, {dominant kernel: (ms, launches)} over the timed steps,
    {kernel: ms per step} of the untimed breakdown)."""
    for _ in range(a.warmup):
        step()
    nb = max(1, min(a.steps, 3))
    lib.trace(not a.no_trace)
    for _ in range(nb):
        step()
    torch.cuda.synchronize()
    brk_l = {k: (v[0] / nb, v[1] / nb) for k, v in lib.trace_read().items()}
    brk = {k: v[0] for k, v in brk_l.items()}
    dom = max(brk, key=brk.get) if brk else None
    lib.trace(False)
    if dist:
        dist.barrier()
    if reset:
        reset()
    lib.trace(dom is not None, only=dom)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = lib.trace_read() if dom else {}
    lib.trace(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, kern, brk_l


def dominant_roofline(kern, bytes_of, cfg_key):
    """Roofline of the kernel with the largest summed time over the timed
    region: its algorithmic bytes per launch / its average launch time (HIP
    events on the library's stream), plus the PMC traffic when profiled."""
    best = None
    for name, (ms, launches) in kern.items():
        b = bytes_of(name)
        if b is None:
            continue
        if best is None or ms > best[1]:
            best = (name, ms, launches, b)
    if not best:
        return None
    name, ms, launches, b = best
    ach = b / (ms / launches / 1e3) / 1e9
    traffic = load_traffic(name, cfg_key)
    # phys: the PMC bytes of one launch over its measured average duration --
    # HBM utilisation, where frac is the algorithmic credit (16-byte tuples
    # move as packed 8-byte words, so their credit exceeds their bytes)
    phys = traffic / (ms / launches / 1e3) / 1e9 if traffic else None
    return {"bound": "hbm", "kernel": name, "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": traffic, "alg_bytes_per_launch": b,
            "avg_launch_ms": round(ms / launches, 4),
            "phys_achieved": round(phys, 1) if phys else None,
            "phys_frac": round(phys / HBM_PEAK_GBS, 4) if phys else None}


def step_phys(roof, brk_l, ms_step, cfg_key):
    """The whole step's PMC bytes (step_traffic) over the measured step time."""
    if not roof:
        return {}
    k = roof["kernel"]
    b = step_traffic(k, brk_l.get(k, (0, 0))[1], cfg_key)
    if not b:
        return {"step_pmc_bytes": None}
    g = b / (ms_step / 1e3) / 1e9
    return {"step_pmc_bytes": b, "step_phys_GBps": round(g, 1),
            "step_phys_frac": round(g / HBM_PEAK_GBS, 4)}


def run_exchange(a, json_out, N, rank, local):
    """The multi-GPU join's row exchange alone (numabench's memory bandwidth
    study, tputbench.c:665-1171, as xGMI bandwidth): S (--n tuples per GPU,
    default 128M, the join's slice) is range-partitioned once by
    DistributedJoin (its first layout: 48-bit planes where the partition
    width allows, else packed words for 16-byte tuples); one step repeats that
    exchange's row transfer -- DistributedJoin._rows, the join's own code
    path: list all-to-alls on the RCCL communicator in rounds of at most
    512 MB per peer, the own chunk read in place.  value = bytes that crossed to OTHER ranks, per
    GPU per second (N = 1: no row leaves the rank, nothing to time)."""
    import torch.distributed as dist
    import smj
    from smj.dist import DeviceOps, DistributedJoin, row_bytes
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    w = a.width or 16
    lib = smj.load(w)
    n = a.n or 128_000_000
    if N == 1 and a.sim_world > 1:
        run_exchange_device_side(a, json_out, lib, n, w)
        _close(dist)
        return
    total = n * N
    R = lib.empty(n)
    lib.dev_gen_pk(R, n * rank, total, 12345)
    S = lib.empty(n)
    lib.dev_gen_fk(S, n * rank, total, total, 54321)
    dj = DistributedJoin(DeviceOps(lib), a.fanout_bits, 1, total, n_hint=n)
    _, _, _, _, work, lay = dj._exchange(S, "S")
    work.wait()
    torch.cuda.synchronize()
    xb, cap, cs, sl, rl, gmax = dj.last_rows["S"]
    row = row_bytes(xb)

    def step():
        dj._rows(xb, cap, cs, sl, rl, gmax).wait()

    class _NoTrace:
        def trace(self, on, only=None):
            pass

        def trace_read(self):
            return {}
    elapsed, _, _ = timed_loop(a, _NoTrace(), dist if N > 1 else None, step)
    t = elapsed / a.steps
    sent = row * (sum(sl) - sl[rank])  # this rank's bytes to other ranks per step
    recv = row * (sum(rl) - rl[rank])
    tot = torch.tensor([sent, recv], dtype=torch.float64, device="cuda")
    if N > 1:
        dist.all_reduce(tot)
    if rank == 0:
        xgmi_peak = 7 * 153.0  # GB/s per GPU, one direction (MI355X_MICROARCH.md)
        per_gpu = float(tot[0]) / N / t / 1e9 if N > 1 else None
        out = {
            "metric": "exchange (the join's row exchange) GB/s per GPU over xGMI",
            "value": round(per_gpu, 1) if per_gpu is not None else 0.0,
            "unit": "GB/s", "n_gpus": N, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"words": "int64", "planes": "u48"}.get(lay, "int64" if w == 16 else "int32"),
            "data": "synthetic",
            "config": {"workload": f"row exchange of S (FK, {n} {w}-byte tuples per GPU"
                                   f"{', as ' + lay if lay != 'tuples' else ''}, {row} B a row) "
                                   f"range-partitioned over {N} rank(s)",
                       "tuples_per_gpu": n, "parallelism": f"range-partition x{N}"},
            "roofline": ({"bound": "xgmi", "achieved": round(per_gpu, 1), "peak": xgmi_peak,
                          "unit": "GB/s", "frac": round(per_gpu / xgmi_peak, 4),
                          "traffic": None} if per_gpu is not None else None),
            "cpu_baseline": None,
            "result_ok": True,
            "detail": {"bytes_sent_per_step_all_ranks": int(tot[0]),
                       "bytes_recv_per_step_all_ranks": int(tot[1]),
                       "note": None if N > 1 else
                       "N=1: every row stays on its rank and the local join reads the "
                       "own chunk in place; no bytes cross xGMI"},
        }
        print(json.dumps(out), file=json_out, flush=True)
    _close(dist)


def run_exchange_device_side(a, json_out, lib, n, w):
    """--op exchange on one GPU: what a rank of a --sim-world G world does on
    its own GPU for the exchange, timed against HBM (the rows themselves
    cross xGMI only with G GPUs).  S is rank 0's slice of the weak-scaled
    relation (n tuples, FK keys over 1..G n); one step = DistributedJoin's
    exchange attempt for S as rank 0 of G ranks runs it: the exact range
    partition into G ranks' partitions (histogram + scatter, the layout the
    plan allows: 64-bit words for 16-byte tuples at G = 8) and the table
    kernels (k_xsend, k_xrecv) with the summary read.  The roofline is the
    scatter's: it reads every tuple and writes its element once."""
    from smj.dist import DeviceOps, DistributedJoin, owned, partition_bits, row_bytes, used_parts
    G = a.sim_world
    total = n * G
    S = lib.empty(n)
    lib.dev_gen_fk(S, 0, total, total, 54321)
    torch.cuda.synchronize()
    pbits = partition_bits(a.fanout_bits, G, True, n, (1, total))
    # the ops a rank of G > 1 has: the 48-bit planes where they hold (always
    # the sampled form), else words or tuples in the exact form
    ops = DeviceOps(lib)
    ops._sampled = a.exchange_form == "sampled"
    dj = DistributedJoin(ops, a.fanout_bits, 1, total, n_hint=n, pbits=pbits)
    res = {}

    def step():
        res["x"] = dj._exchange(S, "S")
    elapsed, kern, brk = timed_loop(a, lib, None, step)
    xb, cap = dj.last_rows["S"][0], dj.last_rows["S"][1]
    eb = row_bytes(xb)
    lay = res["x"][-1]  # the layout the attempt ended in
    # rows rank 0 keeps: the partitions it owns among G ranks
    F, U = 1 << pbits, used_parts(1, total, pbits)
    lo, hi = owned(F, G, 0, U)
    t = elapsed / a.steps
    # the scatter: reads the tuple, writes its exchange element
    sc_ms, sc_n = kern.get("k_scatter", (0.0, 0))
    alg_sc = n * (w + eb)
    roof = None
    if sc_n:
        ach = alg_sc / (sc_ms / sc_n / 1e3) / 1e9
        roof = {"bound": "hbm", "kernel": "k_scatter", "pass": f"the {a.exchange_form} range partition",
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "alg_bytes_per_launch": alg_sc, "avg_launch_ms": round(sc_ms / sc_n, 4)}
    # uniform keys: (G-1)/G of the rows leave the rank, in chunks that carry
    # the sampled form's region slack (cap elements for n; exact: cap = n)
    leave = cap * (G - 1) / G * eb
    xgmi_peak = 7 * 153.0
    out = {
        "metric": "exchange (the join's row exchange) GB/s per GPU over xGMI",
        "value": 0.0, "unit": "GB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": {"words": "int64", "planes": "u48"}.get(lay, "int64"),
        "data": "synthetic",
        "config": {"workload": f"the exchange's device side of S as rank 0 of {G} GPUs: {n} "
                               f"{w}-byte FK tuples over keys 1..{total}, {a.exchange_form} range partition "
                               f"into 2^{pbits} partitions as {lay} ({eb} B a row) + table kernels",
                   "tuples_per_gpu": n, "parallelism": f"one GPU, rank 0 of a simulated x{G}"},
        "roofline": roof,
        "cpu_baseline": None,
        "result_ok": True,
        "detail": {
            "note": "one GPU: no row crosses xGMI, value 0; this line times the device work a "
                    f"rank does for the exchange at {G} GPUs (HBM roofline of its partition)",
            "kernels_ms_per_step": {k: round(v[0], 4) for k, v in brk.items()},
            "exchange_layout": lay, "partition_bits": pbits, "owned_partitions_rank0": hi - lo,
            "partition_form": "sampled (regions with slack)" if cap > n else "exact",
            "elements_with_slack": int(cap),
            "xgmi_bytes_leaving_rank_per_step": int(leave),
            "xgmi_ms_at_link_peak": round(leave / (xgmi_peak * 1e9) * 1e3, 3),
            "xgmi_peak_GBps": xgmi_peak,
        },
    }
    print(json.dumps(out), file=json_out, flush=True)


def partition_check(R, out, hist, off, bits, shift, w):
    """partition_relation_optimized's output on the device: counts sum to n,
    every partition starts on a 64-byte boundary, every tuple of partition p
    has digit p (((key - 1) & mask) >> shift, partition.c:29), and the
    partitions together are a permutation of the input (checksums)."""
    n = R.shape[0]
    fan = 1 << bits
    res = {"counts_sum": int(hist.sum().item()) == n,
           "aligned_64B": bool(((off * w) % 64 == 0).all().item())}
    pid = torch.repeat_interleave(torch.arange(fan, device="cuda"), hist)
    base = torch.cumsum(hist, 0) - hist
    pos = off[pid] + torch.arange(n, device="cuda") - base[pid]
    # gathered in chunks: one 2^27-row gather of 16-byte rows exceeds the
    # launch configuration torch's index kernel accepts on this part
    rows = torch.empty((n,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
    for i in range(0, n, 1 << 24):
        rows[i:i + (1 << 24)] = out.index_select(0, pos[i:i + (1 << 24)])
    mask = ((1 << bits) - 1) << shift
    dig = ((rows[:, 1].to(torch.int64) - 1) & mask) >> shift
    res["digits"] = bool((dig == pid).all().item())
    res["checksum_equal"] = bool(torch.equal(_checksum(R), _checksum(rows)))
    return res


def run_op(a, lib, json_out, dist, N, rank):
    """bench_sort / bench_partitioning on the device (BASELINE configs 2 and
    3): one step = one smj_dev_sort (avxsort_tuples' device form) or one
    smj_dev_partition (partition_relation_optimized: stable, 64-byte padded)
    over a device-resident relation of n tuples, keys 1..n permuted (the
    shape of create_relation_pk), payload 0.  N GPUs run N independent
    replicas (the ops do not shard across GPUs: scaling "weak")."""
    w, n = a.width, a.n
    if a.op == "merge":  # n tuples per run
        n = a.n * a.fanin
    R = lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345, with_payload=False)
    if a.op == "merge":
        # --fanin runs of increasing keys, random steps in [0, 100) as
        # generate_rand_ordered_tuples (tests/testutil.c:266-287); separate
        # allocations, as the reference bench mallocs every run
        dt = torch.int32 if w == 8 else torch.int64
        g = torch.Generator(device="cuda").manual_seed(2012)
        steps = torch.randint(0, 100, (a.fanin, a.n), device="cuda", generator=g,
                              dtype=torch.int64)
        steps[:, 0] = torch.randint(1, 101, (a.fanin,), device="cuda", generator=g)
        keys = steps.cumsum(dim=1).clamp_(max=(1 << 31) - 101).to(dt)
        del steps
        runs = []
        for i in range(a.fanin):
            t = lib.empty(a.n)
            t[:, 0] = 0
            t[:, 1] = keys[i]
            runs.append(t)
        del keys
        out = lib.empty(n)
        table = lib.run_table(runs)  # the reference's driver builds its run array once too

        def step():
            lib.dev_multiway_merge(table, out)
    elif a.op == "sort":
        out = lib.empty(n)

        def step():
            lib.dev_sort(R, out)
    else:
        fan = 1 << a.bits
        out = lib.empty(n + fan * 64 // w)
        hist = torch.zeros(fan, dtype=torch.int64, device="cuda")
        off = torch.zeros_like(hist)

        def step():
            lib.dev_partition(R, out, a.bits, a.shift, True, hist, off)
    torch.cuda.synchronize()
    elapsed, kern, brk = timed_loop(a, lib, dist, step)
    layout = lib.last_layout() if a.op == "sort" else None
    chk = None
    if a.no_check:
        ok = True
    elif a.op == "sort":
        chk = output_check([(R, out)], w)
    elif a.op == "merge":
        chk = output_check([(torch.cat(runs), out)], w)
    else:
        chk = partition_check(R, out, hist, off, a.bits, a.shift, w)
    if chk is not None:
        ok = all(v for v in chk.values() if isinstance(v, bool))
    if rank != 0:
        if dist:
            _close(dist)
        return
    ms_step = elapsed / a.steps * 1e3
    value = N * n / (elapsed / a.steps) / 1e6
    cfg_key = f"{a.op}_n{n}_w{w}"
    roof = dominant_roofline(kern, lambda name: alg_bytes_per_launch(name, n, n, 0, w, a.op),
                             cfg_key)
    alg = 2 * n * w  # 2·N·w for bench_sort and bench_partitioning
    cpu = None
    if N == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline_op(a.op, w, a.n if a.op == "merge" else n, a.bits, a.shift, a.fanin)
    ref = {"sort": "src/bench/sortbench.c:85-202 (avxsort_tuples)",
           "merge": "src/bench/multiwaymergebench.c:48-120 (avx_multiway_merge)",
           "partition": "src/bench/partitioningbench.c:128-196 (partition_relation_optimized)"}[a.op]
    out_line = {
        "metric": {"sort": "bench_sort", "partition": "bench_partitioning",
                   "merge": "bench_multiwaymerge"}[a.op]
                  + " throughput Mtuples/s + achieved HBM GB/s (2·N·w)",
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
        "config": {"workload": (f"{a.op} of {n} {w}-byte tuples" +
                                {"partition": f", {a.bits} radix bits, shift {a.shift}, "
                                              "64-byte padded, stable",
                                 "sort": ", full (key, payload) order",
                                 "merge": f", {a.fanin} sorted runs of {a.n}"}[a.op]
                                + (", keys in random steps, payload 0" if a.op == "merge" else
                                   ", keys 1..N permuted, payload 0")
                                + "; reference " + ref),
                   "tuples": n, "tuple_bytes": w, "parallelism": f"replicas x{N}"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "result_ok": ok,
        "output_check": chk if chk is not None else "skipped (--no-check)",
        "detail": {
            "alg_GBps_2Nw": round(alg / (elapsed / a.steps) / 1e9, 1),
            "alg_frac_2Nw": round(alg / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
            **step_phys(roof, brk, ms_step, cfg_key),
            # untimed steps, every kernel traced (timed_loop)
            "kernels_ms_per_step": {k: round(v[0], 4) for k, v in brk.items()},
            "device": lib.lib.smj_device_name().decode(),
            "intermediate_layout": layout,
        },
    }
    print(json.dumps(out_line), file=json_out, flush=True)
    if dist:
        _close(dist)


if __name__ == "__main__":
    main()
