"""bench.py's timed loop on CPU (no GPU calls): warm-up, an untimed breakdown
with every kernel traced, then exactly K timed steps with only the dominant
kernel traced, and the roofline taken from that kernel."""
import types

import pytest

import bench


class FakeTraceLib:
    """Stands in for smj.Library's trace_* (the kernel times of one step are
    fixed: two scatter launches of 0.6 ms, one group pass of 1.3 ms)."""

    STEP = {"k_scatter": (1.2, 2), "k_groupsort": (1.3, 1), "k_sample": (0.02, 1)}

    def __init__(self):
        self.on, self.only, self.steps, self.calls = False, None, 0, []

    def trace(self, on, only=None):
        self.on, self.only, self.steps = on, only, 0
        self.calls.append((on, only))

    def step(self):
        if self.on:
            self.steps += 1

    def trace_read(self):
        # like smj_trace_read: nothing recorded -> no names
        if not self.steps:
            return {}
        out = {}
        for k, (ms, n) in self.STEP.items():
            if self.only in (None, k):
                out[k] = (ms * self.steps, n * self.steps)
        return out


@pytest.fixture
def no_cuda_sync(monkeypatch):
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda *a, **k: None)


def run(lib, steps=7, warmup=2, no_trace=False):
    a = types.SimpleNamespace(steps=steps, warmup=warmup, no_trace=no_trace)
    n = [0]

    def step():
        n[0] += 1
        lib.step()

    elapsed, kern, brk = bench.timed_loop(a, lib, None, step)
    return n[0], elapsed, kern, brk


def test_dominant_kernel_alone_in_timed_steps(no_cuda_sync):
    lib = FakeTraceLib()
    n, elapsed, kern, brk = run(lib)
    assert n == 2 + 3 + 7  # warm-up, untimed breakdown, timed
    assert elapsed >= 0
    assert {k: v[0] for k, v in brk.items()} == pytest.approx(
        {k: v[0] for k, v in FakeTraceLib.STEP.items()})
    assert {k: v[1] for k, v in brk.items()} == pytest.approx(
        {k: v[1] for k, v in FakeTraceLib.STEP.items()})
    # the timed steps trace the kernel with the largest summed time only
    assert (True, "k_groupsort") in lib.calls
    assert kern == {"k_groupsort": pytest.approx((1.3 * 7, 7))}
    assert lib.calls[-1] == (False, None)


def test_roofline_from_the_timed_kernel(no_cuda_sync):
    lib = FakeTraceLib()
    _, _, kern, _ = run(lib)
    roof = bench.dominant_roofline(kern, lambda name: 8.192e9 if name == "k_groupsort" else None,
                                   "none")
    assert roof["kernel"] == "k_groupsort"
    assert roof["avg_launch_ms"] == pytest.approx(1.3)
    assert roof["frac"] == pytest.approx(8.192e9 / 1.3e-3 / 1e9 / bench.HBM_PEAK_GBS, rel=1e-3)


def test_no_trace_lab_switch(no_cuda_sync):
    lib = FakeTraceLib()
    n, _, kern, brk = run(lib, steps=1, warmup=0, no_trace=True)
    assert n == 1 + 1  # one untimed step (at least one), one timed
    assert kern == {} and brk == {}
    assert bench.dominant_roofline(kern, lambda name: 1.0, "none") is None


def test_phys_fields(monkeypatch):
    """roofline.phys_frac = PMC bytes per launch / average launch time / peak
    beside the credited frac; the step's PMC bytes from every library kernel
    of the profiled run over its step count."""
    pmc = {"k_groupsort": {"bytes": 6.3e9, "launches": 15},
           "k_scatter": {"bytes": 3.2e9, "launches": 30},
           "k_tilepass": {"bytes": 4.1e9, "launches": 15},
           "k_gen_perm": {"bytes": 2e9, "launches": 2}}
    monkeypatch.setattr(bench, "_pmc", lambda key: pmc)
    kern = {"k_groupsort": (1.28 * 10, 10)}
    roof = bench.dominant_roofline(kern, lambda name: 8.192e9, "cfg")
    assert roof["traffic"] == int(6.3e9)
    assert roof["phys_frac"] == pytest.approx(6.3e9 / 1.28e-3 / 1e9 / bench.HBM_PEAK_GBS,
                                              rel=1e-3)
    assert roof["frac"] > roof["phys_frac"]
    sp = bench.step_phys(roof, {"k_groupsort": (1.28, 1.0), "k_scatter": (1.2, 2.0)}, 3.4,
                         "cfg")
    step_bytes = 6.3e9 + 2 * 3.2e9 + 4.1e9  # the generator is not part of a step
    assert sp["step_pmc_bytes"] == pytest.approx(step_bytes, rel=1e-6)
    assert sp["step_phys_frac"] == pytest.approx(step_bytes / 3.4e-3 / 1e9 / bench.HBM_PEAK_GBS,
                                                 rel=1e-3)


@pytest.mark.parametrize("w", [8, 16])
def test_output_check_on_cpu_tensors(w):
    """bench.py's output check (sortedness in the library's order, checksums
    against the input) on CPU tensors of the bench's (n, 2) layout."""
    import torch
    dt = torch.int32 if w == 8 else torch.int64
    g = torch.Generator().manual_seed(5)
    keys = torch.randint(1, 1000, (5000,), generator=g)
    pay = torch.randint(-(1 << 30), 1 << 30, (5000,), generator=g)
    src = torch.stack([pay, keys], 1).to(dt)
    # the library's order: (key, payload), payload unsigned for 8-byte tuples
    p64 = src[:, 0].to(torch.int64)
    pk = p64 & 0xFFFFFFFF if w == 8 else p64
    order = sorted(range(5000), key=lambda i: (int(src[i, 1]), int(pk[i])))
    out = src[torch.tensor(order)]
    assert bench.output_check([(src, out)], w) == {"sorted": True, "checksum_equal": True}
    bad = out.clone()
    bad[10], bad[11] = out[11].clone(), out[10].clone()
    if not torch.equal(bad, out):
        assert bench.output_check([(src, bad)], w)["sorted"] is False
    lost = out.clone()
    lost[7] = lost[8]
    assert bench.output_check([(src, lost)], w)["checksum_equal"] is False


# --gpus N: never a line for fewer GPUs than asked (this container has none)
def _bench(args, env_extra):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, bench.__file__] + args, capture_output=True,
                          text=True, env=env, timeout=300, cwd="/tmp")


def test_gpus_more_than_visible_exits_nonzero():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _bench(["--gpus", str(n)], {})
    assert r.returncode == 2, r.stderr[-500:]
    assert r.stdout.strip() == ""  # no JSON line
    assert "visible" in r.stderr


@pytest.mark.parametrize("world,gpus", [("1", "2"), ("2", "8"), ("8", "1")])
def test_gpus_must_match_the_launcher(world, gpus):
    r = _bench(["--gpus", gpus], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-500:]
    assert r.stdout.strip() == ""
    assert "WORLD_SIZE" in r.stderr


def test_rank_phases_detail():
    rows = [[0.2, 0.05, 0.1, 2.5, 0.01, 2.86, 0.7, 1e9, 1.1e9],
            [0.2, 0.05, 0.3, 2.5, 0.01, 3.06, 0.8, 1.2e9, 0.9e9]]
    d = bench.rank_phases(rows)
    assert d["slowest_rank"] == 1
    assert d["xgmi_bytes_sent_per_gpu"] == int(1.2e9)
    assert d["xgmi_bytes_recv_per_gpu"] == int(1.1e9)
    for r in d["phases_ms_per_rank"]:
        parts = sum(r[p] for p in bench.PHASES[:5])
        assert abs(parts - r["busy_ms"]) < 1e-6
