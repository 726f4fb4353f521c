"""GPU tests of the multi-GPU join reached through the C ABI
(sortmergejoin_mpsm / smj_mgpu_join, csrc/mgpu.hip over csrc/mgpu_orch.hpp).

On a one-GPU box the RCCL form runs one rank (ncclCommInitAll over one device,
the count through ncclAllReduce); the G-rank protocol runs with several ranks
on the one GPU through device-copy collectives (SMJ_MG_COPY): the same
orchestration, partitions, exchange table kernels, row placement and
segmented local joins as on G GPUs, only the bytes move by hipMemcpy instead
of RCCL.  Every case compares the count and the globally sorted relations
(the ranks' shares in rank order) with the oracle.
"""
import numpy as np
import pytest

from smj import MG_COPY, MG_EXACT, MG_NOPLANES, MG_ONECALL, MG_SAMPLED  # noqa: E402

pytestmark = pytest.mark.gpu


def relations(orc, w, n, kind, seed=12345):
    orc.seed(seed)
    R = orc.create_relation_pk(n)
    R["payload"] = np.arange(n) + 5
    orc.seed(seed + 1)
    if kind == "zipf":
        S = orc.create_relation_zipf(n, n, 0.75)
    else:
        S = orc.create_relation_fk(n, n)
        S["payload"] = np.arange(n)
    if kind == "negative":
        S["payload"] = -1 - np.arange(n)
    if kind == "wide48" and w == 16:
        S["payload"] = (1 << 45) + np.arange(n)
    if kind == "outside":
        S["key"] = S["key"] + 2 * n
    return R, S


def check(orc, R, S, got):
    c, sR, sS, counts, stats = got
    want, eR, eS = orc.sortmergejoin(R, S)
    assert c == want
    assert np.array_equal(sR, eR)
    assert np.array_equal(sS, eS)
    assert counts[:, 0].sum() == len(R) and counts[:, 1].sum() == len(S)
    return stats


@pytest.mark.parametrize("G,flags", [(1, 0), (1, MG_COPY), (2, MG_COPY), (3, MG_COPY),
                                     (8, MG_COPY)], ids=["rccl1", "copy1", "copy2", "copy3",
                                                         "copy8"])
@pytest.mark.parametrize("kind", ["uniform", "zipf", "negative", "wide48"])
def test_mgpu_join_vs_oracle(libs, oracles, width, G, flags, kind):
    orc, lib = oracles[width], libs[width]
    n = (1 << 20) + 4097
    R, S = relations(orc, width, n, kind)
    st = check(orc, R, S, lib.mgpu_join(R, S, G, flags))
    if width == 16 and kind == "negative":
        assert st["layout"] == "tuples"
    elif width == 16 and kind == "wide48":
        assert st["layout"] == "words"
    else:
        assert st["layout"] == "planes"
    assert st["replans"] == 0


@pytest.mark.parametrize("G,flags", [(1, 0), (8, MG_COPY)], ids=["rccl1", "copy8"])
def test_mgpu_join_4m(libs, oracles, width, G, flags):
    """The C path at 4M x 4M: sorted outputs bit-exact against the oracle."""
    orc, lib = oracles[width], libs[width]
    R, S = relations(orc, width, 4 << 20, "uniform", seed=54321)
    check(orc, R, S, lib.mgpu_join(R, S, G, flags))


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("flags", [MG_NOPLANES, MG_ONECALL, MG_SAMPLED,
                                   MG_EXACT | MG_NOPLANES],
                         ids=["noplanes", "onecall", "sampled", "exact"])
def test_mgpu_join_forms(libs, oracles, width, G, flags):
    orc, lib = oracles[width], libs[width]
    R, S = relations(orc, width, 300007, "zipf", seed=777)
    st = check(orc, R, S, lib.mgpu_join(R, S, G, flags | MG_COPY))
    if flags & MG_NOPLANES:
        assert st["layout"] == ("words" if width == 16 else "tuples")


@pytest.mark.parametrize("G,flags", [(1, 0), (3, MG_COPY), (8, MG_COPY)],
                         ids=["rccl1", "copy3", "copy8"])
def test_mgpu_join_replan_and_device_input(libs, oracles, width, G, flags):
    """Keys outside the guessed 1..|R|: one replan to the measured range.
    Device-resident input (torch tensors): read in place by the ranks on its
    device, sorted output written to device memory."""
    import torch
    orc, lib = oracles[width], libs[width]
    R, S = relations(orc, width, 200003, "outside", seed=4242)
    st = check(orc, R, S, lib.mgpu_join(R, S, G, flags))
    assert st["replans"] == 1
    it = np.int64 if width == 16 else np.int32
    tR = torch.from_numpy(R.view(it).reshape(-1, 2).copy()).cuda()
    tS = torch.from_numpy(S.view(it).reshape(-1, 2).copy()).cuda()
    c, sR, sS, counts, st = lib.mgpu_join(tR, tS, G, flags)
    want, eR, eS = orc.sortmergejoin(R, S)
    assert c == want
    assert np.array_equal(sR.cpu().numpy().reshape(-1).view(R.dtype), eR)
    assert np.array_equal(sS.cpu().numpy().reshape(-1).view(S.dtype), eS)


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("nR,nS", [(7, 5), (0, 100), (100, 0), (0, 0), (1, 1), (9, 100000)])
def test_mgpu_join_ragged_and_empty(libs, oracles, width, G, nR, nS):
    orc, lib = oracles[width], libs[width]
    orc.seed(5)
    R = orc.create_relation_pk(max(nR, 1))[:nR].copy()
    orc.seed(6)
    S = orc.create_relation_fk(max(nS, 1), max(nR, 1))[:nS].copy()
    check(orc, R, S, lib.mgpu_join(R, S, G, MG_COPY))


def test_mpsm_reference_api(libs, oracles, width):
    """sortmergejoin_mpsm through the reference's relation_t / joinconfig_t
    (NTHREADS 8 -> one rank per visible GPU, RCCL): the count of m-way, the
    materialised output of the oracle."""
    orc, lib = oracles[width], libs[width]
    R, S = relations(orc, width, 500009, "zipf", seed=99)
    want = orc.merge_join(orc.sort(R), orc.sort(S))
    assert lib.sortmergejoin_multiway(R, S, nthreads=8, algo="mpsm") == want
    assert lib.sortmergejoin_multiway(R, S, nthreads=8, algo="m-way") == want
    c, out = lib.sortmergejoin_multiway(R, S, nthreads=8, algo="mpsm", materialize=True)
    exp = orc.merge_join_materialize(orc.sort(R), orc.sort(S))
    assert c == want == len(out)
    assert np.array_equal(out, exp)


def test_mgpu_configurations_alternate(libs, oracles):
    """Calls alternating between configurations (RCCL one rank, copies at
    G = 8, the reference-named mpsm) rebuild the ranks each time and keep
    giving the oracle's answer."""
    orc, lib = oracles[16], libs[16]
    R, S = relations(orc, 16, 100003, "uniform", seed=31)
    want = orc.sortmergejoin(R, S)[0]
    for G, flags in ((1, 0), (8, MG_COPY), (1, 0), (3, MG_COPY)):
        assert lib.mgpu_join(R, S, G, flags, sorted_out=False)[0] == want
        assert lib.sortmergejoin_multiway(R, S, nthreads=4, algo="mpsm") == want
    lib.lib.smj_mgpu_release()


@pytest.mark.parametrize("kind", ["uniform", "zipf", "outside"])
def test_mgpu_rank_comm_world1(libs, oracles, width, kind):
    """The multi-process entry (smj_mgpu_comm_init over ncclCommInitRank +
    ncclCommSplit, smj_mgpu_rank_join, smj_mgpu_rank_sorted) as one rank of a
    world of one: device slices in, count and sorted shares as the oracle's;
    a second call on the same communicator reuses its buffers."""
    import torch
    orc, lib = oracles[width], libs[width]
    R, S = relations(orc, width, 300007, kind, seed=2024)
    want, eR, eS = orc.sortmergejoin(R, S)
    it = np.int64 if width == 16 else np.int32
    tR = torch.from_numpy(R.view(it).reshape(-1, 2).copy()).cuda()
    tS = torch.from_numpy(S.view(it).reshape(-1, 2).copy()).cuda()
    comm = lib.mgpu_comm(1, 0)
    try:
        for _ in range(2):
            c, nR, nS, st = comm.join(tR, tS, guess_max=len(R))
            assert c == want and (nR, nS) == (len(R), len(S))
            assert st["replans"] == (1 if kind == "outside" else 0)
            sR, sS = comm.sorted()
            assert np.array_equal(sR.cpu().numpy().reshape(-1).view(R.dtype), eR)
            assert np.array_equal(sS.cpu().numpy().reshape(-1).view(S.dtype), eS)
    finally:
        comm.close()


def _phases_ok(st):
    """smj_mgpu_stats phases: the five main-stream phases add up to busy_ms
    (wait_ms is its remainder, never negative); the partition and the local
    join took time on the device."""
    five = (st["partition_ms"] + st["tables_ms"] + st["wait_ms"] + st["join_ms"]
            + st["reduce_ms"])
    assert abs(five - st["busy_ms"]) <= 1e-3 + 1e-6 * st["busy_ms"], st
    assert st["partition_ms"] > 0 and st["join_ms"] > 0 and st["wait_ms"] >= 0, st
    assert st["busy_ms"] <= st["ms"] * 1.05 + 0.05, st  # device span within the call


@pytest.mark.parametrize("G,flags", [(1, 0), (3, MG_COPY), (8, MG_COPY)],
                         ids=["rccl1", "copy3", "copy8"])
@pytest.mark.parametrize("kind", ["uniform", "zipf", "wide48"])
def test_mgpu_join_slices_vs_oracle(libs, oracles, width, G, flags, kind):
    """smj_mgpu_join_slices: rank g's slices are separate device tensors
    (ragged, one rank's S slice empty at G > 1), read in place; the ranks'
    sorted shares (smj_mgpu_last_sorted) in rank order are the oracle's
    sorted relations, and every rank reports its device phases
    (smj_mgpu_last_stats)."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = (1 << 20) + 777
    R, S = relations(orc, width, n, kind, seed=808)
    want, eR, eS = orc.sortmergejoin(R, S)
    it = np.int64 if width == 16 else np.int32
    cutR = sorted({0, n} | {n * g // G + 13 * g for g in range(1, G)})
    cutS = sorted({0, n} | {n * g // G - 7 * g for g in range(1, G)})
    if G > 1:
        cutS[1] = cutS[0]  # rank 0 gets no S
    tR = torch.from_numpy(R.view(it).reshape(-1, 2).copy()).cuda()
    tS = torch.from_numpy(S.view(it).reshape(-1, 2).copy()).cuda()
    Rs = [tR[cutR[g]:cutR[g + 1]].clone() for g in range(G)]
    Ss = [tS[cutS[g]:cutS[g + 1]].clone() for g in range(G)]
    for _ in range(2):  # the second call reuses the group's buffers
        c, counts, sts = lib.mgpu_join_slices(Rs, Ss, flags, key_range=None)
        assert c == want
        assert counts[:, 0].sum() == n and counts[:, 1].sum() == n
        outR, outS = [], []
        for g in range(G):
            sR, sS = lib.mgpu_last_sorted(g, "cuda")
            assert (sR.shape[0], sS.shape[0]) == tuple(counts[g])
            outR.append(sR.cpu().numpy().reshape(-1).view(R.dtype))
            outS.append(sS.cpu().numpy().reshape(-1).view(S.dtype))
        assert np.array_equal(np.concatenate(outR), eR)
        assert np.array_equal(np.concatenate(outS), eS)
        for st in sts:
            _phases_ok(st)
        if G > 1:
            assert all(st["rows_ms"] > 0 for st in sts)
    assert lib.mgpu_last_stats(0)["layout"] == sts[0]["layout"]
    with pytest.raises(IndexError):
        lib.mgpu_last_stats(G)
    lib.lib.smj_mgpu_release()


def test_mgpu_rank_comm_phases(libs, oracles):
    """The multi-process entry's stats carry the phases too (one rank)."""
    import torch
    orc, lib = oracles[16], libs[16]
    R, S = relations(orc, 16, 500009, "uniform", seed=11)
    tR = torch.from_numpy(R.view(np.int64).reshape(-1, 2).copy()).cuda()
    tS = torch.from_numpy(S.view(np.int64).reshape(-1, 2).copy()).cuda()
    comm = lib.mgpu_comm(1, 0)
    try:
        for _ in range(2):
            c, _, _, st = comm.join(tR, tS, key_range=(1, len(R)))
            assert c == orc.sortmergejoin(R, S)[0]
            _phases_ok(st)
            assert st["rows_ms"] == 0  # nothing travels on one rank
    finally:
        comm.close()
