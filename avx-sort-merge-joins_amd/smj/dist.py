"""Multi-GPU m-way sort-merge join: one process per GPU over torch.distributed.

SURVEY.md §8(e).  The reference scales over the threads of one host: thread i
range-partitions its chunk of R and S, the co-partitions are redistributed so
that every thread owns whole key ranges, each thread sorts, merges and joins
its own ranges, and the per-thread counts are summed
(src/joins/sortmergejoin_multiway.c:195-330, threads joined in
src/joins/joincommon.c:140-260).  Here a rank plays the part of a thread:

1. range-partition the local slices of R and S on the device into
   F = 2^pbits partitions (``smj_dev_partition_range``: the library's range
   plan over the GLOBAL key range, so partition p holds one contiguous key
   interval of width 2^s1);
2. partition p is owned by rank ``p * world // F`` -- contiguous, balanced
   ownership, so every key lands on exactly one rank;
3. per relation one ``all_to_all_single`` of the owned partition sizes and
   one of the rows (RCCL over xGMI on the GPU, gloo in the CPU tests).  The
   row exchange of R is asynchronous: it runs on the communication stream
   while S is partitioned;
4. the received partitions ARE the level-1 buckets of the local sort
   (``smj_dev_join_segmented``: source s's partitions back to back, one
   segment per source), so the local join starts at its tile pass -- no
   second partition pass -- then an ``all_reduce`` of the count.

The class is written against a small ``ops`` interface (``empty``,
``partition_range``, ``join_segmented``) so that the orchestration the GPU
bench runs is the same code the CPU multi-process tests run (with host
stand-ins for the device ops that live in tests/).
"""
from __future__ import annotations


import torch
import torch.distributed as dist

# Widest exchange partition: 2^10 partitions.  At 8 GPUs that is 128 per
# rank, each ~1M tuples of a relation in 8 source segments (~130 tiles of the
# local tile pass: the group pass takes up to 256 per bucket, and the 1-GPU
# join with 2^7 sampled partitions runs exactly that shape).  The exact
# scatter costs 0.96 / 1.09 / 1.53 / 3.32 ms per 128M 16-byte tuples at
# 9 / 10 / 11 / 12 bits (tools/bench_xpart.py): wider exchange partitions
# scatter too thinly.
MAX_PARTITION_BITS = 10
INT64_MAX = (1 << 63) - 1
# Largest single message of the row exchange.  RCCL 2.26.6 (torch 2.10 ROCm)
# on a one-rank group leaves the second half of an all_to_all_single message
# unwritten once the message exceeds 1 GiB: tools/a2a_bisect.py steps the
# size in bytes for uint8, int32 and int64 elements and the first bad byte is
# exactly half the message every time, from 1100 MiB up (1024 MiB is exact),
# so the limit is a byte count inside RCCL, not an element count of ours
# (profiles/r02_a2a_bisect.txt).  Larger exchanges go as chunked
# point-to-point sends in one group.  (A module attribute: tests lower it to
# exercise the chunked path.)
CHUNK_BYTES = 512 << 20
# The exchange layouts, narrowest last: tuples, 64-bit packed words (16-byte
# tuples only), 48-bit words in two planes (LayP48, both widths; the sampled
# partition's LDS carries hold at most 2^10 partitions of them with 16-byte
# segments: round 6, 2^9 before).  Both relations of a step reach the local
# join in one layout.
LAYOUTS = ("tuples", "words", "planes")
PLANE_MAX_BITS = 10
# a local bucket the tile pass / group pass take in stride: <= 192 tiles of
# 16384 elements (choose_levels' bucket_cap in the library)
LOCAL_BUCKET_CAP = 192 * 16384
# the partition's not-packable bits (smj_common.hpp kBad*): 1 payload wider
# than a 64-bit word holds, 2 key outside the plan, 4 payload wider than a
# 48-bit word holds -- also what a rank where the planes form does not apply
# reports (every rank then takes packed words)
BAD_PAYLOAD, BAD_RANGE, BAD_PAYLOAD48 = 1, 2, 4


class Planes:
    """An exchange buffer of 48-bit words in two planes of one int32 buffer
    (smj_dev_partition_range_planes): lo = int32[stride], then hi =
    int16[stride]; element i is lo[i] | hi[i] << 32 (unsigned).  6 bytes an
    element on the wire and in HBM instead of 8 (words) or 16 (tuples)."""

    def __init__(self, stride: int, device=None):
        assert stride % 32 == 0
        self.stride = stride
        self.buf = torch.empty(stride * 3 // 2, dtype=torch.int32, device=device)
        self.lo = self.buf[:stride]
        self.hi = self.buf[stride:].view(torch.int16)
        self.planes = (self.lo, self.hi)

    @property
    def is_cuda(self):
        return self.buf.is_cuda

    @property
    def device(self):
        return self.buf.device

    def data_ptr(self):
        return self.buf.data_ptr()


def _wire(t):
    """A row piece as RCCL carries it (it has no 16-bit integer type: the hi
    plane goes as bytes)."""
    return t.view(torch.uint8) if t.dtype == torch.int16 else t


def row_bytes(xb) -> int:
    """Bytes one element of an exchange buffer takes (all planes)."""
    planes = xb.planes if isinstance(xb, Planes) else (xb,)
    return sum(p.element_size() * (p[0].numel() if p.dim() > 1 else 1) for p in planes)


class _Works:
    """wait() on several collective works (or none)."""

    def __init__(self, works):
        self.works = [w for w in works if w is not None]

    def wait(self):
        for w in self.works:
            w.wait()


def owners(fanout: int, world: int, used: int | None = None) -> torch.Tensor:
    """Owner rank of each of the `fanout` range partitions (contiguous): the
    `used` partitions the key range reaches (used_parts; None = all) split
    evenly, the ones above them to the last rank.  Splitting the power-of-two
    partition space instead would leave the last rank short whenever the key
    span is not a power of two (keys 1..1024M at 2^10 partitions reach 977:
    ranks 0-6 would own 134M keys each and rank 7 85M)."""
    u = fanout if used is None else used
    p = torch.arange(fanout, dtype=torch.int64)
    return torch.where(p < u, p * world // u, world - 1)


def owned(fanout: int, world: int, rank: int, used: int | None = None) -> tuple[int, int]:
    """[first, last) partition owned by `rank` (the inverse of owners)."""
    u = fanout if used is None else used

    def first(g):
        return fanout if g >= world else -(-g * u // world)
    return first(rank), first(rank + 1)


def used_parts(key_min: int, key_max: int, pbits: int) -> int:
    """The exchange partitions the key range [key_min, key_max] reaches:
    partition p starts at base + p 2^s1 (base = local_range's, key_min moved
    down near INT64_MAX)."""
    L = max(key_max - key_min, 0).bit_length()
    base = min(key_min, INT64_MAX - (1 << L) + 1)
    s1 = plan_shift(base, key_max, pbits)
    return min(1 << pbits, ((max(key_max - base, 0)) >> s1) + 1)


def plan_shift(key_min: int, key_max: int, bits: int) -> int:
    """s1 of the library's range plan (smj_common.hpp make_plan): partition
    p covers keys [key_min + p * 2^s1, key_min + (p + 1) * 2^s1)."""
    width = max(key_max - key_min, 0)
    return max(width.bit_length() - bits, 0)


def range_digit(keys: torch.Tensor, key_min: int, key_max: int, bits: int) -> torch.Tensor:
    """The level-1 digit of the range plan (plan_rel + d1), for host stand-ins."""
    L = max(key_max - key_min, 0).bit_length()
    rel = (keys.to(torch.int64) - key_min).clamp(0, (1 << L) - 1)
    return rel >> plan_shift(key_min, key_max, bits)


def planes_hold(key_min: int, key_max: int, pbits: int) -> bool:
    """Whether 48-bit words are worth trying at 2^pbits exchange partitions:
    a word holds the key's s1 low bits and a payload below 2^(48 - s1), and
    payloads are taken to lie within the key span (the row ids of a PK
    relation, as in the benchmark).  Where they would not, every step would
    partition twice (planes, then 64-bit words once a rank reports a payload
    too wide), so the exchange starts with words: 128M per rank at G = 8 is
    such a case (keys 1..1024M, 2^10 partitions: s1 = 20, payloads below
    2^28); at G = 4 (keys 1..512M, s1 = 19) row ids fit."""
    s1 = plan_shift(key_min, key_max, pbits)
    return 1 <= s1 <= 32 and key_max - key_min < (1 << (48 - s1))


def partition_bits(bucket_bits: int, world: int, planes: bool, n_hint=None,
                   key_range=None) -> int:
    """Exchange partition width: bucket_bits per rank (2^min(bucket_bits +
    log2 G, 10) partitions), unless the 48-bit planes are offered and one bit
    less keeps them (only where PLANE_MAX_BITS < MAX_PARTITION_BITS, as before
    round 6): 2^9 partitions, when every rank's share (n_hint elements
    per relation, balanced) still splits into local buckets of at most
    LOCAL_BUCKET_CAP elements (at 128M per rank up to G = 8: 2^6 local
    buckets of 2M) and, given key_range, the words hold the payloads
    (planes_hold: with the benchmark's row-id payloads only G <= 2)."""
    pbits = min(bucket_bits + ceil_log2(world), MAX_PARTITION_BITS)
    if planes and pbits > PLANE_MAX_BITS and n_hint is not None:
        lbits = PLANE_MAX_BITS - ceil_log2(world)
        fits = key_range is None or planes_hold(key_range[0], key_range[1], PLANE_MAX_BITS)
        if fits and lbits >= 6 and -(-n_hint // (1 << lbits)) <= LOCAL_BUCKET_CAP:
            pbits = PLANE_MAX_BITS
    return pbits


def ceil_log2(x: int) -> int:
    return max(x - 1, 0).bit_length()


def local_range(key_min: int, key_max: int, pbits: int, world: int, rank: int):
    """(plan base, key_lo, key_hi, lbits) of `rank`.

    The global plan covers [base, base + 2^L) with L the bit length of
    key_max - key_min; near INT64_MAX that top would pass the int64 range, so
    the base moves down instead (the width keeps its bit length L; every rank
    computes the same base).  The rank's partitions [p_lo, p_hi) are the
    level-1 buckets of its local plan, 2^lbits of them; [key_lo, key_hi] only
    fixes that plan's bit length s1 + lbits (make_plan), and the smallest such
    width keeps key_hi inside the global range, so inside int64."""
    used = used_parts(key_min, key_max, pbits)
    L = max(key_max - key_min, 0).bit_length()
    if key_min + (1 << L) - 1 > INT64_MAX:
        key_min = INT64_MAX - (1 << L) + 1
    F = 1 << pbits
    p_lo, p_hi = owned(F, world, rank, used)
    lbits = ceil_log2(max(p_hi - p_lo, 1))
    s1 = plan_shift(key_min, key_max, pbits)
    key_lo = key_min + (p_lo << s1)
    key_hi = key_lo + (1 << (s1 + lbits - 1)) if lbits else key_lo + (1 << s1) - 1
    # with fewer keys than partitions (s1 = 0) the top partitions hold no key:
    # a narrower local range keeps s1 = 0 and stays inside int64
    top = key_min + (1 << L) - 1
    key_lo, key_hi = min(key_lo, top), min(key_hi, top)
    return key_min, key_lo, key_hi, lbits


def send_counts(hist: torch.Tensor, world: int, used: int | None = None) -> torch.Tensor:
    """Rows this rank sends to every rank: per-partition counts summed by owner."""
    own = owners(hist.numel(), world, used).to(hist.device)
    out = torch.zeros(world, dtype=torch.int64, device=hist.device)
    return out.index_add_(0, own, hist.to(torch.int64))


HEAD = 4  # message header: chunk size, used elements, flag0 (not packable), flag1 (overflow)


def xsend_torch(start, cnt, flags, world, msg, chunk, used=0):
    """smj_dev_xsend in framework ops (the CPU stand-ins use it; the GPU test
    compares the kernel with it): the message to every rank, rank after rank,
    [chunk size, used, not packable, overflow, owned regions' offsets in the
    chunk, counts], and chunk = [chunk starts | chunk sizes].  flags: int32
    [region overflow, not packable] as the sampled partition writes them."""
    F, K = start.shape
    G = world
    u = used or F
    dev = start.device
    own = owners(F, G, u).to(dev)
    lo_of = torch.tensor([owned(F, G, g, u)[0] for g in range(G)], dtype=torch.int64, device=dev)
    cstart = start[lo_of, 0]
    cend = (start + cnt).max()
    csize = torch.cat([cstart[1:], cend.view(1)]) - cstart
    used = torch.zeros(G, dtype=torch.int64, device=dev).index_add_(0, own, cnt.sum(1))
    rel_start = torch.where(cnt > 0, start - cstart[own].view(F, 1), 0)
    parts = []
    for g in range(G):
        lo, hi = owned(F, G, g, u)
        parts += [torch.stack([csize[g], used[g], flags[1].to(torch.int64),
                               flags[0].to(torch.int64)]),
                  rel_start[lo:hi].reshape(-1), cnt[lo:hi].reshape(-1)]
    msg.copy_(torch.cat(parts))
    chunk[:G] = cstart
    chunk[G:] = csize


def xrecv_torch(msg, chunk, world, rank, mine, K, tstart, tcnt, cap, summary):
    """smj_dev_xrecv in framework ops: the local join's segment tables (own
    chunk in place, the other ranks' rows from `cap` on, rank order) and the
    summary [chunk starts | sizes | receive sizes | used received | the
    flags OR-ed over the ranks]."""
    G = world
    m = msg.view(G, HEAD + 2 * mine * K)
    rl = m[:, 0].tolist()
    base, ro = [], cap
    for s in range(G):
        base.append(int(chunk[rank]) if s == rank else ro)
        ro += 0 if s == rank else rl[s]
    bt = torch.tensor(base, dtype=torch.int64, device=msg.device)
    rs = m[:, HEAD:HEAD + mine * K].view(G, mine, K) + bt.view(G, 1, 1)
    rc = m[:, HEAD + mine * K:].view(G, mine, K)
    tstart.zero_()
    tcnt.zero_()
    tstart[:mine] = rs.permute(1, 0, 2).reshape(mine, G * K)
    tcnt[:mine] = rc.permute(1, 0, 2).reshape(mine, G * K)
    summary[:2 * G] = chunk
    summary[2 * G:3 * G] = m[:, 0]
    summary[3 * G:4 * G] = m[:, 1]
    fl = m[:, 2:HEAD]  # bit masks: OR-ed over the ranks (every rank's reasons)
    acc = fl[0].clone()
    for g in range(1, G):
        acc |= fl[g]
    summary[4 * G:4 * G + 2] = acc


class DeviceOps:
    """The device implementation of the ops interface (libsmj_hip*.so).
    pack: 16-byte tuples may travel as packed 64-bit words
    (smj_dev_partition_range_packed); planes: both widths as 48-bit words in
    two planes (a sampled form only); sampled: the exchange partition's form,
    None = sampled on one rank, exact across ranks (see can_sample)."""

    def __init__(self, lib, pack=True, planes=True, sampled=None):
        self.lib = lib
        self.can_pack = lib.width == 16 and pack
        self.can_planes = planes and sampled is not False
        self._sampled = sampled

    def empty(self, n):
        return self.lib.empty(n)

    def empty_words(self, n):
        return torch.empty(max(n, 1), dtype=torch.int64, device="cuda")[:n]

    def partition_range(self, inp, out, nbits, key_min, key_max, hist):
        self.lib.dev_partition_range(inp, out, nbits, key_min, key_max, hist)

    def partition_range_packed(self, inp, out_words, nbits, key_min, key_max, hist, bad):
        return self.lib.dev_partition_range_packed(inp, out_words, nbits, key_min, key_max,
                                                   hist, bad)

    def join_segmented(self, R, segR, S, segS, bucket_bits, key_lo, key_hi, sR, sS, count,
                       packed=False):
        self.lib.dev_join_segmented(R, segR, S, segS, bucket_bits, key_lo, key_hi,
                                    sR, sS, count, packed=packed)

    # the sampled exchange partition (smj_dev_partition_range_sampled): the
    # 1-GPU join's level-1 scatter, no histogram pass, but every region keeps
    # slack (9/8 of its estimate + 1024 elements per shard) that travels with
    # the rows.  On one rank nothing travels and it is the faster form (5.98
    # -> 5.17 ms at N=1, round 2); across ranks the slack is ~14-19 % more
    # xGMI bytes against one HBM read saved, so there the exact partition is
    # the default.  DeviceOps(sampled=True/False) forces either.
    def can_sample(self, world=1):
        return world == 1 if self._sampled is None else bool(self._sampled)

    def shards(self):
        return self.lib.sampled_shards()

    def sampled_capacity(self, n, nbits):
        return self.lib.sampled_capacity(n, nbits)

    def partition_range_sampled(self, inp, out, nbits, key_min, key_max, packed, seg_start,
                                seg_cnt, flags):
        return self.lib.dev_partition_range_sampled(inp, out, nbits, key_min, key_max, packed,
                                                    seg_start, seg_cnt, flags)

    def partition_range_shards(self, inp, out, nbits, key_min, key_max, packed, seg_start,
                               seg_cnt, flags):
        return self.lib.dev_partition_range_shards(inp, out, nbits, key_min, key_max, packed,
                                                   seg_start, seg_cnt, flags)

    def partition_range_planes(self, inp, out, nbits, key_min, key_max, seg_start, seg_cnt,
                               flags):
        return self.lib.dev_partition_range_planes(inp, out.buf, out.stride, nbits, key_min,
                                                   key_max, seg_start, seg_cnt, flags)

    def join_segmented_tables(self, R, nR, startR, cntR, S, nS, startS, cntS, bucket_bits,
                              key_lo, key_hi, sR, sS, count, packed=False, stage=None):
        if isinstance(R, Planes):
            self.lib.dev_join_segmented_planes(R.buf, R.stride, nR, startR, cntR, S.buf,
                                               S.stride, nS, startS, cntS, bucket_bits,
                                               key_lo, key_hi, sR, sS, count, stage=stage)
            return
        self.lib.dev_join_segmented_tables(R, nR, startR, cntR, S, nS, startS, cntS,
                                           bucket_bits, key_lo, key_hi, sR, sS, count,
                                           packed=packed, stage=stage)

    def xsend(self, start, cnt, flags, world, msg, chunk, used=0):
        self.lib.dev_xsend(start, cnt, flags, world, msg, chunk, used)

    def xrecv(self, msg, chunk, world, rank, mine, K, tstart, tcnt, cap, summary):
        self.lib.dev_xrecv(msg, chunk, world, rank, mine, K, tstart, tcnt, cap, summary)


# The row exchange's own communicator per process group (a second RCCL
# communicator over the same ranks, so R's rows are not queued behind S's
# table exchange): created once per group and shared by every DistributedJoin
# on it.  new_group with use_local_synchronization involves only the group's
# members, so a join built on a sub-group does not need the ranks outside it.
_ROW_GROUPS = {}


def _row_group(group, ranks):
    key = (id(group) if group is not None else None, tuple(ranks))
    g = _ROW_GROUPS.get(key)
    if g is None:
        g = dist.new_group(ranks=ranks, use_local_synchronization=True)
        _ROW_GROUPS[key] = g
    return g


def release_row_groups():
    """Destroy the cached row communicators (before destroy_process_group,
    or when the groups they mirror go away)."""
    for g in _ROW_GROUPS.values():
        dist.destroy_process_group(g)
    _ROW_GROUPS.clear()


class DistributedJoin:
    """One process per device; `step` joins the local slices of R and S
    against the slices on all other ranks and leaves the GLOBAL match count in
    `count` on every rank.  `bucket_bits`: level-1 buckets per rank (2^9 =
    512, what the 1-GPU join uses); `n_hint`: elements per rank and relation,
    identical on every rank (lets the 48-bit planes take 2^9 partitions
    across ranks, partition_bits); `row_group`: the communicator the rows
    travel on (default: one per `group`, cached, see _row_group); `staged`:
    the local join in two calls overlapping S's rows (False: one call);
    `pbits`: force the exchange partition width."""

    def __init__(self, ops, bucket_bits: int, key_min: int, key_max: int,
                 group=None, n_hint=None, row_group=None, staged=True, pbits=None):
        self.ops = ops
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        offers_planes = (bool(getattr(ops, "can_planes", False))
                         and hasattr(ops, "partition_range_planes"))
        # n_hint: elements per rank and relation (the same on every rank)
        self.pbits = partition_bits(bucket_bits, self.world, offers_planes, n_hint,
                                    (key_min, key_max))
        if pbits is not None:  # rehearse the G-GPU partition width on fewer ranks
            self.pbits = pbits
        self.fanout = 1 << self.pbits
        if self.fanout < self.world:
            raise ValueError(f"fanout 2^{self.pbits} < world size {self.world}")
        self.key_min, self.key_lo, self.key_hi, self.lbits = local_range(
            key_min, key_max, self.pbits, self.world, self.rank)
        self.key_max = key_max
        F, G = self.fanout, self.world
        # the partitions the key range reaches, split evenly (owners)
        self.used = used_parts(key_min, key_max, self.pbits)
        self.per_rank = [owned(F, G, g, self.used)[1] - owned(F, G, g, self.used)[0]
                         for g in range(G)]
        self.p_lo, self.p_hi = owned(F, G, self.rank, self.used)
        cs = getattr(ops, "can_sample", False)
        self.sampled = bool(cs(self.world) if callable(cs) else cs)
        # the first layout tried each step: the narrowest the ops offer
        self.can_pack = bool(getattr(ops, "can_pack", False))
        self.can_planes = (offers_planes and self.pbits <= PLANE_MAX_BITS
                           and planes_hold(self.key_min, self.key_max, self.pbits))
        self.layout = "planes" if self.can_planes else "words" if self.can_pack else "tuples"
        # segment-table width: the same on every rank whichever form a rank's
        # partition takes
        self.shards = ops.shards() if hasattr(ops, "shards") else 1
        self.buf = {}
        # the local join in two calls overlapping S's rows (staged=False: one)
        self.staged = staged
        # the rows travel on a communicator of their own: its stream is not
        # ordered behind the table exchange of S (queued behind S's partition)
        self.row_group = row_group
        if self.world > 1 and row_group is None:
            self.row_group = _row_group(group, [self._global(g) for g in range(self.world)])
        self.recv_hint = {}  # remote rows received per relation and layout (sticky)
        self.last_recv = {}
        self.last_rows = {}
        self.last_layout = "tuples"  # the layout of the last step's exchange
        self.last_packed = False  # ... not tuples
        self.stats_reset()

    def stats_reset(self):
        """Exchange statistics since the last reset: bytes this rank sent to
        other ranks, steps, and (GPU) the time of S's row exchange -- from
        its issue to its completion, with nothing else queued behind it."""
        self.stats = {"steps": 0, "sent_B": 0, "recv_B": 0, "gap_B": 0, "xS_ms": 0.0}
        self._ev = []

    def _grow(self, key, n, words=False):
        b = self.buf.get(key)
        if b is None or b.shape[0] < n:
            b = (self.ops.empty_words if words else self.ops.empty)(max(n, 1))
            self.buf[key] = b
        return b[:n]

    def _xbuf(self, key, need, lay, keep=0, dev=None):
        """The exchange buffer of one relation: the rank's own partition (its
        first `cap` elements) followed by the rows received from the other
        ranks, so the local join reads the rank's own rows in place.  Grows
        (sticky across steps) to `need` elements, keeping the first `keep`."""
        b = self.buf.get(key)
        if lay == "planes":
            if b is None or b.stride < need:
                nb = Planes(-(-max(need, 1) // 32) * 32, device=dev)
                if b is not None and keep:
                    for p, q in zip(nb.planes, b.planes):
                        p[:keep].copy_(q[:keep])
                self.buf[key] = b = nb
            return b
        if b is None or b.shape[0] < need:
            nb = (self.ops.empty_words if lay == "words" else self.ops.empty)(max(need, 1))
            if b is not None and keep:
                nb[:keep].copy_(b[:keep])
            self.buf[key] = b = nb
        return b

    def _small(self, key, shape, dtype=torch.int64, dev=None):
        """A small per-relation table, allocated once (reused every step)."""
        t = self.buf.get(key)
        if t is None or t.shape != torch.Size(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=dev)
            self.buf[key] = t
        return t

    def _partition(self, rel, part, packed):
        """Exact range partition of `rel` into `part` (packed words or tuples),
        partitions back to back.  Returns (per-partition start (F, K) and
        count (F, K) with only shard 0 used, flags int32 [overflow (0), not
        packable]), or None when packed words do not apply at all."""
        dev = rel.device
        F, K = self.fanout, self.shards
        hist = torch.zeros(F, dtype=torch.int64, device=dev)
        flags = torch.zeros(2, dtype=torch.int32, device=dev)
        if packed:
            if not self.ops.partition_range_packed(rel, part, self.pbits, self.key_min,
                                                   self.key_max, hist, flags[1:]):
                return None
        else:
            self.ops.partition_range(rel, part, self.pbits, self.key_min, self.key_max, hist)
        start = torch.zeros(F, K, dtype=torch.int64, device=dev)
        cnt = torch.zeros(F, K, dtype=torch.int64, device=dev)
        start[:, 0] = torch.cumsum(hist, 0) - hist
        cnt[:, 0] = hist
        return start, cnt, flags

    def _sampled(self, rel, part, packed, key):
        """Sampled range partition into `part` (no histogram pass): partition
        p is K consecutive shard regions with slack after each.  Returns
        (start (F, K), count (F, K), flags int32 [overflow, not packable],
        zeroed by the partition), or None when the form does not apply."""
        dev = rel.device
        F, K = self.fanout, self.shards
        ss = self._small("ss" + key, (F * K,), dev=dev)
        sc = self._small("sc" + key, (F * K,), dev=dev)
        flags = self._small("fl" + key, (2,), torch.int32, dev)
        if not self.ops.partition_range_sampled(rel, part, self.pbits, self.key_min,
                                                self.key_max, packed, ss, sc, flags):
            return None
        return ss.view(F, K), sc.view(F, K), flags

    def _shards(self, rel, part, packed, key):
        """The exact partition across ranks (round 6): the sampled scatter
        with exactly sized regions back to back (smj_dev_partition_range_shards:
        one count pass, no slack to travel), tables in the sampled shape.
        None when the ops have no such form or it does not apply."""
        if not hasattr(self.ops, "partition_range_shards"):
            return None
        dev = rel.device
        F, K = self.fanout, self.shards
        ss = self._small("ss" + key, (F * K,), dev=dev)
        sc = self._small("sc" + key, (F * K,), dev=dev)
        flags = self._small("fl" + key, (2,), torch.int32, dev)
        if not self.ops.partition_range_shards(rel, part, self.pbits, self.key_min,
                                               self.key_max, packed, ss, sc, flags):
            return None
        return ss.view(F, K), sc.view(F, K), flags

    def _planes(self, rel, xb, key):
        """Sampled range partition of `rel` into the planes `xb` (48-bit
        words); where the form does not apply on this rank, empty tables
        flagged BAD_PAYLOAD48, so that every rank drops the layout together."""
        dev = rel.device
        F, K = self.fanout, self.shards
        ss = self._small("ss" + key, (F * K,), dev=dev)
        sc = self._small("sc" + key, (F * K,), dev=dev)
        flags = self._small("fl" + key, (2,), torch.int32, dev)
        if not self.ops.partition_range_planes(rel, xb, self.pbits, self.key_min,
                                               self.key_max, ss, sc, flags):
            ss.zero_()
            sc.zero_()
            flags[0] = 0
            flags[1] = BAD_PAYLOAD48
        return ss.view(F, K), sc.view(F, K), flags

    def _attempt(self, rel, key, lay, sampled):
        """Enqueue one exchange attempt of `rel`: its range partition (sampled
        or exact; tuples, packed words, or 48-bit planes -- always sampled),
        the table messages (device), their all-to-all and the receive tables,
        and an asynchronous copy of the small summary the host needs.
        Returns the attempt's state (nothing has been waited for), or None
        when packed words do not apply at all."""
        G, me = self.world, self.rank
        dev = rel.device
        F, K = self.fanout, self.shards
        n = rel.shape[0]
        mine = self.p_hi - self.p_lo
        nb = 1 << self.lbits
        sampled = sampled or lay == "planes"
        xkey = {"tuples": "xt", "words": "xw", "planes": "xp"}[lay] + key
        cap = self.ops.sampled_capacity(n, self.pbits) if sampled else n
        # room for the remote rows: last step's, else an even share + 1/8
        extra = self.recv_hint.get(xkey, (cap * (G - 1)) // G + cap // 8 if G > 1 else 0)
        xb = self._xbuf(xkey, cap + extra, lay, dev=dev)
        if lay == "planes":
            res = self._planes(rel, xb, key)
        else:
            packed = lay == "words"
            part = xb[:cap]
            res = self._sampled(rel, part, packed, key) if sampled else None
            if res is None:  # exact partition (the receivers read either form)
                cap = n if sampled else cap
                res = self._shards(rel, part[:n], packed, key)
                if res is None:
                    res = self._partition(rel, part[:n], packed)
                if res is None:
                    return None
        start, cnt, fl = res
        xsend = getattr(self.ops, "xsend", xsend_torch)
        xrecv = getattr(self.ops, "xrecv", xrecv_torch)
        msg_len = sum(HEAD + 2 * K * m for m in self.per_rank)
        inp = self._small("xin" + key, (msg_len,), dev=dev)
        chunk = self._small("xch" + key, (2 * G,), dev=dev)
        tstart = self._small("xts" + key, (nb, G * K), dev=dev)
        tcnt = self._small("xtc" + key, (nb, G * K), dev=dev)
        # [4 G + 2]: the largest row message of any rank (all_to_all rounds)
        summary = self._small("xsm" + key, (4 * G + 3,), dev=dev)
        xsend(start, cnt, fl, G, inp, chunk, self.used)
        if G == 1:
            msg = inp
        else:
            per_in = [HEAD + 2 * m * K for m in self.per_rank]
            msg = self._small("xmsg" + key, (G * (HEAD + 2 * mine * K),), dev=dev)
            dist.all_to_all_single(msg, inp, [HEAD + 2 * mine * K] * G, per_in,
                                   group=self.group)
        xrecv(msg, chunk, G, me, mine, K, tstart, tcnt, cap, summary)
        # every rank must run the same number of row all-to-all rounds (one
        # rank: no rows travel, the entry stays unread)
        if G > 1:
            summary[4 * G + 2:] = summary[G:3 * G].max()
            dist.all_reduce(summary[4 * G + 2:], op=dist.ReduceOp.MAX, group=self.group)
        if summary.is_cuda:
            hs = self.buf.get("xhost" + key)
            if hs is None or hs.shape != summary.shape:
                hs = torch.empty(summary.shape, dtype=torch.int64, pin_memory=True)
                self.buf["xhost" + key] = hs
            hs.copy_(summary, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            hs, ev = summary, None
        return dict(key=key, xkey=xkey, xb=xb, cap=cap, lay=lay, sampled=sampled,
                    tstart=tstart, tcnt=tcnt, host=hs, ev=ev, dev=dev)

    def _next_layout(self, lay, sampled, bad, ovf):
        """The layout and form an invalid attempt repeats with, on every rank
        alike (bad and ovf are OR-ed over the ranks): a region overflow ->
        exact partitions (planes have no exact form: words, else tuples);
        a payload too wide for 48 bits -> words; anything else unpackable ->
        tuples."""
        if lay == "planes":
            wide_only = bad and not bad & (BAD_PAYLOAD | BAD_RANGE)
            lay = "words" if self.can_pack and (wide_only or not bad) else "tuples"
            return lay, self.sampled and not ovf
        if lay == "words" and bad:
            lay = "tuples"
        return lay, sampled and not ovf

    def _finish(self, rel, st):
        """Wait for an attempt's summary; repeat the attempt until every rank
        agrees it is valid (a sampled region overflow anywhere -> every rank
        partitions exactly; an unpackable tuple anywhere -> every rank takes
        a wider layout), then start its row exchange.  Returns (exchange
        buffer, start and count tables (2^lbits, world * K) for the local
        join, elements inside the segments, async work, layout)."""
        G, me = self.world, self.rank
        key = st["key"] if st is not None else None
        while True:
            if st is not None:
                if st["ev"] is not None:
                    st["ev"].synchronize()
                host = st["host"].tolist()
                cs, sl, rl, ru = host[:G], host[G:2 * G], host[2 * G:3 * G], host[3 * G:4 * G]
                bad, ovf, gmax = host[4 * G:]
                if G == 1:  # not computed on one rank (no rows travel)
                    gmax = max(sl[0], rl[0])
                if not ovf and not (st["lay"] != "tuples" and bad):
                    break
                lay, sampled = self._next_layout(st["lay"], st["sampled"], bad, ovf)
            else:  # packed words did not apply at all: tuples, on every rank
                lay, sampled = "tuples", self.sampled
            st = self._attempt(rel, key, lay, sampled)
        xkey, cap = st["xkey"], st["cap"]
        remote = sum(rl) - rl[me]
        self.recv_hint[xkey] = max(remote, self.recv_hint.get(xkey, 0))
        xb = self._xbuf(xkey, cap + remote, st["lay"], keep=cap, dev=st["dev"])
        grown = xb is not st["xb"]
        row = row_bytes(xb)
        self.stats["sent_B"] += row * (sum(sl) - sl[me])
        self.stats["recv_B"] += row * remote
        self.stats["gap_B"] += row * (sum(rl) - sum(ru))
        ev = None
        if xb.is_cuda:
            # the rows are issued from a stream that waits only for this
            # attempt (partition, tables, summary), not for work queued after
            # it (the other relation's partition); a grown buffer's copy of
            # the partition is on the current stream
            rs = self._row_stream()
            if grown:
                rs.wait_stream(torch.cuda.current_stream())
            else:
                rs.wait_event(st["ev"])
            with torch.cuda.stream(rs):
                if key == "S":
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                work = self._rows(xb, cap, cs, sl, rl, gmax)
        else:
            work = self._rows(xb, cap, cs, sl, rl, gmax)
        self.last_recv[key] = (sl, rl)
        self.last_rows[key] = (xb, cap, cs, sl, rl, gmax)  # bench.py --op exchange repeats it
        self._ev_issue = ev
        return xb, st["tstart"], st["tcnt"], sum(ru), work, st["lay"]

    def _exchange(self, rel, key, lay=None):
        """One relation's exchange in `lay` (default: the first layout) or a
        wider one: attempt, wait, start the rows."""
        st = self._attempt(rel, key, lay or self.layout, self.sampled)
        if st is None:
            st = self._attempt(rel, key, "tuples", self.sampled)
        return self._finish(rel, st)

    def _rows(self, xb, cap, cs, sl, rl, gmax=None):
        """Asynchronous row exchange: rank g gets this rank's chunk
        xb[cs[g], cs[g] + sl[g]), the rows from the other ranks land after the
        partition (xb[cap:], in rank order); this rank's own chunk stays where
        it is.  Over RCCL: list all-to-alls on the group's communicator (self
        empty), in rounds of at most CHUNK_BYTES per peer (the RCCL message
        limit above; `gmax`, the largest message of any rank, fixes the
        number of rounds on every rank); elsewhere (gloo) one batch of
        point-to-point pairs."""
        me, G = self.rank, self.world
        if G == 1:
            return _Works([])
        # planes: the same element ranges of each plane, one transfer each
        planes = xb.planes if isinstance(xb, Planes) else (xb,)
        row = max(row_bytes(p) for p in planes)
        step = max(CHUNK_BYTES // row, 1)
        ro, roff = cap, []
        for g in range(G):
            roff.append(ro)
            ro += 0 if g == me else rl[g]
        if xb.is_cuda and dist.get_backend(self._rgroup()) == "nccl":
            if gmax is None:
                raise ValueError("the RCCL row exchange needs the global message maximum")
            rounds = -(-gmax // step)
            works = []
            for k in range(max(rounds, 1)):
                lo = k * step
                for p in planes:
                    def piece(start, n, g):
                        if g == me or lo >= n:
                            return _wire(p[:0])
                        return _wire(p[start + lo:start + min(lo + step, n)])
                    ins = [piece(cs[g], sl[g], g) for g in range(G)]
                    outs = [piece(roff[g], rl[g], g) for g in range(G)]
                    works.append(dist.all_to_all(outs, ins, group=self._rgroup(),
                                                 async_op=True))
            return _Works(works)
        ops = []
        for g in range(G):
            if g == me:
                continue
            peer = self._global(g)
            for p in planes:
                for k in range(0, sl[g], step):
                    ops.append(dist.P2POp(dist.isend, p[cs[g] + k:cs[g] + min(k + step, sl[g])],
                                          peer, group=self._rgroup()))
                for k in range(0, rl[g], step):
                    ops.append(dist.P2POp(dist.irecv,
                                          p[roff[g] + k:roff[g] + min(k + step, rl[g])],
                                          peer, group=self._rgroup()))
        return _Works(dist.batch_isend_irecv(ops) if ops else [])

    def _global(self, g):
        return g if self.group is None else dist.get_global_rank(self.group, g)

    def _rgroup(self):
        return self.row_group if self.row_group is not None else self.group

    def _row_stream(self):
        s = self.buf.get("_rows")
        if s is None:
            s = self.buf["_rows"] = torch.cuda.Stream()
        return s

    def step(self, R, S, count):
        """One join step.  Both relations' attempts (partition, table
        exchange, summary copy) are queued before the first host wait, so the
        device partitions S while the host reads R's summary; R's rows then
        leave at once (their own stream and communicator, ordered only after
        R's attempt, so they overlap S's partition), S's rows after S's
        summary.  The local join runs in two calls: R's tile stage as soon as
        R's rows are in (overlapping S's rows in flight), then S's tile stage,
        the group pass and the count (smj_dev_join_segmented_tables,
        SMJ_SEG_STAGE_R / _REST).  One rank: no rows travel, one call."""
        aR = self._attempt(R, "R", self.layout, self.sampled)
        if aR is None:
            aR = self._attempt(R, "R", "tuples", self.sampled)
        aS = self._attempt(S, "S", self.layout, self.sampled)
        if aS is None:
            aS = self._attempt(S, "S", "tuples", self.sampled)
        if self.world == 1:
            done = self._one_rank(aR, aS, count)
            if done is not None:
                return done
        rR, tR, cR, nR, wR, pR = self._finish(R, aR)
        rS, tS, cS, nS, wS, pS = self._finish(S, aS)
        eS = self._ev_issue
        # both relations must reach the local join in one layout: the one
        # that went out narrower is exchanged again in the other's
        while pR != pS:
            if LAYOUTS.index(pR) > LAYOUTS.index(pS):
                wR.wait()
                rR, tR, cR, nR, wR, pR = self._exchange(R, "R", pS)
            else:
                wS.wait()
                rS, tS, cS, nS, wS, pS = self._exchange(S, "S", pR)
                eS = self._ev_issue
        self.last_layout = pR
        self.last_packed = pR != "tuples"
        if eS is not None:
            # S's row exchange alone: its completion on a stream of its own
            # (the compute stream runs R's tile stage meanwhile)
            side = self._side_stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                wS.wait()
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
            self._ev.append((eS, e1))
        self.stats["steps"] += 1
        sR = self._grow("sortR", nR)
        sS = self._grow("sortS", nS)
        args = (rR, nR, tR, cR, rS, nS, tS, cS, self.lbits, self.key_lo, self.key_hi, sR, sS,
                count)
        if self.world > 1 and self.staged:
            wR.wait()
            self.ops.join_segmented_tables(*args, packed=pR == "words", stage="R")
            wS.wait()
            self.ops.join_segmented_tables(*args, packed=pR == "words", stage="REST")
        else:
            wR.wait()
            wS.wait()
            self.ops.join_segmented_tables(*args, packed=pR == "words")
        if self.world > 1:
            dist.all_reduce(count, group=self.group)
        return sR, sS

    def _one_rank(self, aR, aS, count):
        """One rank, both attempts valid in one layout (the usual case): no
        rows travel, so the local join is issued right after the summaries
        arrive, without the row streams and events of the general path.
        Returns None (nothing issued) otherwise."""
        hs = []
        for st in (aR, aS):
            if st["ev"] is not None:
                st["ev"].synchronize()
            h = st["host"].tolist()
            bad, ovf = h[4], h[5]
            if ovf or (st["lay"] != "tuples" and bad):
                return None
            hs.append(h)
        if aR["lay"] != aS["lay"]:
            return None
        lay = aR["lay"]
        nR, nS = hs[0][3], hs[1][3]  # elements inside the segments
        sR = self._grow("sortR", nR)
        sS = self._grow("sortS", nS)
        self.ops.join_segmented_tables(aR["xb"], nR, aR["tstart"], aR["tcnt"], aS["xb"], nS,
                                       aS["tstart"], aS["tcnt"], self.lbits, self.key_lo,
                                       self.key_hi, sR, sS, count, packed=lay == "words")
        self.last_layout = lay
        self.last_packed = lay != "tuples"
        for st, h in zip((aR, aS), hs):
            self.last_recv[st["key"]] = ([h[1]], [h[2]])
            self.last_rows[st["key"]] = (st["xb"], st["cap"], [h[0]], [h[1]], [h[2]],
                                         max(h[1], h[2]))
            self.stats["gap_B"] += row_bytes(st["xb"]) * (h[2] - h[3])
        self.stats["steps"] += 1
        return sR, sS

    def _side_stream(self):
        s = self.buf.get("_side")
        if s is None:
            s = self.buf["_side"] = torch.cuda.Stream()
        return s

    def stats_read(self):
        """The statistics with S's exchange time summed (synchronises)."""
        for a, b in self._ev:
            b.synchronize()
            self.stats["xS_ms"] += a.elapsed_time(b)
        self._ev = []
        return dict(self.stats)
