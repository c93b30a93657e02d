"""Striping one hwlmExec block across ranks.

HWLM literals are at most 8 bytes (hwlm.h:75, HWLM_MASKLEN 8), so a match
ending at e depends only on bytes [e-7, e].  Rank r owns the end positions
[lo_r, hi_r) of the block and scans the window [lo_r - 7, hi_r) as its own
block (start 0, or the block's `start` mapped into the window); matches that
end in the 7-byte halo belong to rank r-1 and are dropped.  Every owned end
sees the same bytes, the same first-stage lookups (the window's lookups begin
at or before lo_r - 7 >= the block's start) and the same confirm key as in
the one-GPU scan, so the union over ranks is exactly the single-block match
set, already in rank = end order.  No data-path collective: the only
exchange is gathering the (small) match lists to rank 0, which then runs the
sequential host replay (NOREPEAT, groups, terminate) in global order.

The gathers use torch.distributed (RCCL over xGMI with backend "nccl" and
device tensors; gloo with CPU tensors in the tests): one all_gather of the
per-rank counts, then the records padded to the largest count
(gather_matches: all_gather of host lists; gather_to_root: dist.gather of
device tensors to one rank; PackedGather: bench.py's per-step exchange,
packed on the device, headers all-gathered, records gathered to the root).
"""
from dataclasses import dataclass

import numpy as np

HALO = 7  # max literal length (8) - 1


@dataclass
class Stripe:
    rank: int
    wlo: int     # window start (block-relative)
    wlen: int    # window length
    wstart: int  # hwlmExec start inside the window
    own_lo: int  # first owned end (block-relative)
    own_hi: int  # one past the last owned end


def plan_block_stripes(length, start, world, min_stripe=1 << 16):
    """Split one block of `length` bytes (hwlmExec start `start`) into
    `world` stripes.  Blocks too short to split (or with a short first zone,
    fdr.c:712-720) go to rank 0 whole.  Returns one Stripe per rank (empty
    stripes have own_lo == own_hi)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    out = []
    if length - start <= max(16, min_stripe) or world == 1:
        for r in range(world):
            if r == 0:
                out.append(Stripe(0, 0, length, start, start, length))
            else:
                out.append(Stripe(r, length, 0, 0, length, length))
        return out
    span = length - start
    cuts = [start + (span * r) // world for r in range(world + 1)]
    for r in range(world):
        lo, hi = cuts[r], cuts[r + 1]
        wlo = 0 if r == 0 else max(0, lo - HALO)
        wstart = start if r == 0 else max(start - wlo, 0)
        out.append(Stripe(r, wlo, hi - wlo, wstart, lo, hi))
    return out


@dataclass
class Window:
    block: int   # block index (one hs_scan / hwlmExec call each)
    wlo: int     # window start, global corpus offset
    wlen: int    # window length
    rlo: int     # first reported end inside the window (report_lo)


def plan_corpus_stripes(total, block_len, world, align=1 << 16):
    """North-star striping: one corpus of `total` bytes made of
    blocks of `block_len` bytes (the last may be shorter), its end positions
    split into `world` contiguous ranges (cut at multiples of `align`).  Rank r
    owns ends [cut_r, cut_{r+1}); for every block it overlaps it scans the
    window [max(block_lo, lo - 7), hi) as that block's own scan from 0 and
    reports ends >= lo only (vsa_scan_blocks_ex report_lo): exact, because
    literals are <= 8 bytes (hwlm.h:75) and the FDR start state only touches
    a block's first 7 ends.  Returns (cuts, [[Window, ...] per rank])."""
    if world < 1 or block_len < 1:
        raise ValueError("world and block_len must be >= 1")
    cuts = [min(total, ((total * r) // world) // align * align) for r in range(world)]
    cuts.append(total)
    plan = []
    for r in range(world):
        lo, hi = cuts[r], cuts[r + 1]
        wins = []
        b = lo // block_len
        while lo < hi and b * block_len < hi:
            blo, bhi = b * block_len, min(total, (b + 1) * block_len)
            olo, ohi = max(lo, blo), min(hi, bhi)
            if olo < ohi:
                wlo = blo if olo == blo else max(blo, olo - HALO)
                wins.append(Window(b, wlo, ohi - wlo, olo - wlo))
            b += 1
        plan.append(wins)
    return cuts, plan


def localize(stripe, ends, ids):
    """Window-relative results -> block-relative, halo ends dropped."""
    ends = np.asarray(ends, np.int64) + stripe.wlo
    ids = np.asarray(ids, np.int64)
    keep = (ends >= stripe.own_lo) & (ends < stripe.own_hi)
    return ends[keep], ids[keep]


def gather_matches(dist, ends, ids, device=None):
    """all_gather the per-rank (end, id) lists; every rank gets the merged,
    end-ordered list (ranks own increasing end ranges).  `dist` is
    torch.distributed; `device` the tensor device for the collective
    (a cuda device for RCCL, None = CPU for gloo)."""
    import torch
    world = dist.get_world_size()
    n = torch.tensor([len(ends)], dtype=torch.int64, device=device)
    counts = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    rec = torch.zeros((max(m, 1), 2), dtype=torch.int64, device=device)
    if len(ends):
        rec[:len(ends), 0] = torch.as_tensor(np.asarray(ends, np.int64), device=device)
        rec[:len(ends), 1] = torch.as_tensor(np.asarray(ids, np.int64), device=device)
    bufs = [torch.zeros_like(rec) for _ in range(world)]
    dist.all_gather(bufs, rec)
    parts = [b[:c].cpu().numpy() for b, c in zip(bufs, counts)]
    allrec = np.concatenate(parts) if parts else np.zeros((0, 2), np.int64)
    return allrec[:, 0], allrec[:, 1]


def scan_block_striped(ctx, db, d_window, stripe):
    """Scan this rank's window (device buffer holding the window bytes) and
    return block-relative (ends, ids) of its owned ends, in reference order
    (end, bucket, chain) before replay."""
    if stripe.wlen == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    n = ctx.scan_blocks(db, d_window, [0], [stripe.wlen], [stripe.wstart])
    res = ctx.results(n)
    ends = (res["key"] >> np.uint64(24)).astype(np.int64)
    return localize(stripe, ends, res["id"])


def gather_to_root(dist, keys, ids, n, root=0):
    """Gather the first n rows of this rank's (keys, ids) tensors to `root`
    (one all_gather of the counts, one gather per array, padded to the
    largest count).  Returns (keys, ids) concatenated in rank order on root,
    None elsewhere.  Works on device tensors with the nccl (RCCL) backend
    and on CPU tensors with gloo."""
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    cnt = torch.tensor([n], dtype=torch.int64, device=keys.device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    m = max(max(counts), 1)
    out = []
    for t in (keys, ids):
        send = t[:m] if t.shape[0] >= m else torch.cat(
            [t, torch.zeros(m - t.shape[0], dtype=t.dtype, device=t.device)])
        recv = [torch.empty_like(send) for _ in range(world)] if rank == root else None
        dist.gather(send.contiguous(), recv, dst=root)
        if rank == root:
            out.append(torch.cat([r[:c] for r, c in zip(recv, counts)]))
    return tuple(out) if rank == root else None


NOT_READY = 1 << 62  # packed header bit: the records are not usable as packed


class PackedGather:
    """bench.py's per-step exchange, with no host count read before it.

    Every rank packs its sorted records into an int64 buffer
    ``[header | keys (cap) | ids (cap int32)]`` (header = the record count,
    bit 62 set when the records are not final, e.g. the scan overflowed its
    output; on the GPU ``vsa_scan_pack`` queues this behind the scan, on the
    device).  Then ONE all-gather of the 8-byte headers and ONE gather of
    the packed buffers to the root, both queued before the host looks at
    anything.  The host reads the gathered headers after that (every rank,
    so all agree): when some rank's records did not fit ``cap`` or were not
    final, ``cap`` grows to 1.25x the largest count (at least 1,024) and
    the pack and both collectives run once more.

    ``pack(buf, cap)`` fills this rank's buffer; ``wait()``, if given, runs
    between the pack and the collectives (bench.py: the collective stream
    waits on the scan context's stream); ``complete()``, if given, runs
    after the collectives are queued (bench.py: the rank's own scan is
    completed, which performs any output-overflow rescan, so a repeated
    pack is final).  Device tensors use RCCL, CPU tensors gloo (tests);
    gloo with a device (the one-GPU rehearsal of bench.py's N > 1 path)
    packs on the device and runs the collectives on host copies."""

    def __init__(self, dist, world, device=None, root=0):
        self.dist, self.world, self.device, self.root = dist, world, device, root
        self.rank = dist.get_rank()
        self.stage = (device is not None and str(device).startswith("cuda") and
                      dist.get_backend() == "gloo")
        self.cdev = None if self.stage else device  # where the collectives run
        self.cap = 0
        self.pk = self.pk_dev = self.hdr = self.recv = None
        self._grow(0)

    def _grow(self, m):
        import torch
        self.cap = cap = max(1024, m + m // 4)
        words = 1 + cap + (cap + 1) // 2
        self.pk = torch.zeros(words, dtype=torch.int64, device=self.cdev)
        self.pk_dev = (torch.zeros(words, dtype=torch.int64, device=self.device)
                       if self.stage else self.pk)
        self.hdr = torch.zeros(self.world, dtype=torch.int64, device=self.cdev)
        self.recv = ([torch.zeros(words, dtype=torch.int64, device=self.cdev)
                      for _ in range(self.world)] if self.rank == self.root else None)

    def _once(self, pack, wait):
        if pack is not None:  # None: the scan filled pk_dev itself (scan_plan_pack)
            pack(self.pk_dev, self.cap)
        if wait is not None:
            wait()
        if self.stage:
            self.pk.copy_(self.pk_dev)
        self.dist.all_gather_into_tensor(self.hdr, self.pk[0:1])
        self.dist.gather(self.pk, self.recv, dst=self.root)

    def gather(self, pack, wait=None, complete=None):
        """every rank's record count (the records are on the root, merged())"""
        self.start(pack, wait)
        return self.finish(pack, wait, complete)

    def start(self, pack, wait=None):
        """queue the pack and both collectives (nothing is read on the host);
        pack None: the buffer (pk_dev, cap) is already being filled on the
        device stream `wait` orders the collectives after"""
        self._once(pack, wait)

    def finish(self, pack, wait=None, complete=None):
        """after start(): complete(), read the gathered headers, repeat the
        pack and collectives if some rank's records did not fit or were not
        final; every rank's record count"""
        if complete is not None:
            complete()
        hdr = self.hdr.cpu().tolist()
        counts = [h & ~NOT_READY for h in hdr]
        if any(h & NOT_READY for h in hdr) or max(counts) > self.cap:
            if max(counts) > self.cap:
                self._grow(max(counts))
            self._once(pack, wait)
            hdr = self.hdr.cpu().tolist()
            counts = [h & ~NOT_READY for h in hdr]
            if any(h & NOT_READY for h in hdr):
                raise RuntimeError("PackedGather: records still not final after the rescan")
            if max(counts) > self.cap:
                # a count that grew after complete() would make merged()
                # slice past the keys region: fail rather than return junk
                raise RuntimeError("PackedGather: %d records exceed the regrown capacity %d"
                                   % (max(counts), self.cap))
        return counts

    def merged(self, counts):
        """the root's gathered records concatenated in rank order: (keys,
        ids); None on the other ranks"""
        import torch
        if self.rank != self.root:
            return None
        cap = self.cap
        keys = [r[1:1 + c] for r, c in zip(self.recv, counts)]
        ids = [r.view(torch.int32)[2 * (1 + cap):2 * (1 + cap) + c]
               for r, c in zip(self.recv, counts)]
        return torch.cat(keys), torch.cat(ids)


def host_pack(keys, ids, n):
    """pack(buf, cap) for records held in torch tensors (CPU tests): the
    PackedGather layout, header = n"""
    import torch

    def pack(buf, cap):
        m = min(n, cap)
        buf[0] = n
        buf[1:1 + m].copy_(keys[:m])
        buf.view(torch.int32)[2 * (1 + cap):2 * (1 + cap) + m].copy_(ids[:m])
    return pack
