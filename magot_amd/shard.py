"""Multi-GPU job over one shared genome (BASELINE configs[3] "C4").

One process per GPU (torchrun); ``torch.distributed`` with the nccl backend is
RCCL over xGMI on MI355X.  The job:

  1. rank 0 packs the genome once (magot_genome_load) and its compact
     replica image (2-bit codes, soft-mask runs, exception runs) is broadcast
     device-to-device to every rank (``replicate_genome``); the other ranks
     rebuild the packed arena from it (magot_genome_wire_import);
  2. records are sharded in genome order into equal-weight ranges
     (``record_shards``: contigs stay whole except where a range boundary
     splits one at a transcript boundary), so a record never spans ranks and
     there is no exchange during extraction;
  3. each rank extracts its shard (one kernel launch per step);
  4. outputs go back per rank by D2H into pinned host memory (the host is
     the consumer), or are gathered to rank 0 over the collective backend
     (``Gather``: a size exchange, then one padded gather of each output
     buffer into a rank-major buffer); ``reassemble_device`` restores global
     record order with one segment-copy kernel (magot_copy_segments).

With the gloo backend (CPU tests) the same steps run with host tensors.
"""

import os

import numpy as np


def lpt_contigs(contig_weight, n_ranks):
    """Rank of each contig: longest-processing-time-first bin packing."""
    w = np.asarray(contig_weight, dtype=np.float64)
    owner = np.zeros(len(w), dtype=np.int64)
    load = np.zeros(n_ranks, dtype=np.float64)
    for c in np.argsort(-w, kind='stable'):
        r = int(np.argmin(load))
        owner[c] = r
        load[r] += w[c]
    return owner, load


def record_shards(tx_contig, tx_bases, n_contigs, n_ranks, tx_start=None):
    """Records -> ranks, balanced by CDS bases.

    Contig-by-contig LPT cannot balance a genome whose largest contig holds
    more than 1/k of the CDS bases (C3: 23.3 %, so 86 % imbalance at k=8), and
    every rank holds the whole broadcast genome anyway, so a contig may be
    split at transcript boundaries at no cost.  Records are laid out in genome
    order -- (contig, start), ``tx_start`` = the first exon's start, or the
    record index when None -- and the sequence is cut into ``n_ranks``
    contiguous runs of equal weight: each rank owns one genome range (whole
    contigs plus at most one split contig at each end), which also keeps its
    kernel's genome footprint at ~1/k of the genome.  A record goes to the rank
    whose range holds the midpoint of its weight, so the imbalance is below
    one record's weight over the mean load.

    Returns (shards, load, spans): ``shards[r]`` the record ids of rank r in
    global (GFF) order, ``load[r]`` its CDS bases, ``spans[c]`` the (first,
    last) rank holding contig c's records ((-1, -1) for a contig without
    records)."""
    tx_contig = np.asarray(tx_contig, dtype=np.int64)
    w = np.asarray(tx_bases, dtype=np.float64)
    T = len(tx_contig)
    pos = np.arange(T, dtype=np.int64) if tx_start is None else np.asarray(tx_start, np.int64)
    order = np.lexsort((np.arange(T), pos, tx_contig))
    cw = np.cumsum(w[order])
    total = cw[-1] if T else 0.0
    mid = cw - 0.5 * w[order]
    rank_sorted = np.minimum((mid * n_ranks / max(total, 1e-300)).astype(np.int64), n_ranks - 1) \
        if T else np.zeros(0, np.int64)
    rank_of = np.empty(T, dtype=np.int64)
    rank_of[order] = rank_sorted
    shards = [np.nonzero(rank_of == r)[0] for r in range(n_ranks)]
    load = np.bincount(rank_of, weights=w, minlength=n_ranks).astype(np.float64)
    spans = np.full((n_contigs, 2), -1, dtype=np.int64)
    if T:
        lo = np.full(n_contigs, n_ranks, dtype=np.int64)
        hi = np.full(n_contigs, -1, dtype=np.int64)
        np.minimum.at(lo, tx_contig, rank_of)
        np.maximum.at(hi, tx_contig, rank_of)
        has = hi >= 0
        spans[has, 0] = lo[has]
        spans[has, 1] = hi[has]
    return shards, load, spans


def genome_order(records, tx_contig, tx_start):
    """``records`` (global ids) sorted by (contig, first exon start): the order a
    rank of a shared job extracts its shard in.  Its outputs land in that order
    in the rank's buffer; the gather's reassembly puts every record back at its
    global place (``reassembly_tables`` follows the order given), so the job's
    output is unchanged.  Neighbouring records then share genome lines in the
    caches: C3 in coordinate order reads 0.53 instead of 0.88 GB per launch."""
    records = np.asarray(records, dtype=np.int64)
    tx_contig = np.asarray(tx_contig, dtype=np.int64)
    tx_start = np.asarray(tx_start, dtype=np.int64)
    o = np.lexsort((records, tx_start[records], tx_contig[records]))
    return records[o]


def imbalance(load):
    """max / mean - 1 of per-rank loads."""
    load = np.asarray(load, dtype=np.float64)
    return float(load.max() / max(load.mean(), 1e-300) - 1.0) if len(load) else 0.0


# where the library's outputs (and so a Gather's send buffer) live; the CPU
# tests of the collective sequence set 'cpu'
OUTPUT_DEVICE = 'cuda'


def collective_device(dist):
    """Where collective operands live: the device with nccl (RCCL moves
    device memory over xGMI), host memory with gloo.  MAGOT_COLLECTIVE_TENSORS=cuda
    hands gloo device tensors instead (it stages them itself), so a one-GPU
    rehearsal runs the same device-tensor code the nccl job runs; RCCL itself
    refuses two ranks on one device."""
    if dist.get_backend() == 'nccl' or os.environ.get('MAGOT_COLLECTIVE_TENSORS') == 'cuda':
        return 'cuda'
    return 'cpu'


def replicate_genome(dist, rank, contigs, ctx, root_replica=False):
    """The packed genome on every rank: packed once on rank 0, broadcast.

    What crosses the links is the genome's compact replica image
    (magot_genome_wire_export: the forward strand's 2-bit codes, the
    soft-masked bases as runs, the exception runs -- about 0.27 B per base
    against the packed arena's 1 B); every receiving rank rebuilds the nibble
    plane and its mirror from it on its own device (magot_genome_wire_import)
    and frees the image.  The genome's meta blob (contig table, exception run
    list for the planner) goes with the object broadcast.
    ``contigs`` is the (name, sequence) list on rank 0 (ignored elsewhere).
    ``root_replica``: rank 0 too continues on a replica rebuilt from the
    image (its packed original is closed) -- the one-rank job then exercises
    the receiving side as well.
    Returns (DeviceGenome, record): seconds of the export, the broadcast
    (max over ranks is the caller's) and the rebuild, bytes of the image and
    of the meta blob."""
    import time

    import torch

    from . import engine
    if rank == 0:
        dev = engine.DeviceGenome(contigs, ctx=ctx)
        meta, _ = dev.export()
        info = [meta, dev.wire_size(), dev.names, [int(x) for x in dev.lengths]]
    else:
        dev = None
        info = [None, None, None, None]
    t0 = time.perf_counter()
    dist.broadcast_object_list(info, src=0)  # the other ranks wait here for rank 0's pack
    t_meta = time.perf_counter() - t0
    meta, nbytes, names, lengths = info
    where = collective_device(dist)
    buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    t_export = 0.0
    if rank == 0:
        t0 = time.perf_counter()
        dev.wire_export(buf.data_ptr(), nbytes)
        t_export = time.perf_counter() - t0
    dist.barrier()
    t0 = time.perf_counter()
    if where == 'cuda':
        dist.broadcast(buf, src=0)
    else:
        host = buf.cpu()
        dist.broadcast(host, src=0)
        buf.copy_(host)
    torch.cuda.synchronize()
    t_bcast = time.perf_counter() - t0
    t_import = 0.0
    if rank != 0 or root_replica:
        if dev is not None:
            dev.close()
        t0 = time.perf_counter()
        dev = engine.DeviceGenome.from_wire(meta, buf.data_ptr(), nbytes, names, lengths, ctx=ctx)
        t_import = time.perf_counter() - t0
    del buf
    return dev, {'export_s': t_export, 'broadcast_s': t_bcast, 'rebuild_s': t_import,
                 'image_bytes': int(nbytes), 'meta_bytes': len(meta), 'meta_s': t_meta}


class Gather(object):
    """Variable-size byte buffers from every rank to rank 0, buffers allocated
    once: ``send`` (capacity = the largest rank's size) is filled by the
    caller (e.g. magot_plan_copy_outputs), ``run()`` gathers it on the
    collective backend (device to device with nccl/RCCL) into one rank-major
    receive buffer on rank 0 (rank r's bytes at r * ``cap``): ``parts()`` as
    numpy arrays, ``received()`` the whole buffer on the device (for
    ``reassemble_device``)."""

    def __init__(self, dist, rank, world, nbytes, device=None):
        import torch
        self.dist, self.rank, self.world = dist, rank, world
        device = OUTPUT_DEVICE if device is None else device
        where = collective_device(dist)
        self.staged = where != 'cuda'
        sizes = torch.tensor([int(nbytes)], dtype=torch.int64, device=where)
        all_sizes = [torch.zeros(1, dtype=torch.int64, device=where) for _ in range(world)]
        dist.all_gather(all_sizes, sizes)
        self.sizes = [int(x.item()) for x in all_sizes]
        # 16-byte aligned slots, so aligned records stay aligned in the buffer
        self.cap = cap = (max(max(self.sizes), 1) + 15) & ~15
        self.device = device
        self.send = torch.zeros(cap, dtype=torch.uint8, device=device)
        self._host = torch.empty(cap, dtype=torch.uint8) if self.staged else None
        buf_dev = 'cpu' if self.staged else device
        self.recv_all = torch.empty(world * cap, dtype=torch.uint8, device=buf_dev) \
            if rank == 0 else None
        self.recv = [self.recv_all[r * cap:(r + 1) * cap] for r in range(world)] \
            if rank == 0 else None
        # the zero fill runs on torch's stream; the library fills `send` on its
        # own non-blocking stream, which does not wait for it
        if str(device).startswith('cuda'):
            torch.cuda.synchronize()

    def run(self):
        src = self.send
        if self.staged:
            self._host.copy_(self.send)
            src = self._host
        self.dist.gather(src, gather_list=self.recv, dst=0)

    def parts(self):
        if self.rank != 0:
            return None
        return [self.recv[r][:self.sizes[r]].cpu().numpy() for r in range(self.world)]

    def received(self):
        """Rank 0: the rank-major receive buffer as a device tensor."""
        if self.rank != 0:
            return None
        return self.recv_all if not self.staged else self.recv_all.to(self.device)


def gather_bytes(dist, rank, world, src_tensor, nbytes):
    """One-off gather of ``nbytes`` of ``src_tensor`` from every rank to rank 0
    (per-rank numpy arrays on rank 0, None elsewhere)."""
    g = Gather(dist, rank, world, nbytes, device=src_tensor.device)
    if nbytes:
        g.send[:nbytes].copy_(src_tensor[:nbytes])
    g.run()
    return g.parts()


def gather_offsets(dist, rank, world, off):
    """Every rank's offset table (uint64, its records + 1) to rank 0, over the
    collective backend (one padded gather, no pickling): a list of numpy
    arrays on rank 0, None elsewhere."""
    import torch
    off = np.ascontiguousarray(off, dtype=np.int64)
    where = collective_device(dist)
    n = torch.tensor([len(off)], dtype=torch.int64, device=where)
    ns = [torch.zeros(1, dtype=torch.int64, device=where) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    cap = max(ns)
    send = torch.zeros(cap, dtype=torch.int64, device=where)
    send[:len(off)] = torch.from_numpy(off).to(where)
    recv = [torch.zeros(cap, dtype=torch.int64, device=where) for _ in range(world)] \
        if rank == 0 else None
    dist.gather(send, gather_list=recv, dst=0)
    if rank != 0:
        return None
    return [recv[r][:ns[r]].cpu().numpy() for r in range(world)]


def places(off):
    """(starts, lengths) of the records of an output laid out in record order
    with prefix offsets ``off`` (records + 1 entries)."""
    off = np.asarray(off, dtype=np.int64)
    return off[:-1], off[1:] - off[:-1]


def six_frame_blocks(stream_off, stream_len):
    """(starts, lengths) of every record's block of six 16-byte padded streams
    in a six-frame output (magot_orf6_fetch: a record's six streams are one
    contiguous block, wherever the plan placed it)."""
    soff = np.asarray(stream_off, dtype=np.int64)
    slen = np.asarray(stream_len, dtype=np.int64).reshape(-1, 6)
    return soff[0:-1:6], ((slen + 15) & ~15).sum(axis=1)


def reassembly_tables(shards, offs, cap):
    """Segment tables that put per-rank outputs back into global record order.

    ``shards[r]``: rank r's global record ids in its plan's record order;
    ``offs[r]``: where its records are in its part -- prefix offsets (records
    + 1 entries: record j is bytes [offs[r][j], offs[r][j+1])) or a (starts,
    lengths) pair (``places``, ``six_frame_blocks``); ``cap``: the rank stride
    of the gathered buffer.  Returns (src_off, dst_off, goff) for
    magot_copy_segments, with goff the global offsets (n+1): dst is laid out
    in global record order."""
    n_rec = sum(len(sh) for sh in shards)
    lens = np.zeros(n_rec, dtype=np.int64)
    src_off = np.zeros(n_rec, dtype=np.uint64)
    for r, (sh, off) in enumerate(zip(shards, offs)):
        st, ln = off if isinstance(off, tuple) else places(off)
        st = np.asarray(st, dtype=np.int64)
        sh = np.asarray(sh, dtype=np.int64)
        if len(st) != len(sh) or len(ln) != len(sh):
            raise ValueError('rank %d: %d places for %d records' % (r, len(st), len(sh)))
        lens[sh] = ln
        src_off[sh] = (r * int(cap) + st).astype(np.uint64)
    goff = np.zeros(n_rec + 1, dtype=np.int64)
    np.cumsum(lens, out=goff[1:])
    return src_off, goff.astype(np.uint64), goff


def reassemble_device(shards, offs, gathered, cap, ctx=None):
    """Global-order output on the device from a rank-major gathered buffer
    (``gathered``: a device tensor, rank r's part at r * cap): one
    magot_copy_segments launch.  Returns (device tensor, global offsets)."""
    import torch

    from . import engine
    src_off, dst_off, goff = reassembly_tables(shards, offs, cap)
    out = torch.empty(max(int(goff[-1]), 1), dtype=torch.uint8, device=gathered.device)
    torch.cuda.synchronize()
    engine.copy_segments(gathered.data_ptr(), gathered.numel(), out.data_ptr(), src_off, dst_off,
                         ctx=ctx)
    return out[:int(goff[-1])], goff


def reassemble(shards, parts, offs):
    """Global-order bytes + offsets from per-rank (bytes, offsets) in shard
    order, on the host (the CPU tests' twin of reassemble_device)."""
    cap = max([len(p) for p in parts] + [1])
    src_off, _, goff = reassembly_tables(shards, offs, cap)
    flat = np.zeros(cap * len(parts), dtype=np.uint8)
    for r, p in enumerate(parts):
        flat[r * cap:r * cap + len(p)] = p
    lens = goff[1:] - goff[:-1]
    idx = np.repeat(src_off.astype(np.int64) - goff[:-1], lens) + np.arange(int(goff[-1]))
    return flat[idx], goff
