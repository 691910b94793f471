"""Multi-GPU job over one shared genome (BASELINE configs[3] "C4").

One process per GPU (torchrun); ``torch.distributed`` with the nccl backend is
RCCL over xGMI on MI355X.  The job:

  1. rank 0 packs the genome once (magot_genome_load) and the packed arena is
     broadcast device-to-device to every rank (``replicate_genome``); the
     other ranks attach to the received bytes (magot_genome_attach);
  2. records are sharded by contig with LPT bin-packing weighted by CDS bases
     (``lpt_contigs``: largest contig first onto the least-loaded rank), so a
     record never spans ranks and there is no exchange during extraction;
  3. each rank extracts its shard (one kernel launch);
  4. outputs are gathered to rank 0 (``gather_bytes``: a size exchange, then
     one padded gather of each output buffer) and put back into global record
     order (``reassemble``).

With the gloo backend (CPU tests) the same steps run with host tensors.
"""

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


def record_shards(tx_contig, tx_bases, n_contigs, n_ranks):
    """(owner rank per contig, record ids per rank in global order, load)."""
    weight = np.bincount(np.asarray(tx_contig), weights=np.asarray(tx_bases, dtype=np.float64),
                         minlength=n_contigs)
    owner, load = lpt_contigs(weight, n_ranks)
    rec_owner = owner[np.asarray(tx_contig)]
    shards = [np.nonzero(rec_owner == r)[0] for r in range(n_ranks)]
    return owner, shards, load


def _device(dist):
    return 'cuda' if dist.get_backend() == 'nccl' else 'cpu'


def replicate_genome(dist, rank, contigs, ctx):
    """The packed genome on every rank: packed once on rank 0, broadcast.

    ``contigs`` is the (name, sequence) list on rank 0 (ignored elsewhere).
    Returns (DeviceGenome, seconds spent in the broadcast)."""
    import time

    import torch

    from . import engine
    if rank == 0:
        dev = engine.DeviceGenome(contigs, ctx=ctx)
        meta, nbytes = dev.export()
        info = [meta, nbytes, dev.names, [int(x) for x in dev.lengths]]
    else:
        dev = None
        info = [None, None, None, None]
    dist.broadcast_object_list(info, src=0)
    meta, nbytes, names, lengths = info
    where = _device(dist)
    buf = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    if rank == 0:
        dev.copy_arena(buf.data_ptr())
    torch.cuda.synchronize()
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
    if rank != 0:
        dev = engine.DeviceGenome.attach(meta, buf.data_ptr(), names, lengths, ctx=ctx,
                                         keepalive=buf)
    return dev, t_bcast


class Gather(object):
    """Variable-size byte buffers from every rank to rank 0, buffers allocated
    once: ``send`` (capacity = the largest rank's size) is filled by the
    caller (e.g. magot_plan_copy_outputs), ``run()`` gathers it on the
    collective backend (device to device with nccl/RCCL), ``parts()`` gives
    rank 0 the per-rank bytes as numpy arrays."""

    def __init__(self, dist, rank, world, nbytes, device='cuda'):
        import torch
        self.dist, self.rank, self.world = dist, rank, world
        where = _device(dist)
        self.staged = where != 'cuda'
        sizes = torch.tensor([int(nbytes)], dtype=torch.int64, device=where)
        all_sizes = [torch.zeros(1, dtype=torch.int64, device=where) for _ in range(world)]
        dist.all_gather(all_sizes, sizes)
        self.sizes = [int(x.item()) for x in all_sizes]
        cap = max(max(self.sizes), 1)
        self.send = torch.zeros(cap, dtype=torch.uint8, device=device)
        self._host = torch.empty(cap, dtype=torch.uint8) if self.staged else None
        buf_dev = 'cpu' if self.staged else device
        self.recv = [torch.empty(cap, dtype=torch.uint8, device=buf_dev)
                     for _ in range(world)] if rank == 0 else None

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


def gather_bytes(dist, rank, world, src_tensor, nbytes):
    """One-off gather of ``nbytes`` of ``src_tensor`` from every rank to rank 0
    (per-rank numpy arrays on rank 0, None elsewhere)."""
    g = Gather(dist, rank, world, nbytes, device=src_tensor.device)
    if nbytes:
        g.send[:nbytes].copy_(src_tensor[:nbytes])
    g.run()
    return g.parts()


def reassemble(shards, parts, offs):
    """Global-order bytes + offsets from per-rank (bytes, offsets) in shard order."""
    n_rec = sum(len(s) for s in shards)
    lens = np.zeros(n_rec, dtype=np.int64)
    for sh, off in zip(shards, offs):
        off = np.asarray(off, dtype=np.int64)
        lens[sh] = off[1:] - off[:-1]
    goff = np.zeros(n_rec + 1, dtype=np.int64)
    np.cumsum(lens, out=goff[1:])
    out = np.empty(int(goff[-1]), dtype=np.uint8)
    for sh, part, off in zip(shards, parts, offs):
        off = np.asarray(off, dtype=np.int64)
        for j, rec in enumerate(sh):
            out[goff[rec]:goff[rec + 1]] = part[off[j]:off[j + 1]]
    return out, goff
