"""Benchmark: CDS bases extracted (+ translated) per second on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU)

``python bench.py --gpus N`` with N > 1 and no WORLD_SIZE in the environment
starts the N ranks itself (one child process per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set; the parent makes no GPU call, never execs, forwards
rank 0's JSON line and exits non-zero if any rank fails).

Default (``--mode strong``): ONE job of the named configuration over N GPUs
(BASELINE configs[2] C3 at N=1, configs[3] C4 at N>1, and
configs[4] C5's six-frame job at any N).
  * every rank generates the same seeded workload; the genome is packed once
    on rank 0 and its HBM arena broadcast over the collective backend (RCCL
    over xGMI with nccl), timed once as ``genome_broadcast_s``;
  * records are sharded in genome order into equal-weight ranges
    (magot_amd/shard.py: record_shards; contigs split at transcript
    boundaries where a range ends);
  * a step is one launch of the rank's kernel over its resident shard
    (extract_kernel: gather + reverse complement + translate; C5:
    orf6_kernel, gather fused with the six-frame translation); all ranks
    launch concurrently, and the K steps are timed between a barrier +
    device synchronisation on both sides, max over ranks;
  * returning the outputs is its own phase, timed once after the steps:
    per-rank D2H into pinned host memory (the host is the consumer), and for
    N > 1 a gather of every rank's outputs to rank 0 over the collective
    backend, put back into global record order and checked.
At N=1 this is exactly the C3 (or C2 / C5) single-GPU job.
``--mode weak``: each rank runs its own C-shaped job (seed + 1000 * rank).

Rank 0 prints ONE JSON line (contract in DESIGN.md).
"""

import argparse
import faulthandler
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

# a native crash in any thread (HIP runtime, RCCL, c10d's store and watchdog
# threads) prints every thread's Python stack to stderr before the process
# dies (a SIGSEGV during --dist start-up left no record)
faulthandler.enable(all_threads=True)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
CONFIGS = ['C2', 'C3', 'C5', 'small', 'small5']


def log(msg):
    if int(os.environ.get('RANK', '0')) == 0:
        sys.stderr.write('[bench] %s\n' % msg)
        sys.stderr.flush()


def host_threads():
    """Host threads this GPU's share of the box has (16 per GPU on the pool)."""
    return int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)


# ---------------------------------------------------------------------------
# Launching N ranks (no torchrun)
# ---------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, script=None):
    """Start ``n`` ranks of ``script`` (default: this file) with ``argv`` as
    child processes and wait for them.  Called before anything touches the
    GPU (torch.cuda.device_count() does not initialise HIP on this image) and
    never execs.  Rank 0 inherits stdout (it prints the JSON line); the other
    ranks' stdout goes to stderr.  When a rank fails, the others are
    terminated.  Returns the exit status: 0, or the first failing rank's."""
    # MAGOT_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (RCCL refuses
    # ranks sharing a device: profiles/r04r/rccl_probe.json)
    if os.environ.get('MAGOT_DIST_BACKEND') != 'gloo':
        import torch
        ndev = torch.cuda.device_count()
        if n > ndev:
            sys.stderr.write('[bench] --gpus %d but %d device(s) visible (set '
                             'MAGOT_DIST_BACKEND=gloo to rehearse ranks sharing a device)\n'
                             % (n, ndev))
            return 2
    port = _free_port()
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    script = script or os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [c for c in codes if c not in (None, 0)]
            if failed and rc == 0:
                rc = failed[0]
                stop()
            if all(c is not None for c in codes):
                break
            time.sleep(0.05)
        for p in procs:
            p.wait()
    finally:
        signal.signal(signal.SIGTERM, old)
    return rc


def dist_init_kwargs(backend, rank, world, device, env=None):
    """The ``init_process_group`` arguments of this rank, spelled out:
      * ``init_method`` an explicit tcp:// URL on MASTER_ADDR (127.0.0.1 by
        default, never a name to resolve: c10d's lookup of the box's hostname
        fails there, err=-3) and MASTER_PORT, with rank and world size given,
        instead of env:// discovery (under torchrun the agent's store is still
        the one joined: torch's tcp:// handler honours it);
      * ``device_id`` the rank's device under nccl: the process group is bound
        to it and RCCL's communicator is created eagerly, inside this call on
        the main thread, instead of lazily inside the first collective.
    ``device`` is the rank's device index (None without a GPU)."""
    import datetime
    env = os.environ if env is None else env
    kw = {'backend': backend,
          'init_method': 'tcp://%s:%s' % (env.get('MASTER_ADDR') or '127.0.0.1',
                                          env['MASTER_PORT']),
          'rank': rank, 'world_size': world,
          'timeout': datetime.timedelta(seconds=float(env.get('MAGOT_DIST_TIMEOUT_S', '900')))}
    if backend == 'nccl' and device is not None:
        import torch
        kw['device_id'] = torch.device('cuda', device)
    return kw


def rccl_log_env(rank, env=None):
    """NCCL_DEBUG=INFO (subsystem INIT) into one file per rank, so a multi-GPU
    run leaves RCCL's own init record (nranks, rings / channels, "Init
    COMPLETE"); summarised into the JSON line by ``rccl_init_summary``.  Set
    before the communicator exists.  MAGOT_RCCL_LOG=0 turns it off, and a
    caller's own NCCL_DEBUG_FILE wins; a level below INFO is raised to INFO
    (the pool's boxes preset NCCL_DEBUG=VERSION, whose banner then lands in
    the file instead of on rank 0's stdout).  Returns the file (None when off)."""
    env = os.environ if env is None else env
    if env.get('MAGOT_RCCL_LOG', '1') == '0' or 'NCCL_DEBUG_FILE' in env:
        return env.get('NCCL_DEBUG_FILE')
    d = os.path.join(env.get('TMPDIR') or '/tmp', 'magot_rccl_%s' % env.get('MASTER_PORT', '0'))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, 'rank%d.log' % rank)
    if env.get('NCCL_DEBUG', '').upper() in ('', 'VERSION', 'WARN', 'ABORT'):
        env['NCCL_DEBUG'] = 'INFO'
    env.setdefault('NCCL_DEBUG_SUBSYS', 'INIT')
    env['NCCL_DEBUG_FILE'] = path
    return path


_RCCL_KEYS = ('RCCL version', 'Init START', 'Init COMPLETE', 'Init timings', 'Channel 00/',
              'Connected all rings')


def rccl_init_summary(path, max_lines=10):
    """The init lines of one rank's RCCL log (see ``rccl_log_env``)."""
    if not path or not os.path.exists(path):
        return {'file': path, 'lines': []}
    keep = []
    with open(path, errors='replace') as fh:
        for line in fh:
            if any(k in line for k in _RCCL_KEYS):
                keep.append(line.strip()[:240])
                if len(keep) >= max_lines:
                    break
    return {'file': path, 'lines': keep}


_RCCL_LOG = None  # this rank's RCCL log file (nccl backend)


def dist_setup(force=False):
    """The process group of this rank (None for a single rank unless
    ``force``: ``--dist`` runs the multi-rank job's collective path -- the
    genome broadcast, the output gather, the reductions -- through a process
    group of one rank, RCCL with the nccl backend).

    Start-up is ordered so no other thread runs while the HIP runtime comes
    up: the device is selected and its context created on the main thread
    first, then the process group (explicit tcp:// URL, ``device_id`` bound:
    ``dist_init_kwargs``), whose communicator RCCL then creates eagerly."""
    global _RCCL_LOG
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world == 1 and not force:
        return None, rank, local, world
    import torch.distributed as dist
    device = bind_device(local)
    backend = 'gloo' if device is None else 'nccl'    # nccl: RCCL on ROCm
    backend = os.environ.get('MAGOT_DIST_BACKEND', backend)
    if backend == 'nccl':
        _RCCL_LOG = rccl_log_env(rank)
    dist.init_process_group(**dist_init_kwargs(backend, rank, world, device))
    return dist, rank, local, world


def bind_device(local):
    """Select this rank's GPU (one per rank; MAGOT_DIST_BACKEND=gloo rehearses
    N ranks on fewer GPUs) and create its context on the calling thread,
    before any process-group thread exists.  None without a GPU."""
    import torch
    if not torch.cuda.is_available():
        return None
    device = local % torch.cuda.device_count()
    torch.cuda.set_device(device)
    torch.cuda.init()
    torch.empty(1, device='cuda').zero_()
    torch.cuda.synchronize()
    return device


def shard_seed(config, rank):
    """Seed of rank `rank`'s weak-scaling job: SURVEY 8(d) seed for rank 0,
    +1000 per rank (strong mode: every rank uses rank 0's)."""
    from magot_amd import synth
    return synth.SEED_BASE + {'C2': 2, 'C3': 3, 'C5': 5, 'small': 9, 'small5': 9}[config] + \
        1000 * rank


def barrier(dist):
    if dist is not None:
        dist.barrier()


def _reduce(dist, x, op):
    if dist is None:
        return x
    import torch

    from magot_amd.shard import collective_device
    t = torch.tensor([float(x)], dtype=torch.float64, device=collective_device(dist))
    dist.all_reduce(t, op=op)
    return float(t.item())


def allreduce_max(dist, x):
    return _reduce(dist, x, None if dist is None else dist.ReduceOp.MAX)


def allreduce_sum(dist, x):
    return _reduce(dist, x, None if dist is None else dist.ReduceOp.SUM)


def all_values(dist, x):
    """[x of rank 0, x of rank 1, ...] (float64 all_gather on the collective
    device); [x] without a process group."""
    if dist is None:
        return [float(x)]
    import torch

    from magot_amd.shard import collective_device
    dev = collective_device(dist)
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    out = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def settle(fn, sync, ms):
    """Run `fn` back to back until `ms` of wall time have passed (at least 8
    launches), before the W warm-up steps.  After an idle period (the parity
    check keeps the GPU idle for seconds) the first ~30 back-to-back C3 launches
    of a fresh box swing 0.274 -> 0.328 -> 0.279 ms over ~12 ms
    (r02_settle/launch_order.txt in profiles/archive_r01_r04.tar.xz); the timed
    steps measure the steady state after it.  Reported in the JSON line as
    `settle`."""
    n = 0
    t0 = time.perf_counter()
    while True:
        for _ in range(8):
            fn()
        n += 8
        sync()
        el = time.perf_counter() - t0
        if el * 1e3 >= ms:
            return {'launches': n, 'ms': el * 1e3}


# ---------------------------------------------------------------------------
# Box state (C5's fast and slow states): amd-smi counters around
# the timed region and a memory-system probe in this process
# ---------------------------------------------------------------------------

_SMI_FIELDS = [('used_vram_mb', r'USED_VRAM: (\d+) MB'), ('socket_power_w', r'SOCKET_POWER: (\d+) W'),
               ('umc_activity_pct', r'UMC_ACTIVITY: (\d+) %'),
               ('hotspot_c', r'HOTSPOT: (\d+)'), ('mem_temp_c', r'\n\s+MEM: (\d+)'),
               ('mem_clk_mhz', r'MEM_0:\s+CLK: (\d+) MHz'), ('fclk_mhz', r'FCLK_0:\s+CLK: (\d+) MHz'),
               ('energy_j', r'TOTAL_ENERGY_CONSUMPTION: ([\d.]+) J'),
               ('acc_counter', r'ACCUMULATION_COUNTER: (\d+)'),
               ('ppt_acc', r'PPT_ACCUMULATED: (\d+)'),
               ('socket_thermal_acc', r'SOCKET_THERMAL_ACCUMULATED: (\d+)'),
               ('vr_thermal_acc', r'VR_THERMAL_ACCUMULATED: (\d+)'),
               ('hbm_thermal_acc', r'HBM_THERMAL_ACCUMULATED: (\d+)'),
               ('prochot_acc', r'PROCHOT_ACCUMULATED: (\d+)')]


def smi_snapshot(device):
    """A few amd-smi metric fields of `device` (None when amd-smi is not
    there).  A child process, never an exec."""
    import re
    try:
        r = subprocess.run(['amd-smi', 'metric', '-g', str(device)], capture_output=True,
                           text=True, timeout=20)
    except Exception:
        return None
    if r.returncode != 0:
        return None
    out = {'t': time.time()}
    for key, pat in _SMI_FIELDS:
        m = re.search(pat, r.stdout)
        if m:
            out[key] = float(m.group(1))
    return out


def memory_probe(nbytes=4 << 30, iters=5):
    """Streaming store and copy bandwidth of this device now (torch fill_ /
    copy_ of `nbytes`, timed with events on torch's stream): the memory
    system's state in the process that measures the kernel (C5's slow state
    slows a pure store replay as much as the kernel)."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    b = torch.empty(nbytes // 2, dtype=torch.uint8, device='cuda')
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for name, fn, moved in (('store_gbs', lambda: a.fill_(7), nbytes),
                            ('copy_gbs', lambda: b.copy_(a[:nbytes // 2]), nbytes)):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        res[name] = moved * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return res


def box_state(device, before, after, probe_before, probe_after):
    """The run's box record: counter deltas over the timed region, the probes,
    and the used VRAM before the job (another tenant's memory shows here)."""
    st = {'probe_before': probe_before, 'probe_after': probe_after}
    if before and after:
        st['smi_before'] = before
        st['smi_after'] = after
        st['delta'] = {k: after[k] - before[k] for k in
                       ('energy_j', 'acc_counter', 'ppt_acc', 'socket_thermal_acc',
                        'vr_thermal_acc', 'hbm_thermal_acc', 'prochot_acc', 't')
                       if k in before and k in after}
    return st


# ---------------------------------------------------------------------------
# CPU baseline: the reference's per-record loop (CPU oracle restatement of
# genome.py:603-822), single core, on a bounded sample of the same workload.
# ---------------------------------------------------------------------------

def cpu_baseline(w, budget_bases, orfs=False):
    """orfs=False: get_fasta nucleotide + protein per record (C2/C3).
    orfs=True (C5): get_fasta nucleotide, then Sequence.get_orfs on it
    (genome.py:824-851: the six translations, split at stops)."""
    from oracle import magot_oracle as mo
    step = max(1, int(w.cds_bases // max(budget_bases, 1)))
    tx_ids = np.arange(0, w.n_tx, step)
    aset = mo.OracleSet()
    used = sorted(set(w.tx_contig[tx_ids].tolist()))
    seqs = {w.contig_names[c]: w.contig_bytes(c).tobytes().decode('latin-1') for c in used}
    aset.genome = mo.OracleGenome(seqs)
    aset.mRNA = {}
    first = np.concatenate([[0], np.cumsum(w.ex_count)])
    recs = []
    bases = 0
    for t in tx_ids.tolist():
        sid = w.contig_names[w.tx_contig[t]]
        st = '-' if w.tx_strand[t] < 0 else '+'
        kids = []
        for e in range(first[t], first[t + 1]):
            cid = 'cds%d_%d' % (t, e)
            c0 = int(w.ex_start[e]) + 1
            c1 = int(w.ex_start[e] + w.ex_len[e])
            aset.CDS[cid] = mo.OBase(cid, sid, (c0, c1), 'CDS', 'rna%d' % t, st, {}, aset)
            kids.append(cid)
            bases += int(w.ex_len[e])
        rna = mo.OParent('rna%d' % t, sid, 'mRNA', kids, None, st, aset, {})
        aset.mRNA[rna.ID] = rna
        recs.append(rna)
    t0 = time.perf_counter()
    nucs = [mo.get_fasta(r, aset, 'nucleotide') for r in recs]
    t1 = time.perf_counter()
    protein = w.outputs != 'nuc'  # C2 is extraction only (BASELINE configs[1])
    if orfs:
        for text in nucs:
            mo.get_orfs(text.split('\n', 1)[1])
    elif protein:
        for r in recs:
            mo.get_fasta(r, aset, 'protein')
    t2 = time.perf_counter()
    rate = bases / (t2 - t0)
    second = 'get_orfs (six frames)' if orfs else ('protein' if protein else 'no translation')
    cal = None
    cal_path = os.path.join(ROOT, 'profiles', 'cpu_calibration.json')
    if os.path.exists(cal_path) and not orfs and protein:  # calibrated on nucleotide + protein
        with open(cal_path) as fh:
            cj = json.load(fh)
        ratio = cj['port_over_reference_mean']
        lo, hi = cj.get('port_over_reference_min', ratio), cj.get('port_over_reference_max', ratio)
        # the reference's own loop (AnnotationSet.__getitem__ evals, genome.py:536-544)
        # runs this much slower than the port on the same input (scripts/calibrate_cpu.py,
        # the C1 O.biroi subset, the rebuilt C14 and two synthetics)
        cal = {'reference_equivalent_bases_per_s': rate / ratio, 'port_over_reference': ratio,
               'reference_equivalent_range': [rate / hi, rate / lo],
               'port_over_reference_range': [lo, hi],
               'rows': [r['workload'] for r in cj['rows']],
               'source': 'profiles/cpu_calibration.json'}
    return {'value': rate, 'unit': 'bases/s', 'cores': 1, 'kind': 'port', 'calibration': cal,
            'sample': '%d of %d transcripts (every %d-th), %d CDS bases; get_fasta nucleotide '
                      '%.2fs + %s %.2fs; pure-Python restatement of the reference loop '
                      '(oracle/magot_oracle.py)' % (len(recs), w.n_tx, step, bases, t1 - t0,
                                                   second, t2 - t1)}


def cpu_c_port(w, threads):
    """A stronger CPU reference point: the C restatement
    of the same per-record loop (oracle/cds_oracle.c) over the WHOLE
    workload, records split into `threads` contiguous slices run in parallel
    (ctypes releases the GIL).  Only the C calls are timed."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import cds_oracle
    cds_oracle.lib().oracle_extract  # load (and build) before the threads start
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    protein = w.outputs != 'nuc'
    bounds = np.linspace(0, w.n_tx, threads + 1).astype(np.int64)
    jobs = []
    for i in range(threads):
        t0, t1 = int(bounds[i]), int(bounds[i + 1])
        e0, e1 = int(first[t0]), int(first[t1])
        counts = w.ex_count[t0:t1]
        rec_off = np.zeros(t1 - t0 + 1, dtype=np.int64)
        np.cumsum(counts, out=rec_off[1:])
        tx_of = np.repeat(np.arange(t0, t1), counts)
        c0 = w.ex_start[e0:e1] + 1
        c1 = w.ex_start[e0:e1] + w.ex_len[e0:e1]
        sk = np.where(w.tx_strand[tx_of] < 0, ord('-'), ord('+')).astype(np.uint8)
        jobs.append((rec_off, w.tx_contig[tx_of], c0, c1, sk))

    def run(job, prot):
        return cds_oracle.extract(w.genome, w.contig_off, job[0], job[1], job[2], job[3], job[4],
                                  prot)

    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda j: run(j, False), jobs))
        t1 = time.perf_counter()
        if protein:
            list(ex.map(lambda j: run(j, True), jobs))
        t2 = time.perf_counter()
    return {'value': w.cds_bases / (t2 - t0), 'unit': 'bases/s', 'cores': threads,
            'kind': 'port (C)',
            'sample': 'whole workload, %d threads; nucleotide %.3fs%s; oracle/cds_oracle.c'
                      % (threads, t1 - t0, (' + protein %.3fs' % (t2 - t1)) if protein else '')}


# ---------------------------------------------------------------------------
# Parity of the measured configuration (per rank, on its own shard)
# ---------------------------------------------------------------------------

def _pep_matches(pep, poff, pref):
    """Device peptides (untrimmed frame 0) == oracle peptides (trimX applied)."""
    starts = poff[:-1].astype(np.int64)
    lens = (poff[1:] - poff[:-1]).astype(np.int64)
    first = np.zeros(len(starts), dtype=bool)
    first[lens > 0] = pep[starts[lens > 0]] == ord('X')
    keep = np.ones(len(pep), dtype=bool)
    keep[starts[first]] = False
    return np.array_equal(pep[keep], pref)


def verify_extract(w, plan, mine):
    from oracle import cds_oracle
    nuc, noff, pep, poff = plan.run()
    ref, roff, st = cds_oracle.extract_workload(w, False, tx_subset=mine)
    ok = (not st.any()) and np.array_equal(nuc, ref) and \
        np.array_equal(noff.astype(np.int64), roff)
    if ok and pep is not None:
        pref, _, _ = cds_oracle.extract_workload(w, True, tx_subset=mine)
        ok = _pep_matches(pep, poff, pref)
    return ok


def verify_orf6(w, plan, o6, mine):
    """Nucleotides in full, and ALL six frames of ALL records against the C
    oracle's translate(frame, strand) (genome.py:795-851), multi-threaded."""
    from oracle import cds_oracle
    plan.execute()
    o6.execute()
    nuc, noff, _, _ = plan.fetch()
    ref, roff, st = cds_oracle.extract_workload(w, False, tx_subset=mine)
    ok = (not st.any()) and np.array_equal(nuc, ref) and \
        np.array_equal(noff.astype(np.int64), roff)
    del nuc
    out, soff, slen = o6.fetch()
    bad, first = cds_oracle.orf6_compare(ref, roff, out, soff, slen, threads=host_threads())
    if bad:
        log('six-frame mismatch: %d streams, first %d' % (bad, first))
    return ok and bad == 0


# ---------------------------------------------------------------------------
# The job
# ---------------------------------------------------------------------------

_DESC = {
    'C3': '1 Gb genome (64 lognormal contigs) + 500k transcripts x (1+Poisson(7)) exons of '
          'U[50,250] b, both strands; nucleotide + peptide out',
    'C2': '100 Mb genome (16 contigs), 50k single-exon + CDS U[150,1850]; nucleotide out',
    'C5': '3 Gb genome (200 lognormal contigs), 2M transcripts; CDS gather + six-frame '
          'translation (get_orfs)',
    'small': '1 Mb genome (8 contigs), 500 transcripts (test size); nucleotide + peptide out',
    'small5': '1 Mb genome (8 contigs), 500 transcripts (test size); six-frame translation '
              '(the C5 job at test size)',
}


def _rocprof_quote(config, kernel):
    """The committed rocprofv3 kernel-trace average for this configuration's
    kernel (profiles/rocprof_summary.json, written from the --stats CSVs by
    scripts/rocprof_summary.py), quoted beside the live HIP-event time."""
    path = os.path.join(ROOT, 'profiles', 'rocprof_summary.json')
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh).get(config)
    if not d or d.get('kernel') != kernel:
        return None
    return d


def run_job(args, dist, rank, local, world):
    import torch

    from magot_amd import _lib, engine, shard, synth
    strong = args.mode == 'strong'
    # one job over the process group (any world size, --dist at N=1): the
    # genome is broadcast from rank 0 and the outputs gathered back to it
    multi = strong and dist is not None
    c5 = args.config in ('C5', 'small5')
    t_start = t0 = time.perf_counter()
    # the other ranks of a shared job make only the record tables (their
    # stand-in for reading the GFF): the genome reaches them over the
    # collective, and rank 0 checks the whole gathered job
    w = synth.make('small' if args.config == 'small5' else args.config,
                   seed=shard_seed(args.config, 0 if strong else rank), order=args.order,
                   genome=not multi or rank == 0)
    t_gen = time.perf_counter() - t0
    log('generated %s: %d contigs, %d transcripts, %d exons, %d CDS bases (%.1fs)'
        % (args.config, len(w.contig_len), w.n_tx, w.n_exons, w.cds_bases, t_gen))
    ctx = _lib.Context(local)

    mine, imb, t_bcast, t_pack, bcast_bytes, replica = None, 0.0, None, None, None, None
    t_wait = 0.0  # waiting for rank 0's pack in the object broadcast
    shards = None
    rehearse = None
    if args.rehearse_shard and world == 1:
        # diagnostic: this single GPU runs rank r's shard of a K-rank C4 job
        # (what each GPU of the 8-GPU node gets), genome packed locally
        k, r = (int(x) for x in args.rehearse_shard.split(':'))
        first = np.zeros(w.n_tx + 1, dtype=np.int64)
        np.cumsum(w.ex_count, out=first[1:])
        tx_bases = np.add.reduceat(w.ex_len, first[:-1])
        sh, load, _ = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), k,
                                          tx_start=w.ex_start[first[:-1]])
        mine = shard.genome_order(sh[r], w.tx_contig, w.ex_start[first[:-1]])
        rehearse = {'ranks': k, 'rank': r, 'load_imbalance': shard.imbalance(load)}
    if multi:
        first = np.zeros(w.n_tx + 1, dtype=np.int64)
        np.cumsum(w.ex_count, out=first[1:])
        tx_bases = np.add.reduceat(w.ex_len, first[:-1]) if w.n_tx else np.zeros(0)
        shards, load, spans = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len),
                                                  world, tx_start=w.ex_start[first[:-1]])
        # every rank extracts its shard in genome order: its outputs are gathered
        # and put back into global record order anyway (reassembly), so the order
        # inside a rank's buffer is free, and neighbouring records then share
        # genome lines (C4 shares 7.5-9 % faster, profiles/r05/shard_order/)
        shards = [shard.genome_order(sh, w.tx_contig, w.ex_start[first[:-1]]) for sh in shards]
        mine = shards[rank]
        imb = shard.imbalance(load)
        log('%d records over %d ranks: load imbalance %.4f%%, %d contig(s) split'
            % (w.n_tx, world, 100.0 * imb, int((spans[:, 0] != spans[:, 1]).sum())))
        # at N=1 rank 0 extracts from the replica it rebuilds from its own
        # wire image, so the receiving side runs too
        dev, rep = shard.replicate_genome(
            dist, rank, w.contig_views() if rank == 0 else None, ctx,
            root_replica=world == 1)
        t_wait = rep['meta_s']
        t_bcast = allreduce_max(dist, rep['broadcast_s'])
        bcast_bytes = rep['image_bytes'] + rep['meta_bytes']
        replica = {'image_bytes': rep['image_bytes'], 'meta_bytes': rep['meta_bytes'],
                   'export_s': rep['export_s'],
                   'rebuild_s_max_rank': allreduce_max(dist, rep['rebuild_s']),
                   'image': '2-bit forward codes + soft-mask runs + exception runs '
                            '(magot_genome_wire_export); meta blob by object broadcast'}
    else:
        t0 = time.perf_counter()
        dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
        t_pack = time.perf_counter() - t0

    ex, tx = w.plan_tables(tx_subset=mine)
    if c5:
        outputs = engine.OUT_NUC
    else:
        outputs = engine.OUT_NUC | (engine.OUT_PEP if w.outputs == 'nuc+pep' else 0)
        if args.plan_layout == 'genome' and not multi:
            # records laid out in genome order in HBM (MAGOT_OUT_GENOME_ORDER):
            # neighbouring loci run in neighbouring tiles and share genome lines
            # (C3 kernel -4.7 %, C2 -3.0 %, profiles/r05/plan_order/); fetch,
            # copy_outputs and the FASTA text assembly still deliver record order;
            # a shared job's shards are already listed in genome order
            outputs |= engine.OUT_GENOME_ORDER
    t0 = time.perf_counter()
    plan = engine.ExtractionPlan(dev, ex, tx, outputs)
    o6 = engine.Orf6Plan(plan) if c5 else None
    t_plan = time.perf_counter() - t0
    B = plan.nuc_bytes
    P = plan.pep_bytes if outputs & engine.OUT_PEP else 0
    if c5:
        _, slen = o6.fetch_to(None)
        R = int(slen.sum())
        # algorithmic bytes: 2-bit genome reads + six translations + descriptors
        alg = -(-B // 4) + R + 16 * int(plan.n_exons) + 32 * int(plan.n_tx)
        kernel_name = 'orf6_kernel'
        step = o6.execute
    else:
        R = None
        alg = plan.algorithmic_bytes
        kernel_name = 'extract_kernel'
        step = plan.execute

    t_setup = time.perf_counter() - t_start
    # -- correctness of the measured configuration (each rank, its own shard) -----
    parity = 'not checked'
    launches_before = 0  # launches of the measured kernel before the timed steps
    if multi and not args.no_verify:
        parity = 'checked on the gathered job (outputs_gather.parity)'
    elif not args.no_verify:
        launches_before += 1
        t0 = time.perf_counter()
        ok = verify_orf6(w, plan, o6, mine) if c5 else verify_extract(w, plan, mine)
        log('rank-local parity %s (%.1fs)' % ('ok' if ok else 'MISMATCH', time.perf_counter() - t0))
        n_bad = allreduce_sum(dist, 0.0 if ok else 1.0)
        what = ('nucleotides and all six frames of every record' if c5 else 'full output')
        parity = ('bit-exact vs CPU oracle (%s%s)' % (what, ', every rank\'s shard' if world > 1
                                                      else '')) if n_bad == 0 \
            else 'MISMATCH on %d rank(s)' % int(n_bad)

    # -- timed region ---------------------------------------------------------
    record_box = rank == 0 and not args.no_box_state
    if record_box:
        smi0 = smi_snapshot(local)
        probe0 = memory_probe()
    settled = settle(step, ctx.sync, args.settle_ms)
    launches_before += settled['launches'] + args.warmup
    for _ in range(args.warmup):
        step()
    ctx.sync()
    barrier(dist)
    ctx.sync()
    t0 = time.perf_counter()
    ctx.mark(0)
    for _ in range(args.steps):
        step()
    ctx.mark(1)
    ctx.sync()
    elapsed = time.perf_counter() - t0
    barrier(dist)
    elapsed_max = allreduce_max(dist, elapsed)

    # per-launch kernel duration from HIP events on the context stream (the
    # kernel's own stream) around exactly the K timed launches; back-to-back
    # and isolated launches after the timed region are reported beside it
    timer = o6 if c5 else plan
    kernel_ms = ctx.elapsed_ms() / args.steps
    n_b2b = max(20, min(args.steps, 100))
    kernel_b2b = timer.time_b2b(n_b2b)
    kernel_iso = timer.time(10)
    kernel_rec = None
    delivery = None
    if outputs & engine.OUT_GENOME_ORDER and not args.no_layout_compare:
        # beside it, for transparency: the same job in record order (the
        # layout the reference's output has), given the same settle and
        # warm-up as the line's own plan, then timed back to back
        rp = engine.ExtractionPlan(dev, ex, tx, outputs & ~engine.OUT_GENOME_ORDER)
        settle(rp.execute, ctx.sync, args.settle_ms)
        for _ in range(args.warmup):
            rp.execute()
        ctx.sync()
        kernel_rec = rp.time_b2b(n_b2b)
        delivery = record_order_delivery(plan, rp, ctx, B, P)
        rp.close()
    kernel_ms_max = allreduce_max(dist, kernel_ms)
    # per-rank figures of a shared job (where a scaling loss sits: the slowest
    # rank's kernel, or the host's time around it)
    kernel_ms_ranks = all_values(dist, kernel_ms) if dist is not None else None
    elapsed_ranks = all_values(dist, elapsed) if dist is not None else None
    boxrec = None
    if record_box:
        boxrec = box_state(local, smi0, smi_snapshot(local), probe0, memory_probe())
    total_bases = allreduce_sum(dist, float(B))
    alg_mean = allreduce_sum(dist, float(alg)) / world
    value = total_bases * args.steps / elapsed_max
    achieved = alg_mean / (kernel_ms_max * 1e-3) / 1e9

    # -- returning the outputs (its own phase, once) -----------------------------
    phases = {'generate': t_gen, 'pack_h2d': t_pack, 'plan_h2d': t_plan}
    out_bytes = R if c5 else B + P
    pin = torch.empty(max(int(o6.total if c5 else B + P), 1), dtype=torch.uint8,
                      pin_memory=True)
    ctx.sync()
    barrier(dist)
    t0 = time.perf_counter()
    if c5:
        o6.fetch_to(pin.data_ptr())
    else:
        plan.fetch_to(pin.data_ptr() if B else None,
                      pin.data_ptr() + B if P else None)
    t_d2h = allreduce_max(dist, time.perf_counter() - t0)
    barrier(dist)
    phases['outputs_d2h_pinned'] = t_d2h
    del pin
    gather = None
    if multi:
        gather = gather_outputs(args, dist, rank, world, w, plan, o6, shards, ctx)
        if rank == 0 and not args.no_verify:
            parity = gather['parity']
    import resource
    rss_gb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2.0 ** 20  # KiB -> GiB
    rss_all = all_values(dist, rss_gb)
    setup_all = all_values(dist, t_setup - t_wait)
    wait_all = all_values(dist, t_wait)
    rccl_init = None
    if dist is not None and dist.get_backend() == 'nccl':
        # every rank's RCCL init record (NCCL_DEBUG=INFO, subsystem INIT) into the line
        rccl_init = [None] * world
        dist.all_gather_object(rccl_init, rccl_init_summary(_RCCL_LOG))
    host = {'peak_rss_gib_max_rank': max(rss_all),
            'peak_rss_gib_rank0': rss_gb,
            'peak_rss_gib_per_rank': rss_all,
            'setup_s_max_rank': max(setup_all),
            'setup_s_per_rank': setup_all,
            'setup_wait_s_per_rank': wait_all,
            'setup': 'own set-up work: workload generation (ranks > 0 of a shared job: record '
                     'tables only) + genome pack, or the image broadcast and rebuild + plan '
                     'upload, before the parity check; setup_wait_s: time the rank waited in '
                     'the object broadcast for rank 0 to generate and pack the genome'}

    # -- roofline / traffic / baselines --------------------------------------------
    traffic = None
    if world == 1 and os.path.exists(args.pmc_json):
        with open(args.pmc_json) as fh:
            pmc = json.load(fh)
        if pmc.get('config') == args.config and pmc.get('kernel') == kernel_name:
            traffic = pmc.get('hbm_bytes_per_launch')
    rp = _rocprof_quote(args.config, kernel_name) if world == 1 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log('timing the CPU baseline on a bounded sample ...')
        if c5:
            cpu = cpu_baseline(w, args.cpu_sample_bases / 10, orfs=True)
        else:
            cpu = cpu_baseline(w, args.cpu_sample_bases)
            cpu['c_port_all_cores'] = cpu_c_port(w, host_threads())

    if rank == 0:
        if multi and world == 1:
            label = '%s through the multi-GPU path at N=1 (%s process group of one rank)' \
                % (args.config, dist.get_backend())
        elif multi:
            label = 'C4: one %s job over %d GPUs' % (args.config, world) if args.config == 'C3' \
                else '%s: one job over %d GPUs' % (args.config, world)
        elif strong:
            label = args.config
        else:
            label = '%s per rank' % args.config
        rec = {
            'metric': 'CDS bases extracted+translated/sec',
            'value': value,
            'unit': 'bases/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed_max / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'strong' if strong else 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic (seeded, SURVEY.md 8(d))',
            'config': {'workload': '%s: %s' % (label, _DESC[args.config]),
                       'cds_bases': int(total_bases), 'cds_bases_rank0': B,
                       'residues_rank0': R if c5 else P,
                       'exons_rank0': int(plan.n_exons), 'transcripts_rank0': int(plan.n_tx),
                       'parallelism': 'contig-sharded x%d (%s)' % (world,
                                                                  'strong' if strong else 'weak'),
                       'plan_layout': None if c5 else (
                           'record (shard tables listed in genome order)' if multi
                           else args.plan_layout),
                       'shard_record_order': ('genome: each rank extracts its shard in '
                                              'coordinate order; the gather\'s reassembly '
                                              'restores global record order') if multi
                       else None,
                       'backend': dist.get_backend() if dist is not None else None},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': kernel_name, 'kernel_ms': kernel_ms_max,
                         'kernel_ms_per_rank': kernel_ms_ranks,
                         'step_ms_per_rank': [e / args.steps * 1e3 for e in elapsed_ranks]
                         if elapsed_ranks else None,
                         'kernel_ms_source': 'HIP events on the kernel\'s stream around the K '
                                             'timed launches, / K (max over ranks)',
                         'kernel_ms_b2b': kernel_b2b,
                         'kernel_ms_b2b_source': 'HIP events around %d back-to-back launches '
                                                 'after the timed region' % n_b2b,
                         'kernel_ms_isolated': kernel_iso,
                         'kernel_ms_b2b_record_layout': kernel_rec,
                         'record_order_delivery': delivery,
                         'timed_launches': {'kernel': kernel_name, 'first': launches_before,
                                            'count': args.steps,
                                            'note': 'dispatch indices of this kernel in the '
                                                    'process (0-based): the K timed launches '
                                                    '(scripts/rocprof_summary.py --timed)'},
                         'rocprof_kernel_ms': rp['avg_ms'] if rp else None,
                         'rocprof_frac': (alg_mean / (rp['avg_ms'] * 1e-3) / 1e9 / HBM_PEAK_GBS)
                         if rp else None,
                         'rocprof_source': rp['source'] if rp else None,
                         'per': 'GPU (algorithmic bytes per launch, mean over ranks)',
                         'algorithmic_bytes_per_launch': alg_mean},
            'cpu_baseline': cpu,
            'settle': settled, 'device': ctx.info(),
            'parity': parity,
            'phases_s': phases,
            'host': host,
            'box_state': boxrec,
            'outputs_d2h_bases_per_s': total_bases / t_d2h if t_d2h else None,
            'output_bytes_rank0': out_bytes,
        }
        if rehearse:
            rec['rehearsal'] = rehearse
            rec['config']['workload'] = 'REHEARSAL (not a bench line): rank %d of a %d-rank ' \
                '%s job on one GPU' % (rehearse['rank'], rehearse['ranks'], args.config)
        if multi:
            rec['genome_broadcast_s'] = t_bcast
            rec['genome_broadcast_bytes'] = bcast_bytes
            rec['genome_replica'] = replica
            rec['genome_arena_bytes'] = int(dev.device_bytes)
            rec['load_imbalance'] = imb
            rec['outputs_gather'] = gather
        if rccl_init is not None:
            rec['rccl_init'] = rccl_init
        print(json.dumps(rec), flush=True)
    if o6 is not None:
        o6.close()
    plan.close()
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def record_order_delivery(plan, rec_plan, ctx, B, P, iters=5):
    """What a genome-ordered line costs a caller who wants the buffers in
    record order on the device: ``plan.copy_outputs`` (magot_plan_copy_outputs,
    one segment copy per record) against the same call on the record-order
    plan ``rec_plan`` (a plain device-to-device copy), both timed with HIP
    events on the library's stream.  The FASTA text assembly (gff2fasta)
    reads the genome-ordered buffers in place and pays neither."""
    import torch
    nuc = torch.empty(max(B, 1), dtype=torch.uint8, device='cuda')
    pep = torch.empty(max(P, 1), dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    na, pa = nuc.data_ptr(), (pep.data_ptr() if P else None)

    def timed(p):
        p.copy_outputs(na, pa)
        ctx.mark(0)
        for _ in range(iters):
            p.copy_outputs(na, pa)
        ctx.mark(1)
        ctx.sync()
        return ctx.elapsed_ms() / iters

    reassemble = timed(plan)
    plain = timed(rec_plan)
    del nuc, pep
    torch.cuda.empty_cache()
    return {'reassemble_ms': reassemble, 'plain_d2d_copy_ms': plain,
            'extra_ms': reassemble - plain,
            'note': 'record-order device buffers: magot_plan_copy_outputs on the genome-ordered '
                    'plan (segment copies) vs on the record-order plan (plain D2D copy); once '
                    'per job, outside the step; gff2fasta\'s device text assembly reads the '
                    'genome-ordered buffers in place'}


def gather_outputs(args, dist, rank, world, w, plan, o6, shards, ctx):
    """Every rank's outputs to rank 0 over the collective backend (device to
    device with RCCL), once, timed; rank 0 puts them back into global record
    order on the device (one magot_copy_segments launch, timed) and, unless
    --no-verify, checks the whole job against the oracle.  C3: nucleotides
    and peptides, per-record segments; C5: the six-frame streams, one segment
    per record (a record's six padded streams are contiguous, in the same
    layout as the single-GPU job: magot_orf6_sizes over the global order)."""
    import torch

    from magot_amd import engine, shard
    items = []  # (name, bytes, copy to device address, record (starts, lengths))
    if o6 is not None:
        soff, slen = o6.fetch_to(None)
        items.append(('six-frame residues', o6.total, o6.copy_outputs,
                      shard.six_frame_blocks(soff, slen)))
    else:
        noff, poff = plan.fetch_to(None, None)  # the offset tables only
        items.append(('nucleotides', plan.nuc_bytes,
                      lambda a: plan.copy_outputs(a, None), shard.places(noff)))
        if plan.outputs & engine.OUT_PEP:
            items.append(('peptides', plan.pep_bytes,
                          lambda a: plan.copy_outputs(None, a), shard.places(poff)))
    gathers = [shard.Gather(dist, rank, world, nb) for _, nb, _, _ in items]
    for g, (_, nb, copy, _) in zip(gathers, items):
        if nb:
            copy(g.send.data_ptr())
    torch.cuda.synchronize()
    barrier(dist)
    t0 = time.perf_counter()
    for g in gathers:
        g.run()
    torch.cuda.synchronize()
    t_gather = allreduce_max(dist, time.perf_counter() - t0)
    offs = []
    for _, _, _, (st, ln) in items:
        g_st = shard.gather_offsets(dist, rank, world, st)
        g_ln = shard.gather_offsets(dist, rank, world, ln)
        offs.append(list(zip(g_st, g_ln)) if rank == 0 else None)
    res = {'seconds': t_gather, 'bytes': int(allreduce_sum(dist, float(sum(it[1] for it in items)))),
           'backend': dist.get_backend(), 'collective_tensors': shard.collective_device(dist),
           'outputs': [it[0] for it in items]}
    if rank != 0:
        return res
    t0 = time.perf_counter()
    glob = []
    for g, off in zip(gathers, offs):
        glob.append(shard.reassemble_device(shards, off, g.received(), g.cap, ctx=ctx))
    torch.cuda.synchronize()
    res['reassembly_s'] = time.perf_counter() - t0
    res['reassembly'] = 'magot_copy_segments on rank 0\'s device: %d records into global order' \
        % w.n_tx
    check = 'not checked'
    if not args.no_verify:
        from oracle import cds_oracle
        ref, roff, st = cds_oracle.extract_workload(w, False)
        ok = not st.any()
        if o6 is not None:
            out, goff = glob[0]
            soff, slen = engine.orf6_sizes(roff)  # the single-GPU record-order layout
            ok = ok and np.array_equal(goff, soff[0::6].astype(np.int64))
            if ok:
                bad, first = cds_oracle.orf6_compare(ref, roff, out.cpu().numpy(), soff, slen,
                                                     threads=host_threads())
                ok = bad == 0
        else:
            nuc, goff = glob[0]
            ok = ok and np.array_equal(nuc.cpu().numpy(), ref) and np.array_equal(goff, roff)
            if ok and len(glob) > 1:
                pep, pgoff = glob[1]
                pref, _, _ = cds_oracle.extract_workload(w, True)
                ok = _pep_matches(pep.cpu().numpy(), pgoff, pref)
        check = ('bit-exact vs CPU oracle (gathered, global record order%s)'
                 % (', all six frames of every record' if o6 is not None else '')) if ok \
            else 'MISMATCH'
    res['parity'] = check
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # C3 kernel durations drift by up to 15 % over the first few dozen launches
    # on a fresh box (r01_v13/kt_launch_order.txt, profiles/archive_r01_r04.tar.xz);
    # 20 untimed warm-up steps and 100 timed ones (about 30 ms of C3 work) measure
    # the steady state.
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--settle-ms', type=float, default=100.0,
                    help='back-to-back launches before the warm-up steps (power-state settle)')
    ap.add_argument('--config', default='C3', choices=CONFIGS)
    ap.add_argument('--order', default='random', choices=['random', 'sorted'],
                    help='record order of the synthetic GFF: random within each contig '
                         '(default, SURVEY 8(d)) or coordinate-sorted (diagnostic)')
    ap.add_argument('--plan-layout', default='genome', choices=['genome', 'record'],
                    help='extraction plans: records laid out in HBM in genome order (default; '
                         'delivery returns record order) or in record order')
    ap.add_argument('--no-layout-compare', action='store_true',
                    help='skip the record-layout timing beside a genome-order line (PMC passes: '
                         'only the line\'s own plan launches the kernel)')
    ap.add_argument('--no-verify', action='store_true', help='skip the oracle byte check')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-box-state', action='store_true',
                    help='skip the amd-smi snapshots and memory probes around the timed region')
    ap.add_argument('--cpu-sample-bases', type=float, default=1.0e8)
    ap.add_argument('--pmc-json', default=None,
                    help='per-launch HBM traffic measured with rocprofv3 --pmc '
                         '(default profiles/pmc_<config>.json)')
    ap.add_argument('--mode', default='strong', choices=['strong', 'weak'],
                    help='strong (default): one job over N GPUs, genome broadcast, records '
                         'sharded (C3 at N=1, C4 at N>1); weak: one job per rank')
    ap.add_argument('--dist', action='store_true',
                    help='create the process group even for one rank (nccl = RCCL on a GPU): '
                         'the N=1 job takes the multi-GPU path (genome broadcast from the '
                         'wire image, output gather, reassembly, collective reductions)')
    ap.add_argument('--rehearse-shard', default=None, metavar='K:r',
                    help='diagnostic, one GPU: run only rank r\'s shard of a K-rank strong job '
                         '(the per-GPU work of the K-GPU line; not a bench line)')
    raw = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(raw)
    if args.rehearse_shard and args.gpus > 1:
        ap.error('--rehearse-shard runs one rank')
    if args.rehearse_shard and args.dist:
        ap.error('--rehearse-shard runs without a process group')
    if args.pmc_json is None:
        args.pmc_json = os.path.join(ROOT, 'profiles', 'pmc_%s.json' % args.config)

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, raw)
    if args.dist and 'WORLD_SIZE' not in os.environ:
        os.environ.update(WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                          MASTER_PORT=str(_free_port()))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        log('--gpus %d but WORLD_SIZE=%d: running %d rank(s)' % (args.gpus, world, world))
    dist, rank, local, world = dist_setup(force=args.dist)
    if os.environ.get('MAGOT_DIST_BACKEND') == 'gloo':
        import torch
        local = local % max(torch.cuda.device_count(), 1)
    os.environ.setdefault('MAGOT_DEVICE', str(local))
    run_job(args, dist, rank, local, world)
    return 0


if __name__ == '__main__':
    sys.exit(main())
