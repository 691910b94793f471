"""Can RCCL run two ranks on one GPU?  If it can, the nccl branches of the
multi-GPU path (device-arena broadcast, device gather) can be rehearsed on a
one-GPU box before the driver's 8-GPU run.

    python scripts/rccl_same_device_probe.py          # parent: starts 2 ranks
Prints one JSON line per rank: backend, the collectives run and whether their
results were right, or the error RCCL raised.
"""
import json
import os
import subprocess
import sys
import time


def rank_main():
    import torch
    import torch.distributed as dist
    rank = int(os.environ['RANK'])
    torch.cuda.set_device(0)
    out = {'rank': rank, 'ok': False}
    try:
        dist.init_process_group(backend='nccl')
        out['backend'] = dist.get_backend()
        n = 64 << 20
        buf = torch.full((n,), rank + 1, dtype=torch.uint8, device='cuda')
        dist.broadcast(buf, src=0)
        torch.cuda.synchronize()
        out['broadcast_ok'] = bool((buf == 1).all().item())
        part = torch.full((1 << 20,), 10 + rank, dtype=torch.uint8, device='cuda')
        ws = dist.get_world_size()
        recv = [torch.empty_like(part) for _ in range(ws)] if rank == 0 else None
        dist.gather(part, recv, dst=0)
        torch.cuda.synchronize()
        if rank == 0:
            out['gather_ok'] = all(bool((r == 10 + i).all().item()) for i, r in enumerate(recv))
        t = torch.tensor([float(rank)], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out['allreduce_ok'] = float(t.item()) == ws - 1
        t0 = time.perf_counter()
        dist.broadcast(buf, src=0)
        torch.cuda.synchronize()
        out['broadcast_64MiB_s'] = time.perf_counter() - t0
        dist.barrier()
        dist.destroy_process_group()
        out['ok'] = True
    except Exception as e:  # report, do not hide: the parent prints it
        out['error'] = '%s: %s' % (type(e).__name__, str(e)[:400])
    print(json.dumps(out), flush=True)
    return 0 if out['ok'] else 1


def main():
    if 'RANK' in os.environ:
        return rank_main()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import _free_port
    base = dict(os.environ, WORLD_SIZE='2', LOCAL_WORLD_SIZE='2', MASTER_ADDR='127.0.0.1',
                MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(2)]
    return max(p.wait() for p in procs)


if __name__ == '__main__':
    sys.exit(main())
