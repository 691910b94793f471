"""Where RCCL's INIT log goes under bench.dist_setup (one rank, nccl): the
file named by NCCL_DEBUG_FILE, its size and its lines, after the group's
creation, after a collective, and after the group is destroyed."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def state(tag):
    f = bench._RCCL_LOG
    d = os.path.dirname(f) if f else None
    files = sorted(glob.glob(os.path.join(d, '*'))) if d else []
    out = {'tag': tag, 'file': f, 'env': {k: os.environ.get(k) for k in
                                          ('NCCL_DEBUG', 'NCCL_DEBUG_SUBSYS', 'NCCL_DEBUG_FILE')},
           'dir_files': {p: os.path.getsize(p) for p in files}}
    if f and os.path.exists(f):
        with open(f, errors='replace') as fh:
            out['head'] = [x.strip()[:200] for x in fh.readlines()[:6]]
    out['summary'] = bench.rccl_init_summary(f)
    print(json.dumps(out), flush=True)


def main():
    os.environ.update(WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(bench._free_port()))
    d, rank, local, world = bench.dist_setup(force=True)
    state('after init_process_group')
    import torch
    t = torch.ones(4, device='cuda')
    d.all_reduce(t)
    torch.cuda.synchronize()
    state('after all_reduce')
    d.destroy_process_group()
    state('after destroy')


if __name__ == '__main__':
    main()
