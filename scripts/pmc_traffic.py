"""Per-launch HBM traffic of extract_kernel from a gpu_round.sh PMC summary.

Follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE come from separate passes; FETCH_SIZE (KiB, = TCC_EA0_RDREQ x 64 B)
reports half the bytes of 128-B line fills on gfx950, so it is doubled;
WRITE_SIZE is taken as is.   usage: pmc_traffic.py SUMMARY.json OUT.json [config] [kernel]
"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
cfg = sys.argv[3] if len(sys.argv) > 3 else 'C3'
kern = sys.argv[4] if len(sys.argv) > 4 else 'extract_kernel'
pmc = json.load(open(src))
flat = {}
for grp in pmc.values():
    flat.update(grp)
fetch = flat['FETCH_SIZE'] * 1024.0
write = flat['WRITE_SIZE'] * 1024.0
rec = {'config': cfg, 'kernel': kern, 'source': src,
       'fetch_size_bytes_raw': fetch, 'write_size_bytes': write,
       'hbm_read_bytes_per_launch': 2.0 * fetch,
       'hbm_bytes_per_launch': 2.0 * fetch + write,
       'tcc_ea_rdreq': flat.get('TCC_EA0_RDREQ_sum'), 'tcc_ea_wrreq': flat.get('TCC_EA0_WRREQ_sum'),
       'correction': 'FETCH_SIZE x2 (gfx950 128-B fills tallied at 64 B), WRITE_SIZE x1'}
json.dump(rec, open(dst, 'w'), indent=1)
print(json.dumps(rec))
