set -o pipefail
O=gpurun_out/ab_order; mkdir -p $O
B="python bench.py --config C5 --steps 100 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 $B > $O/genome_v.json 2> $O/genome_v.err &&
MAGOT_ORF6_ORDER=record timeout -k 10 240 $B --no-verify > $O/record1.json 2>$O/e1 &&
timeout -k 10 240 $B --no-verify > $O/genome1.json 2>$O/e2 &&
MAGOT_ORF6_ORDER=record timeout -k 10 240 $B --no-verify > $O/record2.json 2>$O/e3 &&
timeout -k 10 240 $B --no-verify > $O/genome2.json 2>$O/e4 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pg -o pmc -- python bench.py --config C5 --steps 3 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > $O/pg.log 2>&1 &&
MAGOT_ORF6_ORDER=record timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pr -o pmc -- python bench.py --config C5 --steps 3 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > $O/pr.log 2>&1
echo rc=$?
for f in $O/*.json; do echo $f; python -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['ms_per_step'], d['roofline']['frac'], d.get('verify'))"; done
