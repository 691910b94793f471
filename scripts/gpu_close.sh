#!/bin/bash
# A round's closing check on HEAD: every GPU test (slow included), smoke(),
# the C3 line (defaults and the driver's 20/5), C5 and C2 lines, the two-rank
# C4 rehearsal launched by bench itself, one GPU's share of the 2/4/8-GPU job,
# and kernel traces of the C3 / C5 / C2 lines.   usage: scripts/gpu_close.sh TAG
cd "$(dirname "$0")/.."
TAG=${1:-close}
bash scripts/gpu_round.sh $TAG tests slow smoke bench driver c5 c2 multi multi5 rehearse kt kt5 kt2 traffic e2e || exit 1
python scripts/rocprof_summary.py --timed C3=gpurun_out/$TAG/kt/kt_kernel_trace.csv,gpurun_out/$TAG/kt.json \
    C5=gpurun_out/$TAG/kt_C5/kt_kernel_trace.csv,gpurun_out/$TAG/kt_C5.json \
    C2=gpurun_out/$TAG/kt_C2/kt_kernel_trace.csv,gpurun_out/$TAG/kt_C2.json > gpurun_out/$TAG/rocprof_summary.txt
for f in bench bench_driver_cfg_20_5 bench_c5 bench_c2; do
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/$f.json'));r=d['roofline'];print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['kernel_ms'],4), round(r['frac'],4), d['parity'][:24])"
done
