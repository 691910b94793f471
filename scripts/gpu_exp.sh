#!/bin/bash
# Timing experiments: record order x debug paths (kernel trace only), then TLB counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp; rm -rf $OUT; mkdir -p $OUT
for order in random sorted; do
  for dbg in 0 1 2; do
    MAGOT_DEBUG_PATHS=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${order}_$dbg -o kt -- python scripts/prof_kernel.py --order $order --iters 10 > $OUT/kt_${order}_$dbg.log 2>&1 || exit 1
    echo "$order dbg=$dbg $(grep extract_kernel $OUT/kt_${order}_$dbg/kt_kernel_stats.csv | cut -d, -f4)"
  done
done
for order in random sorted; do
  timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/tlb_$order -o pmc -- python scripts/prof_kernel.py --order $order --iters 5 > $OUT/tlb_$order.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq_$order -o pmc -- python scripts/prof_kernel.py --order $order --iters 5 > $OUT/sq_$order.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/ins_$order -o pmc -- python scripts/prof_kernel.py --order $order --iters 5 > $OUT/ins_$order.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$order -o pmc -- python scripts/prof_kernel.py --order $order --iters 5 > $OUT/fetch_$order.log 2>&1 || exit 1
done
python scripts/pmc_summary.py $OUT
