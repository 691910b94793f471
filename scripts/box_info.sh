#!/bin/bash
# Dump the box's GPU state (static info, clocks, partition modes, metrics) into
# DIR, for correlating C5's slow state with the hardware.  Never fails.
D=${1:-gpurun_out/box}; mkdir -p $D
timeout -k 5 30 amd-smi static > $D/static.txt 2>&1
timeout -k 5 30 amd-smi metric > $D/metric.txt 2>&1
timeout -k 5 30 amd-smi partition > $D/partition.txt 2>&1
timeout -k 5 30 rocm-smi --showclocks --showmemuse --showpower > $D/rocm_smi.txt 2>&1
hostname > $D/host.txt 2>&1
true
