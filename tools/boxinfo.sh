#!/bin/bash
# Identify the GPU box a measurement ran on (partition modes, clocks): boxes
# differ by up to 25% in HBM store rate, so A/B numbers are only compared
# within one process (tools/ab_step.py) and each result file names its box.
hostname
rocm-smi --showmemorypartition --showcomputepartition 2>&1 | grep -E "Partition:"
rocm-smi --showclocks 2>&1 | grep -iE "mclk|fclk"
rocm-smi --showserial 2>&1 | grep -i serial
