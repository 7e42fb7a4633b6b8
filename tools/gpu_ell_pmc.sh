#!/bin/bash
# PMC passes over tools/ell_lab (256^3): where the DV SpMV's time goes.  One pass per counter group.
set -o pipefail
O=gpurun_out/${1:-ell_pmc}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $O/p1 -o run -f csv -- tools/ell_lab 256 3 > $O/p1.out 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum -d $O/p2 -o run -f csv -- tools/ell_lab 256 3 > $O/p2.out 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INST_LEVEL_VMEM -d $O/p3 -o run -f csv -- tools/ell_lab 256 3 > $O/p3.out 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum -d $O/p4 -o run -f csv -- tools/ell_lab 256 3 > $O/p4.out 2>&1
echo "exit $?" > $O/status
