#!/bin/bash
# PMC of the headline GEMM families at M = 2560 (HEAD plan): MFMA busy, clock,
# issue stalls, LDS traffic; one counter pass each (rocprofv3 limits).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4z}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -f rocpd -d $O/a -o run -- python -u tools/pmc_gemm_head.py 2560 > $O/a.log 2>&1 || { echo "pmc pass a failed"; tail -5 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f rocpd -d $O/b -o run -- python -u tools/pmc_gemm_head.py 2560 > $O/b.log 2>&1 || { echo "pmc pass b failed"; tail -5 $O/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f rocpd -d $O/c -o run -- python -u tools/pmc_gemm_head.py 2560 > $O/c.log 2>&1 || { echo "pmc pass c failed"; tail -5 $O/c.log; exit 1; }
echo done
