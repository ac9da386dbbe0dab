set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcd
for v in 51 49 -1; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcd/a$v -o run -- python3 tools/gpu/gemm_one.py $v 2560 4096 14336 > gpurun_out/pmcd/a$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcd/b$v -o run -- python3 tools/gpu/gemm_one.py $v 2560 4096 14336 > gpurun_out/pmcd/b$v.log 2>&1 || exit 1
done
for v in 51 49 -1; do
  for p in a b; do
    echo "== variant $v pass $p"
    python3 tools/pmc_summary.py $(ls gpurun_out/pmcd/$p$v/*.db 2>/dev/null | head -1) "$( [ $v = -1 ] && echo Cijk || echo gemm_tn )" || true
  done
done > gpurun_out/pmc_down_summary.txt
rm -rf gpurun_out/pmcd
