set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_gemm_variants.py ${VARS:-49,53,51,54} "4096,28672,4096;4096,4096,14336;4096,6144,4096;4096,4096,4096;2600,4096,4096;2600,28672,4096;2600,4096,14336" > gpurun_out/stg_ab.log 2>&1
