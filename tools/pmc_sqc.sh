set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_sqc
for v in base u6; do
ART_LIB=$PWD/variants/libart_$v.so timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ SQC_TC_STALL SQC_DCACHE_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sqc/$v -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 --frames 1 > gpurun_out/pmc_sqc/$v.log 2>&1
done
