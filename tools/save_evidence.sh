#!/bin/bash
# Copy an evidence session's records (gpurun_out/round_<tag>) into profiles/ as <prefix>_*.  Usage: save_evidence.sh <tag> <prefix>
set -e
src=gpurun_out/round_$1; p=profiles/$2
cp $src/bench.json ${p}_bench.json
cp $src/trace/run_kernel_stats.csv ${p}_kernel_stats.csv
cp $src/pmc_summary.txt ${p}_pmc_summary.txt
cp $src/pytest_gpu.log ${p}_pytest_gpu.txt
cp $src/smoke.log ${p}_smoke.txt
for f in $src/bench_*.json $src/strong_*.json $src/host_path_*.json; do cp $f ${p}_$(basename $f); done
cp $src/percall.json ${p}_percall.json
[ -f $src/cfg4p_kernel_stats.csv ] && cp $src/cfg4p_kernel_stats.csv ${p}_cfg4p_kernel_stats.csv
[ -f $src/pmc_cfg4p_summary.txt ] && cp $src/pmc_cfg4p_summary.txt ${p}_cfg4p_pmc_summary.txt
[ -f $src/bloom_kernel_stats.csv ] && cp $src/bloom_kernel_stats.csv ${p}_bloom_kernel_stats.csv
[ -f $src/pmc_bloom_summary.txt ] && cp $src/pmc_bloom_summary.txt ${p}_bloom_pmc_summary.txt
ls ${p}_* | wc -l
