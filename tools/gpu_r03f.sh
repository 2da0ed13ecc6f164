set -o pipefail
mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1 || { tail -40 gpurun_out/r03f/pytest.log; exit 1; }
tail -2 gpurun_out/r03f/pytest.log
L=dp-tokenization_amd/csrc/build
for wl in cfg2 cfg4 cfg5; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $L/var_prep0/libdpt.so || exit 1
done
bash tools/ab_libs_wl.sh bloom dp-tokenization_amd/dptok/libdpt.so || exit 1
