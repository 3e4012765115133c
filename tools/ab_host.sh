# One gpurun call: host-path GPU tests, PCIe probe, host-resident benches (span-copy kernels,
# zero-copy, DMA-staged) and RX
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "host or rx or cipher_state" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/probe_pcie.py 10 || exit $?
for m in host host-kcopy host-staged; do for c in 1 2 3; do
timeout -k 10 300 python bench.py --config $c --mode $m --steps 10 --warmup 3 2>/dev/null | cut -c1-250 || exit $?
done; done
timeout -k 10 300 python bench.py --config 1 --mode rx --steps 10 --warmup 3 2>/dev/null | cut -c1-200 || exit $?
timeout -k 10 300 python bench.py --config 2 --mode rx --steps 10 --warmup 3 2>/dev/null | cut -c1-200 || exit $?
