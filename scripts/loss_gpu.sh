# GPU check of the loss row: parity tests, then the micro-benchmark
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_losses.py -q -rA > gpurun_out/loss_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python scripts/loss_bench.py > gpurun_out/loss_bench.json 2> gpurun_out/loss_bench.err
  echo "bench rc=$?"
fi
